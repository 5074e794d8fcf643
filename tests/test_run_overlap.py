"""Host plumbing of the helper-context overlap (CPU): engine.ctx() is per thread and restored after
`using_context`; `_beside` keeps the work on the calling thread when DQ_RUN_SERIAL is set, on a multi-device
context, or when the caller already runs on a helper context (nothing nests); `_Pending` hands back the helper's
result and re-raises its exception."""
import threading

import pytest

from deequ_amd import engine, runners


def test_using_context_is_per_thread_and_restored():
    sentinel, other = object(), object()
    seen = {}
    with engine.using_context(sentinel):
        assert engine.ctx() is sentinel

        def worker():
            seen["ctx"] = getattr(engine._local, "ctx", None)
            with engine.using_context(other):
                seen["inner"] = engine.ctx()
        th = threading.Thread(target=worker)
        th.start()
        th.join()
        assert engine.ctx() is sentinel
    assert getattr(engine._local, "ctx", None) is None
    assert seen == {"ctx": None, "inner": other}


def test_beside_stays_serial_when_asked(monkeypatch):
    monkeypatch.setenv("DQ_RUN_SERIAL", "1")
    assert runners._beside(lambda: 1, "x") is None
    monkeypatch.delenv("DQ_RUN_SERIAL")
    monkeypatch.setenv("DQ_DEVICES", "0,0")
    assert runners._beside(lambda: 1, "x") is None
    monkeypatch.delenv("DQ_DEVICES")
    with engine.using_context(object()):  # already on a helper context: no nesting
        assert runners._beside(lambda: 1, "x") is None


def test_pending_returns_and_reraises():
    assert runners._Pending(lambda: 41 + 1).result() == 42

    def boom():
        raise ValueError("helper failed")
    with pytest.raises(ValueError, match="helper failed"):
        runners._Pending(boom).result()

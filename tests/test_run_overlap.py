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


def _helper_threads():
    return [t for t in threading.enumerate() if t.name.startswith("dq-helper")]


def test_helpers_are_joined_when_the_caller_raises(monkeypatch):
    """an exception on the calling thread (or in one helper) never leaves another helper running: the
    run's helper group joins every helper before the exception propagates."""
    import time
    gate = threading.Event()
    finished = []

    def slow():
        gate.wait(5)
        time.sleep(0.2)
        finished.append(1)
        return 1
    monkeypatch.setattr(runners, "_beside", lambda fn, slot: runners._Pending(fn, "dq-helper-" + slot))
    with pytest.raises(RuntimeError, match="main thread failed"):
        with runners._Helpers() as helpers:
            helpers.beside(slow, "group0")
            helpers.beside(lambda: (_ for _ in ()).throw(ValueError("helper failed")), "group1")
            gate.set()
            raise RuntimeError("main thread failed")
    assert finished == [1] and not _helper_threads()
    # a helper's error is re-raised by result() only after the group has joined the others
    with pytest.raises(ValueError, match="helper failed"):
        with runners._Helpers() as helpers:
            helpers.beside(lambda: (_ for _ in ()).throw(ValueError("helper failed")), "group0")
            helpers.beside(slow, "group1")
            for h in helpers.pending:
                h.result()
    assert not _helper_threads()


class _FakeLib:
    def __init__(self):
        self.trims = []

    def dq_scratch_trim(self, handle, keep):
        self.trims.append((handle, keep))


def test_aux_contexts_are_leased_to_one_thread_at_a_time(monkeypatch):
    """dq.h: calls on one ctx are not re-entrant. Two helpers of one slot (e.g. two user threads running the same
    analysis) get two contexts; a released context is leased again and keeps at most the idle scratch cap."""
    from deequ_amd import native as N
    lib = _FakeLib()

    class FakeContext:
        n = 0

        def __init__(self, device):
            FakeContext.n += 1
            self.device, self.lib, self.handle = device, lib, FakeContext.n
            self.priorities = []

        def set_priority(self, p):
            self.priorities.append(p)
    monkeypatch.setattr(N, "Context", FakeContext)
    monkeypatch.setattr(N, "_aux_pool", {})
    monkeypatch.setattr(N, "_aux_leased", set())
    a = N.lease_aux_context(0, "group0")
    b = N.lease_aux_context(0, "group0")
    assert a is not b
    N.release_aux_context(a)
    assert lib.trims == [(a.handle, N.AUX_IDLE_SCRATCH_BYTES)]
    assert N.lease_aux_context(0, "group0") is a
    assert N.lease_aux_context(1, "group0") not in (a, b)  # per device
    N.release_aux_context(a)
    N.release_aux_context(b)
    assert N.lease_aux_context(0, "group0", priority=1).priorities[-1] == 1  # the lease sets the stream priority
    assert not N._aux_leased - {id(c) for pool in N._aux_pool.values() for c in pool if c.device == 1} - {id(a)} - {id(c) for pool in N._aux_pool.values() for c in pool if c.device == 1}


def test_run_async_is_a_helper_run_or_done_here(monkeypatch):
    """AnalysisRunBuilder.runAsync: run() handed to a helper slot "async", or computed on this thread (a done handle)
    where no helper may be used."""
    sentinel = object()
    monkeypatch.setattr(runners.AnalysisRunner, "doAnalysisRun", staticmethod(lambda *a: sentinel))
    monkeypatch.setenv("DQ_RUN_SERIAL", "1")
    h = runners.AnalysisRunBuilder(None).runAsync()
    assert isinstance(h, runners._Done) and h.result() is sentinel
    monkeypatch.delenv("DQ_RUN_SERIAL")
    slots = []

    def fake_beside(fn, slot, priority=0):
        slots.append(slot)
        return runners._Pending(fn)
    monkeypatch.setattr(runners, "_beside", fake_beside)
    assert runners.AnalysisRunBuilder(None).runAsync().result() is sentinel
    assert slots == ["async"]


def test_run_async_lets_its_run_start_helpers_one_level_deep(monkeypatch):
    """DQ_ASYNC_NESTED=1: runAsync's run may put its own grouping sets on helper contexts (at its priority); their
    helpers may not. Off (the default): the whole run stays on its one helper context."""
    leases = []

    def lease(dev, slot, priority=0):
        leases.append((slot, priority))
        return object()
    monkeypatch.setattr(runners.N, "lease_aux_context", lease)
    monkeypatch.setattr(runners.N, "release_aux_context", lambda c: None)
    monkeypatch.setattr(runners.engine, "device", lambda: 0)
    monkeypatch.delenv("DQ_RUN_SERIAL", raising=False)
    monkeypatch.setenv("DQ_ASYNC_NESTED", "1")
    seen = {}

    def fake_run(self):
        inner = runners._beside(lambda: runners._beside(lambda: 1, "deeper"), "inner")
        seen["inner"] = inner is not None
        seen["deeper"] = inner.result() if inner is not None else "n/a"
        return 7
    monkeypatch.setattr(runners.AnalysisRunBuilder, "run", fake_run)
    assert runners.AnalysisRunBuilder(None).runAsync(priority=1).result() == 7
    assert seen == {"inner": True, "deeper": None}
    assert leases == [("async", 1), ("inner", 1)]
    monkeypatch.setenv("DQ_ASYNC_NESTED", "0")
    seen.clear()
    assert runners.AnalysisRunBuilder(None).runAsync().result() == 7
    assert seen == {"inner": False, "deeper": "n/a"}


def test_helper_priority_default_from_the_environment(monkeypatch):
    """Helpers started outside a runAsync thread take DQ_HELPER_PRIORITY (default 0)."""
    leases = []
    monkeypatch.setattr(runners.N, "lease_aux_context", lambda dev, slot, priority=0: leases.append(priority) or object())
    monkeypatch.setattr(runners.N, "release_aux_context", lambda c: None)
    monkeypatch.setattr(runners.engine, "device", lambda: 0)
    monkeypatch.delenv("DQ_RUN_SERIAL", raising=False)
    monkeypatch.delenv("DQ_HELPER_PRIORITY", raising=False)
    assert runners._beside(lambda: 5, "x").result() == 5
    monkeypatch.setenv("DQ_HELPER_PRIORITY", "-1")
    assert runners._beside(lambda: 6, "x").result() == 6
    assert leases == [0, -1]

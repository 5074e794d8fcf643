"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the pure host code (SURVEY.md §5 race detection /
sanitizers row; VERDICT r2 missing #6): libdq's state algebra, HLL++ estimate, Spark hash, Spark / Java string
parsers and multi-device shard arithmetic (deequ_amd/csrc/host_algebra.cpp + dq_parse.h built with -DDQ_HOST_ONLY),
and the CPU oracle (oracle/dq_oracle.c), each on exactly-sized heap buffers. Built and run here, on the CPU."""
import os
import subprocess

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")


def _run(exe):
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    p = subprocess.run([os.path.join(HERE, "build", exe)], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0 and "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, \
        (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    return p.stdout


def test_host_algebra_parsers_and_shards_under_asan_ubsan():
    assert "host_checks: ok" in _run("host_checks")


def test_oracle_under_asan_ubsan():
    assert "oracle_checks: ok" in _run("oracle_checks")

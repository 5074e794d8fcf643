#!/bin/bash
# One GPU call: tests -> smoke -> bench -> rocprof kernel-trace summary. Stops at the first crash;
# a failing test (pytest rc 1) still lets the bench run so numbers are collected.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
ROWS=${ROWS:-1e9}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${TAG}_smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --rows $ROWS --steps 20 --warmup 3 --cpu-seconds 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; tail -5 gpurun_out/${TAG}_bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/${TAG}_prof" -o run --output-format csv -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --rows $ROWS --steps 10 --warmup 2 --no-cpu > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/${TAG}_prof_bench.json" 2>&1
rc=$?; echo "rocprof rc=$rc"
find "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/${TAG}_prof" -name "*stats*" | head
exit $rc

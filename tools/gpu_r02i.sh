set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multidevice.py tests/test_native_abi.py -m "gpu or not gpu" -x -v --timeout 200 --timeout-method thread > gpurun_out/r02i_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r02i_tests.log | tail -25
exit $rc

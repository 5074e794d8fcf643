set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_grouping.py tests/test_gpu_multidevice.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02o_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r02o_tests.log
exit 0

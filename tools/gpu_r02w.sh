set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multidevice.py tests/test_gpu_freq_merge.py tests/test_gpu_grouping.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02w_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/r02w_tests.log
exit 0

set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_scan.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r02b_tests.log
exit $rc

set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 > gpurun_out/r02c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r02c_tests.log
exit $rc

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k c4_full --timeout 400 --timeout-method thread > gpurun_out/r02aa_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r02aa_tests.log
exit 0

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_heavy.py tests/test_gpu_configs.py -k "not c4" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ax_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02ax_tests.log
[ $rc -ne 0 ] && exit $rc
for c in c3 suite10; do timeout -k 10 300 python -u tools/bench_configs.py --config $c --steps 5 2>/dev/null | cut -c1-150; done
exit 0

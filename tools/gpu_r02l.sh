set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_multidevice.py tests/test_gpu_grouping.py tests/test_gpu_freq_merge.py tests/test_gpu_regex.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02l_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02l_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --config c4 --steps 5 > gpurun_out/r02l_c4.json 2>&1; echo "c4 rc=$? $(tail -1 gpurun_out/r02l_c4.json | head -c 400)"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r02l_bench.json 2> gpurun_out/r02l_bench.err; echo "bench rc=$?"; tail -c 3000 gpurun_out/r02l_bench.json
exit 0

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_grouping.py tests/test_gpu_freq_merge.py tests/test_gpu_multidevice.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02j_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02j_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r02j_bench.json 2> gpurun_out/r02j_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/r02j_bench.json; tail -3 gpurun_out/r02j_bench.err
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02j_prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/r02j_prof_bench.json" 2>&1; echo "prof rc=$?"
exit 0

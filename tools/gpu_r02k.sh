set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_grouping.py tests/test_gpu_freq_merge.py tests/test_gpu_regex.py tests/test_gpu_scan.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02k_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02k_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --config c4 --steps 5 > gpurun_out/r02k_c4.json 2>&1; echo "c4 rc=$? $(tail -1 gpurun_out/r02k_c4.json | head -c 400)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02k_prof" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config c4 --steps 3 > "$R/gpurun_out/r02k_prof.log" 2>&1; echo "prof rc=$?"
exit 0

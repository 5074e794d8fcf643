set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_heavy.py tests/test_gpu_scan.py tests/test_gpu_configs.py -k "not c4" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02bm_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02bm_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-secondary --no-cpu --steps 20 > gpurun_out/r02bm_c2_$i.json 2>/dev/null; echo "c2 $(python3 -c "import json;d=json.load(open('gpurun_out/r02bm_c2_$i.json'));print(round(d['ms_per_step'],3), round(d['roofline']['frac'],4))")"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02bm_c2" -o run --output-format csv -- python3 "$R/bench.py" --no-secondary --no-cpu > /dev/null 2>&1; echo "prof rc=$?"
grep -h "scan_values_kernel" "$R/gpurun_out/r02bm_c2/run_kernel_stats.csv" | cut -d, -f1,4 | cut -c1-60,140-200
exit 0

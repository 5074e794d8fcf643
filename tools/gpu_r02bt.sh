# Bitmap words by scalar loads in the striped kernel: parity, where-cost and C2 timing.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_pred_simple.py tests/test_gpu_scan.py tests/test_gpu_heavy.py tests/test_gpu_configs.py -k "not c4" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02bt_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02bt_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/where_cost.py > gpurun_out/r02bt_where.log 2>&1 || exit 1
grep ms gpurun_out/r02bt_where.log
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-secondary --no-cpu > gpurun_out/r02bt_c2_$i.json 2>/dev/null || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r02bt_c2_$i.json'));print('c2', round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"; done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02bt_prof" -o run --output-format csv -- python3 "$R/tools/where_cost.py" > /dev/null 2>&1; echo "prof rc=$?"
exit 0

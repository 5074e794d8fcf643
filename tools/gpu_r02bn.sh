set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_heavy.py tests/test_gpu_scan.py tests/test_gpu_configs.py -k "not c4" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02bn_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02bn_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/r02bn_bench.json 2> gpurun_out/r02bn_bench.err; echo "bench rc=$?"
python3 -c "
import json
for l in open('gpurun_out/r02bn_bench.json'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d.get('config',{}).get('workload'), round(d['ms_per_step'],3), d.get('roofline',{}).get('frac'))
    else: print(l[:200])
"
exit 0

# Concurrent scan launches (DQ_SCAN_CONCURRENT): parity with the knob on, then bench A/B of every line.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
DQ_SCAN_CONCURRENT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_heavy.py tests/test_gpu_strings.py tests/test_gpu_profile_c5.py tests/test_gpu_profiles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02bo_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02bo_tests.log
[ $rc -ne 0 ] && exit $rc
for c in 0 1; do
  DQ_SCAN_CONCURRENT=$c timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/r02bo_bench_$c.json 2> gpurun_out/r02bo_bench_$c.err || { echo "bench $c failed"; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r02bo_bench_$c.json') if l.startswith('{')][0])
print('conc=$c C2', round(d['ms_per_step'],3))
for k,s in d['secondary'].items(): print('conc=$c', k, round(s['ms_per_step'],3))
"
done

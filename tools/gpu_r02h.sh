set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_scan.py tests/test_gpu_freq_merge.py tests/test_gpu_grouping.py tests/test_gpu_state_provider.py -m gpu -x -v --timeout 200 --timeout-method thread -s > gpurun_out/r02h_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|merge .* MI" gpurun_out/r02h_tests.log | tail -3
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for c in hll8 suite10; do
  timeout -k 10 120 python -u tools/bench_configs.py --config $c --steps 5 > gpurun_out/r02h_$c.json 2> gpurun_out/r02h_$c.err; rc=$?
  echo "$c rc=$rc $(cat gpurun_out/r02h_$c.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["frac_of_peak"])')"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

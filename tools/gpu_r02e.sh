set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 100 -k suite10 > gpurun_out/r02e_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r02e_parity.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in base b2 b3 b4; do
  if [ $v = base ]; then export DQ_SCAN_NO_LEAN=1; unset DQ_LIBRARY; else unset DQ_SCAN_NO_LEAN; export DQ_LIBRARY=$R/tools/micro/libdq_$v.so; fi
  timeout -k 10 120 python -u tools/bench_configs.py --config suite10 --steps 5 > gpurun_out/r02e_s10_$v.json 2> gpurun_out/r02e_s10_$v.err; rc=$?
  echo "$v rc=$rc $(cat gpurun_out/r02e_s10_$v.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["frac_of_peak"])')"
  [ $rc -ne 0 ] && exit $rc
done
unset DQ_SCAN_NO_LEAN DQ_LIBRARY
exit 0

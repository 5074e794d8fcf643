set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 100 > gpurun_out/r02f_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r02f_parity.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in pipe m3; do
  if [ $v = pipe ]; then unset DQ_LIBRARY; else export DQ_LIBRARY=$R/tools/micro/libdq_$v.so; fi
  timeout -k 10 120 python -u tools/bench_configs.py --config suite10 --steps 5 > gpurun_out/r02f_s10_$v.json 2> gpurun_out/r02f_s10_$v.err; rc=$?
  echo "$v rc=$rc $(cat gpurun_out/r02f_s10_$v.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["frac_of_peak"])')"
  [ $rc -ne 0 ] && exit $rc
done
unset DQ_LIBRARY
timeout -k 10 120 python -u tools/bench_configs.py --config c3 --steps 5 > gpurun_out/r02f_c3.json 2>&1; echo "c3 rc=$? $(head -c 300 gpurun_out/r02f_c3.json)"
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r02f_c2.json 2>gpurun_out/r02f_c2.err; echo "c2 rc=$? $(head -c 400 gpurun_out/r02f_c2.json)"
exit 0

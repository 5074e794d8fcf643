set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in def nt def nt; do
  if [ $v = nt ]; then export DQ_LIBRARY=$R/variants/libdq_nt.so; else unset DQ_LIBRARY; fi
  timeout -k 10 200 python -u bench.py --no-secondary --no-cpu --steps 20 > gpurun_out/r02ao_$v.json 2> gpurun_out/r02ao_$v.err; rc=$?
  echo "$v rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/r02ao_$v.json'));print(round(d['ms_per_step'],3), d['roofline']['kernel'][:60], round(d['roofline']['frac'],4))")"
  [ $rc -ne 0 ] && exit $rc
done
unset DQ_LIBRARY
for v in def nt; do
  if [ $v = nt ]; then export DQ_LIBRARY=$R/variants/libdq_nt.so; else unset DQ_LIBRARY; fi
  timeout -k 10 200 python -u tools/bench_configs.py --config c3 --steps 5 > gpurun_out/r02ao_c3_$v.json 2>/dev/null; echo "c3 $v $(cat gpurun_out/r02ao_c3_$v.json | cut -c1-120)"
done
exit 0

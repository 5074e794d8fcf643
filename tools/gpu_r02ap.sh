set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in def nt lean lean0 def nt lean lean0; do
  case $v in def) unset DQ_LIBRARY;; *) export DQ_LIBRARY=$R/variants/libdq_$v.so;; esac
  timeout -k 10 200 python -u bench.py --no-secondary --no-cpu --steps 20 > gpurun_out/r02ap_$v.json 2> gpurun_out/r02ap_$v.err; rc=$?
  echo "$v rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/r02ap_$v.json'));print(round(d['ms_per_step'],3), round(d['roofline']['frac'],4))")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

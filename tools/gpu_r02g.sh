set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in hll8 corr4 s10_nocorr suite10; do
  timeout -k 10 120 python -u tools/bench_configs.py --config $c --steps 5 > gpurun_out/r02g_$c.json 2> gpurun_out/r02g_$c.err; rc=$?
  echo "$c rc=$rc $(cat gpurun_out/r02g_$c.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["frac_of_peak"])')"
  [ $rc -ne 0 ] && exit $rc
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02g_prof" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config suite10 --steps 3 > "$R/gpurun_out/r02g_prof.log" 2>&1; echo "prof rc=$?"
exit 0

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/r02ad_pmc_$c" -o run --output-format csv -- python3 "$R/tools/c4_phases.py" 1e9 2 > "$R/gpurun_out/r02ad_pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

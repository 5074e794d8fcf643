set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d "$R/gpurun_out/r02av_pmc_$c" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-secondary > "$R/gpurun_out/r02av_pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 240 rocprofv3 --pmc $c -d "$R/gpurun_out/r02av_s10_$c" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config suite10 --steps 2 --warmup 0 > "$R/gpurun_out/r02av_s10_$c.log" 2>&1
  rc=$?; echo "s10 pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02av_bench" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$R/gpurun_out/r02av_bench.log" 2>&1
rc=$?; echo "bench prof rc=$rc"; grep -h '^{' "$R/gpurun_out/r02av_bench.log" | cut -c1-200
exit $rc

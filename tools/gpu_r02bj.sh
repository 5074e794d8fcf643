set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02bj_c2" -o run --output-format csv -- python3 "$R/bench.py" --no-secondary --no-cpu > "$R/gpurun_out/r02bj_c2.log" 2>&1
rc=$?; echo "c2 prof rc=$rc"; grep -h '^{' "$R/gpurun_out/r02bj_c2.log" | cut -c1-200
grep -h "scan_values_kernel\|reduce_partials\|finalize_kernel" "$R/gpurun_out/r02bj_c2/run_kernel_stats.csv" | cut -d, -f1,2,4 | cut -c1-60,140-200
exit $rc

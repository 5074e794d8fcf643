set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02aw_def" -o run --output-format csv -- python3 "$R/tools/c4_p1_exp.py" > "$R/gpurun_out/r02aw_def.log" 2>&1; echo "def rc=$?"
DQ_LIBRARY=$R/variants/libdq_p1priv.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02aw_priv" -o run --output-format csv -- python3 "$R/tools/c4_p1_exp.py" > "$R/gpurun_out/r02aw_priv.log" 2>&1; echo "priv rc=$?"
grep -h "partition1_fast" "$R/gpurun_out/r02aw_def/run_kernel_stats.csv" "$R/gpurun_out/r02aw_priv/run_kernel_stats.csv" | cut -d, -f1,3,4 | cut -c1-40,100-200
exit 0

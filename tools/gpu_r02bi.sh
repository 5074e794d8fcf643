set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for v in def k128; do
  case $v in def) unset DQ_LIBRARY;; *) export DQ_LIBRARY=$R/variants/libdq_$v.so;; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02bi_$v" -o run --output-format csv -- python3 "$R/tools/c5_shard.py" 1e8 2 > /dev/null 2>&1; echo "prof $v rc=$?"
  grep -h "kll_compact_x_kernel<256, 8>\|kll_compact_x_kernel<128, 16>" "$R/gpurun_out/r02bi_$v/run_kernel_stats.csv" | cut -d, -f1,2,3 | cut -c1-70,100-160
done
exit 0

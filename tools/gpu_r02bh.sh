set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in def t2048 t8192 def t2048; do
  case $v in def) unset DQ_LIBRARY;; *) export DQ_LIBRARY=$R/variants/libdq_$v.so;; esac
  timeout -k 10 200 python -u tools/bench_configs.py --config c4 --steps 5 > gpurun_out/r02bh_$v.json 2>/dev/null; echo "$v $(cut -c1-110 gpurun_out/r02bh_$v.json)"
done
unset DQ_LIBRARY
cd /tmp
for v in def t2048; do
  case $v in def) unset DQ_LIBRARY;; *) export DQ_LIBRARY=$R/variants/libdq_$v.so;; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02bh_prof_$v" -o run --output-format csv -- python3 "$R/tools/c4_p1_exp.py" > /dev/null 2>&1; echo "prof $v rc=$?"
  grep -h "partition1_fast\|scatter2_fast\|build_kernel" "$R/gpurun_out/r02bh_prof_$v/run_kernel_stats.csv" | cut -d, -f1,4 | cut -c1-60,150-200
done
exit 0

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
for c in suite10 hll8; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02ak_$c" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config $c --steps 3 > "$R/gpurun_out/r02ak_$c.log" 2>&1
rc=$?; echo "$c prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES -d "$R/gpurun_out/r02ak_sqh" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config hll8 --steps 1 --warmup 0 > "$R/gpurun_out/r02ak_sqh.log" 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d "$R/gpurun_out/r02ak_sql" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config hll8 --steps 1 --warmup 0 > "$R/gpurun_out/r02ak_sql.log" 2>&1
rc=$?; echo "pmc2 rc=$rc"; tail -2 "$R/gpurun_out/r02ak_sql.log"
exit $rc

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES -d "$R/gpurun_out/r02d_sq" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config suite10 --steps 1 --warmup 0 > "$R/gpurun_out/r02d_sq.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 "$R/gpurun_out/r02d_sq.log"
exit $rc

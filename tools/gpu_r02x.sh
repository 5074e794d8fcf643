set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES -d "$R/gpurun_out/r02x_sq" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config c2 --steps 1 --warmup 0 > "$R/gpurun_out/r02x_sq.log" 2>&1; echo "sq rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02x_prof" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config c2 --steps 5 > "$R/gpurun_out/r02x_prof.log" 2>&1; echo "prof rc=$?"
exit 0

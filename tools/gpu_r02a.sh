set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/valu_rates > gpurun_out/r02a_valu.txt 2>&1; echo "valu rc=$?"; cat gpurun_out/r02a_valu.txt
timeout -k 10 120 ./tools/micro/hll_micro > gpurun_out/r02a_hll.txt 2>&1; echo "hll rc=$?"; cat gpurun_out/r02a_hll.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r02a_s10prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --config suite10 --steps 3 > "$GRAFT_REPO_ROOT/gpurun_out/r02a_s10.log" 2>&1; echo "s10 rc=$?"; tail -2 "$GRAFT_REPO_ROOT/gpurun_out/r02a_s10.log"

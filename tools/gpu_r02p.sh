set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES -d "$R/gpurun_out/r02p_sq1" -o run --output-format csv -- python3 "$R/tools/c4_phases.py" 1e9 2 > "$R/gpurun_out/r02p_sq1.log" 2>&1; echo "sq1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU -d "$R/gpurun_out/r02p_sq2" -o run --output-format csv -- python3 "$R/tools/c4_phases.py" 1e9 2 > "$R/gpurun_out/r02p_sq2.log" 2>&1; echo "sq2 rc=$?"
exit 0

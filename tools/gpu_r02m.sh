set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/c4_phases.py 1e9 6 > gpurun_out/r02m_phases.log 2>&1; echo "phases rc=$?"; cat gpurun_out/r02m_phases.log | tail -7
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$R/gpurun_out/r02m_prof" -o run --output-format csv -- python3 "$R/tools/c4_phases.py" 1e9 4 > "$R/gpurun_out/r02m_prof.log" 2>&1; echo "prof rc=$?"
exit 0

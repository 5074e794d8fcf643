set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d "$R/gpurun_out/r02ar_trace" -o run --output-format csv -- python3 "$R/tools/c5_shard.py" 1e8 1 > "$R/gpurun_out/r02ar.log" 2>&1; echo "trace rc=$?"; grep -h '^{' "$R/gpurun_out/r02ar.log" | cut -c1-300
exit 0

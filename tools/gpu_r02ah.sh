set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02ah_prof" -o run --output-format csv -- python3 "$R/tools/c5_shard.py" 1e8 2 > "$R/gpurun_out/r02ah_prof.log" 2>&1; echo "prof rc=$?"
exit 0

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg_c5.py 1e8 > gpurun_out/r02ag.log 2>&1; echo "rc=$?"; tail -8 gpurun_out/r02ag.log
timeout -k 10 400 python -u tools/c5_shard.py 1e8 2 > gpurun_out/r02ag_c5.json 2>&1; echo "c5 1e8 rc=$?"; tail -c 900 gpurun_out/r02ag_c5.json
exit 0

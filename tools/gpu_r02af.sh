set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c5_shard.py 1e7 2 > gpurun_out/r02af_c5_small.json 2>&1; rc=$?; echo "c5 1e7 rc=$rc"; tail -c 1500 gpurun_out/r02af_c5_small.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/c5_shard.py 1e8 2 > gpurun_out/r02af_c5.json 2>&1; echo "c5 1e8 rc=$?"; tail -c 800 gpurun_out/r02af_c5.json
exit 0

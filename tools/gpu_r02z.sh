set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in c3 suite10 c2; do
timeout -k 10 200 python -u tools/bench_configs.py --config $c --steps 5 > gpurun_out/r02z_$c.json 2>&1; echo "$c rc=$? $(tail -1 gpurun_out/r02z_$c.json | head -c 300)"
done
exit 0

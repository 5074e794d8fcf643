set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_configs.py --config kll_nulls --rows 2.5e8 --steps 3 > gpurun_out/r02ae_kll.json 2>&1; echo "kll rc=$? $(tail -1 gpurun_out/r02ae_kll.json | head -c 300)"
exit 0

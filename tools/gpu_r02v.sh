set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r02v_bench.json 2> gpurun_out/r02v_bench.err; echo "bench rc=$?"; tail -c 1500 gpurun_out/r02v_bench.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02v_prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu > "$R/gpurun_out/r02v_prof.log" 2>&1; echo "prof rc=$?"
exit 0

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02bw_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r02bw_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02bw_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r02bw_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r02bw_bench.json 2> gpurun_out/r02bw_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/r02bw_bench.json
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02bw_prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$R/gpurun_out/r02bw_prof_bench.json" 2>/dev/null; echo "prof rc=$?"
exit 0

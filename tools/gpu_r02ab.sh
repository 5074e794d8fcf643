set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_grouping.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02ab_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02ab_tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02ab_prof" -o run --output-format csv -- python3 "$R/tools/c4_phases.py" 1e9 5 > "$R/gpurun_out/r02ab_prof.log" 2>&1; echo "prof rc=$?"
grep "step 4" "$R/gpurun_out/r02ab_prof.log"
exit 0

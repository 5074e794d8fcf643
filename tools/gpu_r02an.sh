set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_strings.py tests/test_gpu_profile_c5.py tests/test_gpu_profiles.py tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02an_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r02an_tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02an_prof" -o run --output-format csv -- python3 "$R/tools/c5_shard.py" 1e8 2 > "$R/gpurun_out/r02an_prof.log" 2>&1; echo "prof rc=$?"; grep -h '^{' "$R/gpurun_out/r02an_prof.log"
exit 0

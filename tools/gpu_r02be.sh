set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kll.py tests/test_gpu_profiles.py tests/test_gpu_profile_c5.py tests/test_gpu_quantiles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02be_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02be_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/c5_shard.py 1e8 3 > gpurun_out/r02be_c5.json 2>&1; echo "c5 rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02be_c5.json
exit 0

# Simple-predicate kernel: parity (vs the VM and the oracle) + where-cost A/B.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pred_simple.py tests/test_gpu_scan.py tests/test_gpu_verification.py tests/test_gpu_heavy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02br_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r02br_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/where_cost.py > gpurun_out/r02br_where_fast.log 2>&1 || exit 1
DQ_PRED_VM=1 timeout -k 10 300 python -u tools/where_cost.py > gpurun_out/r02br_where_vm.log 2>&1 || exit 1
echo fast; cat gpurun_out/r02br_where_fast.log | grep ms; echo vm; cat gpurun_out/r02br_where_vm.log | grep ms
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02br_prof" -o run --output-format csv -- python3 "$R/tools/where_cost.py" > /dev/null 2>&1; echo "prof rc=$?"
exit 0

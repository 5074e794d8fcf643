set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_configs.py -k "not c4" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02aj_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r02aj_tests.log
[ $rc -ne 0 ] && exit $rc
for c in suite10 hll8 c3; do
  timeout -k 10 300 python -u tools/bench_configs.py --config $c --steps 5 > gpurun_out/r02aj_$c.json 2> gpurun_out/r02aj_$c.err; rc=$?; echo "$c rc=$rc"; cat gpurun_out/r02aj_$c.json
  [ $rc -ne 0 ] && exit $rc
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES -d "$R/gpurun_out/r02aj_sq" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config suite10 --steps 1 --warmup 0 > "$R/gpurun_out/r02aj_sq.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 "$R/gpurun_out/r02aj_sq.log"
exit $rc

#!/bin/bash
# One GPU-box call, several steps: tools/gpu.sh TAG STEP [STEP ...], run from the repo root (gpurun does that).
#   test:ARGS    python -m pytest ARGS -m gpu (per-test timeout 300 s)        -> gpurun_out/TAG_test<i>.log
#   smoke        __graft_entry__.smoke()                                      -> gpurun_out/TAG_smoke.log
#   bench:ARGS   python bench.py ARGS                                         -> gpurun_out/TAG_bench<i>.json / .err
#   py:ARGS      python -u ARGS (a tools/ script)                             -> gpurun_out/TAG_py<i>.log
#   prof:ARGS    rocprofv3 --kernel-trace --stats -- python -u ARGS           -> gpurun_out/TAG_prof<i>/
#   pmc:CTRS:ARGS  rocprofv3 --pmc CTRS -- python -u ARGS (one counter pass)  -> gpurun_out/TAG_pmc<i>/
# Every step runs under its own time limit; the call stops at the first crash / abort / time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
shift
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=${step#*:}
  case $kind in
    test)
      timeout -k 10 900 python -u -m pytest $arg -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_test$i.log 2>&1
      rc=$?; tail -4 gpurun_out/${TAG}_test$i.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > gpurun_out/${TAG}_bench$i.json 2> gpurun_out/${TAG}_bench$i.err
      rc=$?; cat gpurun_out/${TAG}_bench$i.json; tail -3 gpurun_out/${TAG}_bench$i.err ;;
    py)
      timeout -k 10 600 python -u $arg > gpurun_out/${TAG}_py$i.log 2>&1
      rc=$?; tail -20 gpurun_out/${TAG}_py$i.log ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof$i -o p -- python -u $arg > gpurun_out/${TAG}_prof$i.log 2>&1
      rc=$?; tail -5 gpurun_out/${TAG}_prof$i.log ;;
    pmc)
      ctrs=${arg%%:*}
      cmd=${arg#*:}
      timeout -s KILL 180 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/${TAG}_pmc$i -o p -- python -u $cmd > gpurun_out/${TAG}_pmc$i.log 2>&1
      rc=$?; tail -3 gpurun_out/${TAG}_pmc$i.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "== step $i ($kind) rc=$rc"
  # pytest: 1 = test failures (the GPU is fine, go on); anything else non-zero ends the call
  if [ $rc -ne 0 ] && ! { [ "$kind" = test ] && [ $rc -eq 1 ]; }; then exit $rc; fi
done

#!/bin/bash
# SQ counters of bench_configs CONFIG per libdq variant: tools/ab_pmc.sh TAG CONFIG LIB ...  (one --pmc pass each)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
CTRS=${CTRS:-"SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY"}
i=0
for lib in "$@"; do
  i=$((i + 1))
  if [ "$lib" = main ]; then L=""; else L="DQ_LIBRARY=$PWD/tools/ab/$lib.so"; fi
  env $L timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/${TAG}_$i -o p -- python3 -u tools/bench_configs.py --config $CFG --steps 2 > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; echo "pmc $lib rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_$i.log; exit $rc; fi
done

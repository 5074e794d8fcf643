#!/bin/bash
# A/B of libdq variants on the GPU box: tools/ab_run.sh TAG CONFIG LIB[:ENV=VAL] ...   (CONFIG: c4 | c5)
# each variant under rocprofv3 --kernel-trace --stats -> gpurun_out/TAG_<i>/ plus its JSON line in TAG_<i>.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
i=0
for v in "$@"; do
  i=$((i + 1))
  lib=${v%%:*}; envs=""
  [ "$lib" != "$v" ] && envs=${v#*:}
  case $CFG in
    c4) cmd="tools/bench_configs.py --config c4 --steps 6" ;;
    c5) cmd="tools/c5_shard.py 2.5e8 3" ;;
    s10) cmd="tools/bench_configs.py --config suite10 --steps 6" ;;
    *) echo "unknown config"; exit 2 ;;
  esac
  if [ "$lib" = main ]; then L=""; else L="DQ_LIBRARY=$PWD/tools/ab/$lib.so"; fi
  echo "== variant $i: $lib $envs"
  env $L $envs timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$i -o p -- python3 -u $cmd > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; grep '^{' gpurun_out/${TAG}_$i.log | cut -c1-300; echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_$i.log; exit $rc; fi
done

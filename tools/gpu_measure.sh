#!/bin/bash
# HEAD measurement refresh (one GPU call): HBM traffic (rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, separate passes)
# of C2 (bench.py headline), C4 (bench_configs c4), the C5 shard and suite10, plus a C2-only kernel-trace CSV.
#   tools/gpu_measure.sh TAG [c2 c4 c5 s10 ...]      -> gpurun_out/TAG_<cfg>_<counter>/ and TAG_c2trace/
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
CFGS=${@:-c2 c4 c5 s10}
for cfg in $CFGS; do
  case $cfg in
    c2) cmd="$R/bench.py --steps 3 --warmup 1 --no-cpu --no-secondary" ;;
    c4) cmd="$R/tools/bench_configs.py --config c4 --steps 3" ;;
    c5) cmd="$R/tools/c5_shard.py 2.5e8 1" ;;
    s10) cmd="$R/tools/bench_configs.py --config suite10 --steps 3" ;;
    c3) cmd="$R/tools/bench_configs.py --config c3 --steps 3" ;;
    c2where) cmd="$R/tools/bench_configs.py --config c2where --steps 3" ;;
    *) echo "unknown $cfg"; exit 2 ;;
  esac
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/${TAG}_${cfg}_$c" -o run -- python3 -u $cmd) > "$R/gpurun_out/${TAG}_${cfg}_$c.log" 2>&1
    rc=$?; echo "$cfg $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/${TAG}_${cfg}_$c.log"; exit $rc; fi
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_c2trace" -o run -- python3 -u "$R/bench.py" --steps 10 --warmup 2 --no-cpu --no-secondary) > "$R/gpurun_out/${TAG}_c2trace.log" 2>&1
echo "c2 trace rc=$?"

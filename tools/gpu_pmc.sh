#!/bin/bash
# HBM traffic of the bench's dominant pass: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
# they cannot share a pass on gfx950), then a per-kernel summary. Also a kernel-trace of suite10.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01f}
ROWS=${ROWS:-1e9}
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d "$R/gpurun_out/${TAG}_pmc_$c" -o run --output-format csv -- python3 "$R/bench.py" --rows $ROWS --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/${TAG}_pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/${TAG}_pmc_$c.log"; exit $rc; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_s10prof" -o run --output-format csv -- python3 "$R/tools/bench_configs.py" --config suite10 --steps 3 > "$R/gpurun_out/${TAG}_s10prof.log" 2>&1
rc=$?; echo "suite10 prof rc=$rc"
exit $rc

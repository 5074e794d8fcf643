#!/bin/bash
# distributed GPU tests + 2-rank gloo rehearsal of bench.py on one GPU + secondary configs
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r01c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${T}_dist.log 2>&1
rc=$?; echo "dist tests rc=$rc"; tail -3 gpurun_out/${T}_dist.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --rows 2e8 --dist-backend gloo --device-override 0 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.err
rc=$?; echo "bench 2-rank rc=$rc"; cat gpurun_out/${T}_bench2.json; tail -3 gpurun_out/${T}_bench2.err
if [ $rc -ne 0 ]; then exit $rc; fi
for c in c3 suite10 c4; do
  timeout -k 10 300 python -u tools/bench_configs.py --config $c --steps 5 > gpurun_out/${T}_${c}.json 2> gpurun_out/${T}_${c}.err
  rc=$?; echo "$c rc=$rc"; cat gpurun_out/${T}_${c}.json; tail -3 gpurun_out/${T}_${c}.err
  if [ $rc -ne 0 ]; then exit $rc; fi
done

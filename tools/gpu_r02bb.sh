set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02bb_dist.log 2>&1; rc=$?; echo "dist tests rc=$rc"; tail -3 gpurun_out/r02bb_dist.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --rows 2e8 --dist-backend gloo --device-override 0 > gpurun_out/r02bb_bench2.json 2> gpurun_out/r02bb_bench2.err
rc=$?; echo "bench 2-rank rc=$rc"; grep '^{' gpurun_out/r02bb_bench2.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline())
print({k:(round(v['ms_per_step'],2)) for k,v in d['secondary'].items()})"; grep -v Gloo gpurun_out/r02bb_bench2.err | grep -i "error\|assert" | head -5
exit $rc

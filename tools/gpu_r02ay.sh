set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --rows 2e8 --dist-backend gloo --device-override 0 > gpurun_out/r02ay_bench2.json 2> gpurun_out/r02ay_bench2.err
rc=$?; echo "bench 2-rank rc=$rc"; cut -c1-400 gpurun_out/r02ay_bench2.json; python3 -c "
import json; d=json.load(open('gpurun_out/r02ay_bench2.json'))
print({k:(round(v['ms_per_step'],2)) for k,v in d['secondary'].items()})"; tail -3 gpurun_out/r02ay_bench2.err
exit $rc

set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --rows 4e8 --dist-backend gloo --device-override 0 --no-cpu > gpurun_out/r02ac_bench2.json 2> gpurun_out/r02ac_bench2.err; echo "bench2 rc=$?"; tail -c 1200 gpurun_out/r02ac_bench2.json
exit 0

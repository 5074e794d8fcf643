set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in new old new old; do
  if [ $v = old ]; then export DQ_LIBRARY=$R/variants/libdq_oldkll.so; else unset DQ_LIBRARY; fi
  timeout -k 10 200 python -u tools/c5_shard.py 1e8 3 > gpurun_out/r02bf_$v.json 2>&1; echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02bf_$v.json)"
done
exit 0

cd ${GRAFT_REPO_ROOT:-/root/repo}
DQ_KLL_TIMING=1 timeout -k 10 300 python3 -u tools/c5_shard.py 2.5e8 2 > gpurun_out/${KT_TAG:-kll_timing}.log 2>&1
echo rc=$?
grep dq_kll_sketch gpurun_out/${KT_TAG:-kll_timing}.log | tail -6

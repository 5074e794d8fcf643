set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in win nowin; do
  if [ $v = nowin ]; then E="DQ_FREQ_NO_WINDOW=1"; else E="DQ_FREQ_WINDOW_PARTS=2"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    env $E timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r05g_${v}_$c -o p -- python3 -u tools/bench_configs.py --config c4 --steps 2 > gpurun_out/r05g_${v}_$c.log 2>&1
    rc=$?; echo "$v $c rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0

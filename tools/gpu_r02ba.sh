set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1.25e8 2.5e8 5e8; do
timeout -k 10 200 python -u bench.py --no-secondary --no-cpu --rows $r --steps 40 > gpurun_out/r02ba_$r.json 2>/dev/null; echo "rows $r rc=$? $(python3 -c "import json;d=json.load(open('gpurun_out/r02ba_$r.json'));print(round(d['ms_per_step'],3), d['roofline']['kernel'][85:120])")"
done
exit 0

set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in 1 2; do for v in base gramfirst gramhi gramfirst,gramhi; do
  BISCOTTI_EXP=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$v.txt 2>&1 || { echo FAIL $v; tail -5 gpurun_out/ab_$v.txt; exit 1; }
  grep "^{" gpurun_out/ab_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3), 'kw', round(d['phase_ms_per_round']['verify.krum_wait'],3), 'rb', round(d['phase_ms_per_round']['recover.readback'],3))"
done; done

# Same-box A/B of BISCOTTI_EXP variants (temporary experiment toggles): driver-style and long benches,
# interleaved.  VARIANTS (comma-free list, space separated), REPS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
VARIANTS=${VARIANTS:-base}
for rep in $(seq 1 ${REPS:-2}); do for v in $VARIANTS; do
  BISCOTTI_EXP=$v timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/ab_$v.txt 2>&1 || { echo FAIL $v; tail -5 gpurun_out/ab_$v.txt; exit 1; }
  grep "^{" gpurun_out/ab_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$v', round(d['ms_per_step'],3), 'kw', round(p['verify.krum_wait'],3), 'rb', round(p['recover.readback'],3), 'qa', round(p['verify.queue_agg'],3), 'pv', round(p['pre_vrf'],3), 'rblk', round(p['recover.block'],3))"
done; done

# Same-box A/B of the working tree (new) against ab_base (scripts/make_ab_base.sh: a copy of an earlier commit's package, built
# libraries included): driver-style benches, alternating order per repetition, then one long run each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
R=$PWD
run() {  # $1 = variant, $2 = steps, $3 = warmup, $4 = tag
  if [ $1 = base ]; then D=$R/ab_base; else D=$R; fi
  (cd $D && timeout -k 10 300 python bench.py --steps $2 --warmup $3) > gpurun_out/abt_$1_$4.txt 2>&1 || { echo "FAIL $1 $4"; tail -5 gpurun_out/abt_$1_$4.txt; return 1; }
  grep '^{' gpurun_out/abt_$1_$4.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$1 $4', round(d['ms_per_step'],3), 'drain', round(d.get('drain_ms',0),2), 'rb', round(p['recover.readback'],3), 'audit', round(p['recover.audit'],3), 'idle', round(p.get('recover.idle',0),3), 'qa', round(p['verify.queue_agg'],3), 'pv', round(p['pre_vrf'],3), 'blk', round(p['recover.block'],3), 'kw', round(p['verify.krum_wait'],3))"
}
for rep in $(seq 1 ${REPS:-3}); do
  if [ $((rep % 2)) = 1 ]; then order="base new"; else order="new base"; fi
  for v in $order; do run $v 20 5 s$rep || exit 1; done
done
if [ "${LONG:-1}" = 1 ]; then for v in base new; do run $v 200 10 long || exit 1; done; fi

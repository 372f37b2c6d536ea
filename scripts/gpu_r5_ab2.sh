# Round-5 A/B on one box: the working tree (VRF-job joins and the signature prep moved into the next round's VRF
# wait, latest_hash) against ab_base (HEAD), driver-style alternating x3 + one 200-round run each; then the
# speculative MSM's CU mask on the working tree (7/8, all CUs) x3 each; then a cProfile of a 200-round bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5ab2; mkdir -p $O
run() {  # variant tag steps warmup [args]
  v=$1; t=$2; st=$3; w=$4; shift 4
  if [ $v = base ]; then D=$R/ab_base; else D=$R; fi
  (cd $D && timeout -k 10 300 python bench.py --steps $st --warmup $w "$@") > $O/${v}_$t.txt 2>&1 || { echo "FAIL $v $t"; tail -5 $O/${v}_$t.txt; return 1; }
  grep '^{' $O/${v}_$t.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$v $t', round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'rb', round(p['recover.readback'],3), 'kw', round(p['verify.krum_wait'],3), 'pv', round(p.get('pre_vrf',0),3), 'vj', round(p.get('vrf_join',0),3), 'idle', round(p.get('recover.idle',0),3), flush=True)"
}
for i in 1 2 3; do
  if [ $((i % 2)) = 1 ]; then order="base new"; else order="new base"; fi
  for v in $order; do run $v s$i 20 5 || exit 1; done
done
for v in base new; do run $v long 200 10 || exit 1; done
for i in 1 2 3; do
  run new c78_$i 20 5 --set ablation=side_cus_7of8 || exit 1
  run new call_$i 20 5 --set ablation=side_cus_all || exit 1
done
timeout -k 10 400 python scripts/host_cprofile.py --steps 200 --warmup 10 > $O/cprof.txt 2> $O/cprof.err || { echo "CPROF FAILED"; tail -5 $O/cprof.err; exit 1; }
grep -A45 "by tottime" $O/cprof.txt | head -50

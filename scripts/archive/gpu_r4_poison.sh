# Poisoning (MNIST 100 peers, 30 % 1->7 label flip, epsilon 1) on the working tree and on the round-2 tree
# (ab_r2, scripts/make_ab_base.sh 3177831 ab_r2): digit-1 error over the last 10 rounds per seed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
R=$PWD
for t in ${TREES:-new r2}; do
  if [ $t = r2 ]; then D=$R/ab_r2; else D=$R; fi
  (cd $D && timeout -k 10 500 python scripts/poison_diag.py --config ${CFG:-mnist100_po30_ep1} --seeds ${SEEDS:-5} --rounds 100 \
      -o $R/gpurun_out/poison_$t.json) > gpurun_out/poison_$t.log 2>&1 || { echo "POISON $t FAILED"; tail -5 gpurun_out/poison_$t.log; exit 1; }
  python -c "
import json,statistics as st; d=json.load(open('gpurun_out/poison_$t.json'))
runs=d['runs']; a=[r['attack_last10'] for r in runs]; e=[r['err_last10'] for r in runs]; rj=[r['rejection_rate_after_burnin'] for r in runs]
print('$t', 'attack_last10', [round(x,3) for x in a], 'mean', round(st.mean(a),3), 'sd', round(st.pstdev(a),3), 'err', round(st.mean(e),3), 'rej', round(st.mean(rj),3))"
done

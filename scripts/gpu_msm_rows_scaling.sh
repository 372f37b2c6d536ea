# Isolated speculative-MSM time against the row count (throughput- vs latency-bound), dense and sparse updates
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for dens in 0.8 0.3; do
  for r in 10 20 35 50 72; do
    timeout -k 10 200 python scripts/bench_msm.py --rows $r --density $dens --iters 5 > gpurun_out/msm_rows_${r}_${dens}.json 2>&1 || { echo "FAIL $r $dens"; tail -3 gpurun_out/msm_rows_${r}_${dens}.json; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/msm_rows_${r}_${dens}.json').read().strip().splitlines()[-1]); print('rows', $r, 'density', $dens, 'witness_only_ms', round(d['shares_witness_only_ms'],3), 'commit_all_ms', round(d['commit_rows_all_workers_ms'],3))"
  done
done

# A/B of k_shares_msm builds (exp/libhip_w*.so: occupancy caps) on the isolated MSM microbench
set -o pipefail
for v in ${VARIANTS:-3 4 5}; do for r in 35 62; do
  BISCOTTI_HIP_LIB=$PWD/exp/libhip_w$v.so timeout -k 10 120 python scripts/bench_msm.py --rows $r --iters 20 > gpurun_out/msm_w${v}_r$r.json 2>&1 || { echo "w$v r$r FAILED"; tail -3 gpurun_out/msm_w${v}_r$r.json; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/msm_w${v}_r$r.json').read().strip().splitlines()[-1]);print('w$v r$r', round(d['shares_approved_ms'],3), round(d['commit_rows_all_workers_ms'],3))"
done; done

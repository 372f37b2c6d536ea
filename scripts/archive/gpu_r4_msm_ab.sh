# Same-box A/B of the share MSM: the working tree's kernels vs libbiscotti_hip_base.so (the previous
# commit's kernels, built in-tree beforehand), alternating, headline-size rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then L="--lib biscotti_amd/libbiscotti_hip_base.so"; else L=""; fi
    timeout -k 10 200 python scripts/bench_msm.py --rows 70 --workers 100 --iters 7 $L > gpurun_out/msmab_${v}_$rep.txt 2>&1 || { echo "MSM $v FAILED"; tail -5 gpurun_out/msmab_${v}_$rep.txt; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/msmab_${v}_$rep.txt').read().strip().splitlines()[-1]); print('$v $rep', {k: round(v, 3) for k, v in d.items() if k.endswith('_ms')})"
  done
done

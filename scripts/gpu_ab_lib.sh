# A/B of two builds of the kernel library on ONE box (BISCOTTI_HIP_LIB selects the alternative):
# the MSM micro-benchmark at the headline size and the driver-style bench, alternating A B A B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
ALT=${ALT:-biscotti_amd/libbiscotti_hip_ab.so}
for rep in 1 2; do
  for v in new alt; do
    if [ $v = alt ]; then export BISCOTTI_HIP_LIB=$PWD/$ALT; else unset BISCOTTI_HIP_LIB; fi
    timeout -k 10 200 python scripts/bench_msm.py --rows 70 --workers 94 --iters 5 > gpurun_out/ab_msm_${v}_$rep.txt 2>&1 || { echo "MSM $v FAILED"; tail -5 gpurun_out/ab_msm_${v}_$rep.txt; exit 1; }
    echo "msm $v $rep: $(tail -1 gpurun_out/ab_msm_${v}_$rep.txt | head -c 400)"
    timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 > gpurun_out/ab_bench_${v}_$rep.txt 2>&1 || { echo "BENCH $v FAILED"; tail -5 gpurun_out/ab_bench_${v}_$rep.txt; exit 1; }
    grep '^{' gpurun_out/ab_bench_${v}_$rep.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench $v $rep', round(d['ms_per_step'],3))"
  done
done

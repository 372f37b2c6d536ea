# A/B of the kernel library (new = in-tree build, old = exp/libhip_old.so): bit-exactness tests, the MSM
# micro-benchmark at several coefficient densities, then driver-style benches alternating new/old.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
OLD=${OLD:-exp/libhip_old.so}
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn256.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ab2_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab2_tests.txt; exit 1; }
tail -1 gpurun_out/ab2_tests.txt
for dens in ${DENS:-0.15 0.4 1.0}; do for v in new old; do
  if [ $v = old ]; then export BISCOTTI_HIP_LIB=$PWD/$OLD; else unset BISCOTTI_HIP_LIB; fi
  timeout -k 10 200 python scripts/bench_msm.py --rows 70 --workers 94 --iters 9 --density $dens > gpurun_out/ab2_msm_${v}_$dens.txt 2>&1 || { echo "MSM $v FAILED"; tail -5 gpurun_out/ab2_msm_${v}_$dens.txt; exit 1; }
  tail -1 gpurun_out/ab2_msm_${v}_$dens.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('msm $v dens $dens shares', round(d['shares_approved_ms'],3), 'commit', round(d['commit_rows_all_workers_ms'],3))"
done; done
for rep in ${REPS:-1 2}; do for v in new old; do
  if [ $v = old ]; then export BISCOTTI_HIP_LIB=$PWD/$OLD; else unset BISCOTTI_HIP_LIB; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab2_bench_${v}_$rep.txt 2>&1 || { echo "BENCH $v FAILED"; tail -5 gpurun_out/ab2_bench_${v}_$rep.txt; exit 1; }
  grep '^{' gpurun_out/ab2_bench_${v}_$rep.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('bench $v $rep', round(d['ms_per_step'],3), 'rb', round(p['recover.readback'],3), 'audit', round(p['recover.audit'],3), 'kw', round(p['verify.krum_wait'],3), 'drain', round(d['drain_ms'],2))"
done; done

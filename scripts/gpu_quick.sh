# Quick GPU check after a protocol change: the engine/pipeline GPU tests, then N driver-style and one long
# bench.  Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_ml.py tests/test_gpu_bn256.py tests/test_gpu_engine_paths.py}
REPS=${REPS:-3}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/quick_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/quick_tests.txt; exit 1; }
  tail -1 gpurun_out/quick_tests.txt
fi
for i in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/quick_short_$i.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/quick_short_$i.txt; exit 1; }
  grep "^{" gpurun_out/quick_short_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('short', round(d['ms_per_step'],3), 'acc', d['final_test_acc'], 'kw', round(p['verify.krum_wait'],3), 'rb', round(p['recover.readback'],3), 'drain', d.get('drain_ms'))"
done
if [ "${LONG:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/quick_long.txt 2>&1 || { echo "LONG FAILED"; tail -20 gpurun_out/quick_long.txt; exit 1; }
  grep "^{" gpurun_out/quick_long.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('long', round(d['ms_per_step'],3), 'acc', d['final_test_acc'], {k: round(v,3) for k,v in p.items() if v > 0.03})"
fi

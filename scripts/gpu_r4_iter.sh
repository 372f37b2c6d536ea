# Iteration check: GPU suite (TESTS), driver-style 1-GPU benches (NB of them), optional 2-rank rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
T=${TESTS:-tests}
if [ "$T" != none ]; then
timeout -k 10 ${TT:-800} python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/it_tests.txt 2>&1 || { echo "GPU TESTS FAILED"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/it_tests.txt | tail -30; exit 1; }
echo "passed: $(grep -c PASSED gpurun_out/it_tests.txt)"
fi
for i in $(seq 1 ${NB:-2}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/it_bench_$i.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/it_bench_$i.txt; exit 1; }
  grep '^{' gpurun_out/it_bench_$i.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('bench', round(d['ms_per_step'],3), 'acc', d['final_test_acc'], 'rb', round(p['recover.readback'],3), 'qa', round(p['verify.queue_agg'],3), 'blk', round(p['recover.block'],3), 'stats', d['engine_stats'])"
done
if [ "${LONG:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/it_bench_long.txt 2>&1 || { echo "LONG BENCH FAILED"; tail -20 gpurun_out/it_bench_long.txt; exit 1; }
  grep '^{' gpurun_out/it_bench_long.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('long', round(d['ms_per_step'],3))"
fi
if [ "${RCCL:-0}" = 1 ]; then
  BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 30 --warmup 5 --set ablation=spec_head_shared > gpurun_out/it_bench2r.txt 2>&1 || { echo "RCCL BENCH FAILED"; grep -v "Train Error\|Attack Rate" gpurun_out/it_bench2r.txt | tail -20; exit 1; }
  grep '^{' gpurun_out/it_bench2r.txt | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bench2r', round(d['ms_per_step'],3))
for p in d['per_rank']: print(p['rank'], round(p['host_cpu_ms_per_round'],2), p['thread_cpu_ms_per_round'], p['engine_stats'])"
fi

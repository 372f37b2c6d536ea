# Round-4 GPU check: the one-rank-per-GPU fast path (RCCL rehearsal, spec head forced), the GPU suite,
# a driver-style 1-GPU bench and a 2-rank RCCL bench rehearsal with per-thread CPU attribution.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
T=${TESTS:-tests}
timeout -k 10 ${TT:-900} python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.txt 2>&1 || { echo "GPU TESTS FAILED"; grep -E "PASS|FAIL|Error|error" gpurun_out/gputests.txt | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/gputests.txt
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench1.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench1.txt; exit 1; }
  grep '^{' gpurun_out/bench1.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench1', round(d['ms_per_step'],3), d['engine_stats'], d['thread_cpu_ms_per_round'])"
fi
if [ "${RCCL:-1}" = 1 ]; then
  BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 30 --warmup 5 --set ablation=spec_head_shared > gpurun_out/bench2r.txt 2>&1 || { echo "RCCL BENCH FAILED"; grep -v "Train Error\|Attack Rate" gpurun_out/bench2r.txt | tail -20; exit 1; }
  grep '^{' gpurun_out/bench2r.txt | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bench2r', round(d['ms_per_step'],3))
for p in d['per_rank']: print(p['rank'], round(p['host_cpu_ms_per_round'],2), p['thread_cpu_ms_per_round'], p['engine_stats'])"
fi

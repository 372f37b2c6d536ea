# Full GPU suite, then a 4-rank RCCL rehearsal bench (spec head forced) with per-thread CPU attribution,
# then a rocprofv3 kernel-stats pass of the 1-GPU bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 ${TT:-800} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests_full.txt 2>&1 || { echo "GPU TESTS FAILED"; grep -E "PASS|FAIL|Error|error" gpurun_out/gputests_full.txt | tail -30; exit 1; }
echo "passed: $(grep -c PASSED gpurun_out/gputests_full.txt)"
BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 300 python bench.py --gpus 4 --steps 30 --warmup 5 --set ablation=spec_head_shared > gpurun_out/bench4r.txt 2>&1 || { echo "RCCL4 BENCH FAILED"; grep -v "Train Error\|Attack Rate" gpurun_out/bench4r.txt | tail -20; exit 1; }
grep '^{' gpurun_out/bench4r.txt | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bench4r', round(d['ms_per_step'],3))
for p in d['per_rank']: print(p['rank'], round(p['host_cpu_ms_per_round'],2), p['thread_cpu_ms_per_round'], {k: v for k, v in p['phase_ms_per_round'].items() if v > 0.2})"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python bench.py --steps 40 --warmup 5 > gpurun_out/prof1.txt 2>&1 || { echo "PROF FAILED"; tail -20 gpurun_out/prof1.txt; exit 1; }
find gpurun_out/prof1 -name "*kernel_stats.csv" | head -3

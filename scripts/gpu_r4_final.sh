# Round-4 closing evidence on one box: the GPU suite, three driver-style benches, a 200-round bench, a 2-rank
# RCCL rehearsal, and a rocprofv3 kernel-trace timeline + stats; everything lands in gpurun_out/final/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/final/gputests.txt 2>&1 || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error" gpurun_out/final/gputests.txt | tail -20; exit 1; }
echo "gpu tests passed: $(grep -c PASSED gpurun_out/final/gputests.txt)"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench_driver_$i.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/final/bench_driver_$i.txt; exit 1; }
  grep '^{' gpurun_out/final/bench_driver_$i.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver', d['ms_per_step'], 'acc', d['final_test_acc'], 'drain', round(d['drain_ms'],2))"
done
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/final/bench_long.txt 2>&1 || { echo "LONG FAILED"; exit 1; }
grep '^{' gpurun_out/final/bench_long.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('long', d['ms_per_step'])"
BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 30 --warmup 5 --set ablation=spec_head_shared > gpurun_out/final/bench_rccl2.txt 2>&1 || { echo "RCCL2 FAILED"; tail -20 gpurun_out/final/bench_rccl2.txt; exit 1; }
grep '^{' gpurun_out/final/bench_rccl2.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rccl2', d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/final/kt" -o run -- python3 "$R/bench.py" --steps 60 --warmup 5 > "$R/gpurun_out/final/kt_bench.txt" 2>&1 || { echo PROF FAILED; exit 1; }
cd "$R"
T=$(find gpurun_out/final/kt -name '*kernel_trace.csv' | head -1)
S=$(find gpurun_out/final/kt -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/final/kernel_stats.csv
python scripts/kt_timeline.py "$T" 40 43 > gpurun_out/final/kt_timeline.txt
rm -f "$T"
head -18 gpurun_out/final/kt_timeline.txt

# GPU tests first, then the headline bench under several settings (one JSON line each)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.txt 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/gputests.txt; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/gputests.txt
: > gpurun_out/sweep.jsonl
for s in "$@"; do
  timeout -k 10 300 python bench.py --steps 100 $s > gpurun_out/sweep_one.txt 2>&1 || { echo "BENCH FAILED: $s"; tail -20 gpurun_out/sweep_one.txt; exit 1; }
  echo "{\"args\": \"$s\", \"result\": $(tail -1 gpurun_out/sweep_one.txt)}" >> gpurun_out/sweep.jsonl
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep.jsonl').readlines()[-1]); print(d['args'], round(d['result']['ms_per_step'],3))"
done

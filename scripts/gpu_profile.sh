# bench + rocprofv3 kernel trace (CSV) of the headline config (SETS: extra bench args); summaries land in gpurun_out/
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/prof"
timeout -k 10 400 python bench.py $SETS > "$R/gpurun_out/bench.txt" 2>&1 || { echo BENCH FAILED; tail -20 "$R/gpurun_out/bench.txt"; exit 1; }
tail -1 "$R/gpurun_out/bench.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 40 --warmup 3 $SETS > "$R/gpurun_out/prof_bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/gpurun_out/prof_bench.txt"; exit 1; }
cd "$R"
T=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
S=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
echo "trace=$T stats=$S"
python scripts/rocprof_timeline.py "$T" --rounds 2 --skip 20 > gpurun_out/timeline.json
cp "$S" gpurun_out/kernel_stats.csv
rm -f "$T"
head -c 600 gpurun_out/timeline.json; echo
python - <<'PY'
import json; d = json.load(open("gpurun_out/timeline.json")); print("wall", d.get("mean_wall_us"), "busy", d.get("mean_busy_us"))
PY

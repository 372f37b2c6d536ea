# rocprofv3 kernel stats of one bench config: CONFIG (preset), SETS (--set args); summary -> gpurun_out/prof_<tag>/
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${TAG:-cfg}
mkdir -p "$R/gpurun_out/prof_$TAG"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --config ${CONFIG:-headline} --steps ${STEPS:-30} --warmup 3 $SETS > "$R/gpurun_out/prof_$TAG/bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/gpurun_out/prof_$TAG/bench.txt"; exit 1; }
cd "$R"
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/prof_$TAG/kernel_stats.csv
find gpurun_out/prof_$TAG -name '*kernel_trace.csv' -delete
head -12 gpurun_out/prof_$TAG/kernel_stats.csv | cut -d, -f1-6

# kernel -> (queue, stream) map of a short bench under rocprofv3 (hardware-queue sharing check)
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/qmap"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/qmap" -o run -- python3 "$R/bench.py" --steps 40 --warmup 3 $SETS > "$R/gpurun_out/qmap/bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/gpurun_out/qmap/bench.txt"; exit 1; }
cd "$R"
T=$(find gpurun_out/qmap -name '*kernel_trace.csv' | head -1)
python scripts/queue_map.py "$T" > gpurun_out/qmap/queue_map.json
find gpurun_out/qmap -name '*kernel_trace.csv' -delete
cat gpurun_out/qmap/queue_map.json

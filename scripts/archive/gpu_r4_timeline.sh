# Kernel-trace timeline of the headline bench (current tree): per-kernel stats + two rounds' device timelines
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; mkdir -p gpurun_out/kt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt" -o run -- python3 "$R/bench.py" --steps ${STEPS:-60} --warmup 5 > "$R/gpurun_out/kt_bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/gpurun_out/kt_bench.txt"; exit 1; }
cd "$R"
T=$(find gpurun_out/kt -name '*kernel_trace.csv' | head -1)
S=$(find gpurun_out/kt -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/kt_stats.csv
python scripts/kt_timeline.py "$T" ${A:-40} ${B:-43} > gpurun_out/kt_timeline.txt
rm -f "$T"
head -20 gpurun_out/kt_timeline.txt

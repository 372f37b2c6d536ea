# HIP runtime API calls of the headline round: per-call counts and host durations (rocprofv3 --hip-runtime-trace --stats)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5api; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --stats --output-format csv -d "$R/$O/api" -o run -- python3 "$R/bench.py" --steps 100 --warmup 10 \
  > "$R/$O/bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/$O/bench.txt"; exit 1; }
cd "$R"
S=$(find $O/api -name '*hip_api_stats.csv' | head -1)
cp "$S" $O/hip_api_stats.csv
head -40 $O/hip_api_stats.csv
rm -rf $O/api

# The round's side kernels timed alone (scripts/kernel_alone.py), under rocprofv3 kernel stats -> gpurun_out/r5alone/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5alone; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt" -o run -- python3 "$R/scripts/kernel_alone.py" --reps 20 \
  > "$R/$O/alone.txt" 2> "$R/$O/alone.err" || { echo "FAILED"; tail -20 "$R/$O/alone.err"; exit 1; }
cd "$R"
S=$(find $O/kt -name '*kernel_stats.csv' | head -1)
cp "$S" $O/kernel_stats_alone.csv
rm -rf $O/kt
cat $O/alone.txt
head -30 $O/kernel_stats_alone.csv | cut -d, -f1-4

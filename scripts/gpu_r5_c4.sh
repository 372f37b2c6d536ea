# Round-5 check 4: (1) the double-FMA Montgomery multiplier prototype (scripts/isa/fpmul_f64.hip) -- exact check
# of 2^20 pairs + throughput against the FIPS multiplier; (2) a 1-GPU kernel + HIP runtime trace of the headline
# bench: per-kernel stats, the round timeline and which API call queued each runtime blit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5c4; mkdir -p $O
timeout -k 10 120 ./scripts/isa/fpmul_f64 /tmp/fpmul_f64_check.bin > $O/fpmul_f64.jsonl 2>&1 || { echo "F64 BENCH FAILED"; cat $O/fpmul_f64.jsonl; exit 1; }
timeout -k 10 300 python scripts/isa/fpmul_f64_check.py /tmp/fpmul_f64_check.bin >> $O/fpmul_f64.jsonl || { echo "F64 CHECK FAILED"; exit 1; }
rm -f /tmp/fpmul_f64_check.bin
cat $O/fpmul_f64.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d "$R/$O/kt" -o run -- \
  python3 "$R/bench.py" --steps 60 --warmup 5 > "$R/$O/kt_bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/$O/kt_bench.txt"; exit 1; }
cd "$R"
T=$(find $O/kt -name '*kernel_trace.csv' | head -1)
H=$(find $O/kt -name '*hip_api_trace.csv' | head -1)
S=$(find $O/kt -name '*kernel_stats.csv' | head -1)
cp "$S" $O/kernel_stats.csv
python scripts/kt_timeline.py "$T" 40 43 > $O/kt_timeline.txt
python scripts/blit_attrib.py "$T" "$H" > $O/blits.json
gzip -c "$T" > $O/kernel_trace.csv.gz
rm -rf $O/kt
head -24 $O/kt_timeline.txt
head -40 $O/blits.json

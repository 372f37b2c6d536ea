# PMC counters of the share MSM (k_shares_msm) in isolation: scripts/bench_msm.py with the round's
# speculative row count.  Two passes (SQ issue/stall breakdown; HBM fetch + instruction mix), each
# its own rocprofv3 run under a hard time limit; summaries land in gpurun_out/pmc/.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ROWS=${ROWS:-62}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o p1 -- python3 "$R/scripts/bench_msm.py" --rows "$ROWS" --iters 3 > "$OUT/p1.txt" 2>&1 || { echo PASS1 FAILED; tail -5 "$OUT/p1.txt"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS GRBM_COUNT --output-format csv -d "$OUT/p2" -o p2 -- python3 "$R/scripts/bench_msm.py" --rows "$ROWS" --iters 3 > "$OUT/p2.txt" 2>&1 || { echo PASS2 FAILED; tail -5 "$OUT/p2.txt"; exit 1; }
cd "$R"
python3 scripts/pmc_summary.py gpurun_out/pmc k_shares_msm k_commit_rows > gpurun_out/pmc/summary.json && cat gpurun_out/pmc/summary.json

# Round-5 end: the full GPU test suite and smoke() on the final code, then the closing bench runs
# (scripts/gpu_r5_close.sh: driver-style x3, 200 rounds, emulated N = 2/4/8, 2-rank rehearsals, host timeline)
# and a kernel-stats profile of a driver-style run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5end; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.txt | tail -20; exit 1; }
echo "gpu tests: $(tail -1 $O/tests.txt)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 > $O/prof_bench.txt 2>&1 \
  || { echo "PROF FAILED"; tail -20 $O/prof_bench.txt; exit 1; }
echo "profiled: $(grep '^{' $O/prof_bench.txt | tail -1 | head -c 200)"
bash scripts/gpu_r5_close.sh

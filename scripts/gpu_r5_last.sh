# Round-5 last check on the committed tree: GPU tests, smoke, one driver-style bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5last; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.txt | tail -20; exit 1; }
echo "gpu tests: $(tail -1 $O/tests.txt)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench.txt 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench.txt; exit 1; }
grep '^{' $O/bench.txt | tail -1 | head -c 400

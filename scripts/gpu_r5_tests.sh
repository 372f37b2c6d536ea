# The whole GPU test suite on the working tree (one pytest process, per-test timeouts), then the poisoning guard's
# deterministic run printed (-s) for its ceiling.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 \
  || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error" $O/gputests.txt | tail -20; exit 1; }
echo "gpu tests passed: $(grep -c PASSED $O/gputests.txt)"

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.txt 2>&1 || { echo "GPU TESTS FAILED rc=$?"; tail -30 gpurun_out/gputests.txt; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.txt; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.txt; exit 1; }
tail -1 gpurun_out/bench.txt

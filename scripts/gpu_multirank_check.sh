# multi-rank GPU tests (chains equal the single-process chain) + the 2-rank RCCL shared-device rehearsal bench
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_multirank.txt 2>&1 || { echo MULTIRANK FAILED; tail -40 gpurun_out/pytest_multirank.txt; exit 1; }
tail -2 gpurun_out/pytest_multirank.txt
N=2 STEPS=60 bash scripts/gpu_rccl_bench.sh

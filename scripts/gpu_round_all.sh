# Round-end check on one MI355X: every GPU test, the smoke, the headline bench (SEEDS seeds) and a
# rocprofv3 kernel trace of it; summaries land in gpurun_out/
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/pytest_gpu.txt | head -20; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
SETS="--seeds ${SEEDS:-1}" bash scripts/gpu_profile.sh

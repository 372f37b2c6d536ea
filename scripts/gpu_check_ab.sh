# GPU tests of the engine/Krum paths, then A/B of engine settings (VARIANTS) and of the upload path
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ml.py tests/test_gpu_engine_paths.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ml.txt 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error|error|assert" gpurun_out/pytest_ml.txt | head -30; tail -30 gpurun_out/pytest_ml.txt; exit 1; }
tail -2 gpurun_out/pytest_ml.txt
VARIANTS="${VARIANTS:-none;none}" STEPS=200 bash scripts/gpu_ab_bench.sh
echo "--- BISCOTTI_H2D=torch"
BISCOTTI_H2D=torch VARIANTS="none" STEPS=200 bash scripts/gpu_ab_bench.sh

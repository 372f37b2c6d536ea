# GPU tests for the engine paths, then the same-box A/B of the working tree against exp/base.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_engine_paths.py tests/test_gpu_bn256.py tests/test_gpu_kzg.py} -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/iter_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/iter_tests.txt; exit 1; }
tail -1 gpurun_out/iter_tests.txt
bash scripts/gpu_ab_tree.sh

# A/B of the upload path (bare hipMemcpyAsync vs the framework's pinned copy), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
  echo "--- direct"; TAG=d$r VARIANTS="none" STEPS=200 bash scripts/gpu_ab_bench.sh || exit 1
  echo "--- torch"; BISCOTTI_H2D=torch TAG=t$r VARIANTS="none" STEPS=200 bash scripts/gpu_ab_bench.sh || exit 1
done

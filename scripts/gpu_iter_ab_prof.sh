# gpu_iter_ab.sh, then a kernel-trace profile of the working tree's driver-style bench (database output).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_iter_ab.sh || exit 1
rm -rf gpurun_out/prof_it
timeout -k 10 300 rocprofv3 --kernel-trace -d $PWD/gpurun_out/prof_it -o run -- python3 $PWD/bench.py --steps 20 --warmup 5 > gpurun_out/prof_it.txt 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/prof_it.txt; exit 1; }
echo prof done

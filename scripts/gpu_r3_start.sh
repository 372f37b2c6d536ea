# Session-start check: GPU tests, smoke, two driver-style benches, one long bench, and a kernel-trace
# profile of a driver-style bench.  Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=tests,smoke,short,long TAG=${TAG:-r3b} bash scripts/gpu_session.sh || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/short2_${TAG:-r3b}.txt 2>&1 || { echo "BENCH2 FAILED"; exit 1; }
grep '^{' gpurun_out/short2_${TAG:-r3b}.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('short2', round(d['ms_per_step'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG:-r3b} -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_${TAG:-r3b}.txt 2>&1 || { echo "PROF FAILED"; tail -20 gpurun_out/prof_${TAG:-r3b}.txt; exit 1; }
echo done

# Host-side diagnostics on the GPU: per-phase host timeline of steady-state rounds, a cProfile of a
# driver-style bench, and driver-style benches with the device VRF prover flushed every N rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/host_timeline.py --rounds 3 --warm 20 > gpurun_out/host_tl.json 2> gpurun_out/host_tl.err || { echo "TL FAILED"; tail -5 gpurun_out/host_tl.err; exit 1; }
timeout -k 10 200 python scripts/host_cprofile.py --steps 60 --warmup 5 > gpurun_out/cprof.txt 2>&1 || { echo "CPROF FAILED"; tail -5 gpurun_out/cprof.txt; exit 1; }
for rep in 1 2; do for vb in 16 2 1; do
  BISCOTTI_VRF_BATCH=$vb timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/vb_${vb}_$rep.txt 2>&1 || { echo "BENCH FAILED"; tail -5 gpurun_out/vb_${vb}_$rep.txt; exit 1; }
  grep '^{' gpurun_out/vb_${vb}_$rep.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('vrfbatch $vb rep $rep', round(d['ms_per_step'],3), 'drain', round(d['drain_ms'],2), 'walls', d['round_wall_ms'])"
done; done

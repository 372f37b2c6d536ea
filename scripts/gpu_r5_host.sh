# Host-side timeline of steady-state headline rounds (phases + the engine methods on the block -> next MSM path and
# the VRF jobs), and the double-FMA multiplier prototype's exact check with the corrected constants.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true \
  --wrap _early_vrf_submit,_spec_head_launch,_prepare_next_in_wait,_open_round,_select_noisers,_launch_krum,_resolve_evals,native.spec_msm,native.after_select,_finish_secagg,_secure_aggregation,_verification \
  > $O/host_tl.json 2> $O/host_tl.err || { echo "HOST TL FAILED"; tail -20 $O/host_tl.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5h/host_tl.json"))
for r in d[:2]:
    print("wall", r["wall_us"], r["jobs (kind, submit_us, queued_us, run_us)"])
    for n, s, dur in r["phases"]:
        print(f"  {n:32s} {s:9.1f} {dur:8.1f}")
PY

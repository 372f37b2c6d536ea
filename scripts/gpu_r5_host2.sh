# Host timeline of steady-state headline rounds with every native RoundFSM call timed (--fsm-proxy)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5h2; mkdir -p $O
timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true --fsm-proxy \
  --wrap _early_vrf_submit,_spec_head_launch,_open_round,_select_noisers,_launch_krum,native.spec_msm,native.after_select,_finish_secagg,_secure_aggregation,_round_front,_finish_verification,_noise_ids_np,_krum_static,_on_accept,_spec_aggregate_native,_vrf_key_rows,_resolve_evals,_prepare_next_in_wait \
  > $O/host_tl.json 2> $O/host_tl.err || { echo "HOST TL FAILED"; tail -20 $O/host_tl.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5h2/host_tl.json"))
for r in d[1:3]:
    print("wall", r["wall_us"])
    for n, s, dur in r["phases"]:
        print(f"  {n:34s} {s:8.1f} {dur:8.1f}")
PY

# One parametrised runner for the GPU box (replaces the per-round gpu_r*_*.sh one-offs).
#
#   gpurun --timeout 1200 -- bash scripts/gpu.sh OUT STEP [STEP ...]
#
# OUT is a directory under gpurun_out/; each STEP runs under its own time limit and the steps are chained: the
# first failure ends the call (no GPU step runs after a fault, an abort or a time limit).  Steps:
#   tests                 the GPU test suite (one pytest process, per-test timeouts)
#   test:EXPR             the GPU tests matching -k EXPR
#   smoke                 __graft_entry__.smoke()
#   b1xK                  K driver-style headline runs (bench.py --steps 20 --warmup 5)
#   long                  200 timed rounds
#   emuN[xK]              K driver-style runs of rank 0 of an N-rank job (bench.py --emulate-world N)
#   rehN[:ROUNDS]         an N-rank RCCL rehearsal, every rank on the one GPU (default 60 rounds)
#   cfg:NAME[:STEPS]      a bench preset (bench.py --config NAME)
#   bench:TAG:A+B+C       bench.py with arguments A B C ('+' separates them), output OUT/TAG.txt
#   set:K=V[,K=V][xK]     driver-style runs with --set K=V ... (A/B ablations)
#   seeds:NAME:N          bench.py --config NAME --seeds N (accuracy over seeds)
#   prof                  rocprofv3 --kernel-trace --stats of a driver-style run (OUT/prof/)
#   hosttl[:N|w:N]        the host timeline of 4 steady rounds (scripts/host_timeline.py; :N emulated rank 0 of N,
#                         w:N the same with 100 peers per rank)
#   mrprof:N              cProfile of rank 0 of an N-rank job (scripts/prof_rounds.py --emulate-world N)
#   kt:TAG:A+B+C          rocprofv3 kernel + memory-copy trace of bench.py A B C (OUT/kt_TAG/; scripts/kt_timeline.py)
#   ht:TAG:A+B+C          rocprofv3 HIP API + kernel trace of bench.py A B C (OUT/ht_TAG/; scripts/hip_api_costs.py)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"
O="gpurun_out/$1"; shift; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$R"

summ() {   # one line per bench JSON: mean, median, max, rounds over 3x the median, throttles, host CPU, drain
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
w = d.get('round_wall_ms') or [d['ms_per_step']]; med = sorted(w)[len(w) // 2]
pr = d.get('per_rank', [d]); p = d.get('phase_ms_per_round', {})
print(sys.argv[2], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', round(max(w), 3),
      '>3x', sum(x > 3 * med for x in w), 'acc', d.get('final_test_acc'), 'contrib', d.get('contributors_per_block'),
      'thr', [r.get('cgroup_cpu_stat_delta', {}).get('nr_throttled') for r in pr],
      'cpu', [round(r.get('host_cpu_ms_per_round', 0), 1) for r in pr],
      'coll_p50', [max([c.get('p50_ms') or 0 for c in r.get('collective_ms', {}).values()] or [0]) for r in pr],
      'rb', round(p.get('recover.readback', 0), 3), 'drain', round(d.get('drain_ms', 0), 2), flush=True)
PY
}
bench() {   # bench NAME TIMEOUT ARGS...  (a NAME already used in OUT gets a suffix: repeated steps keep every run)
  local n="$1" t="$2" k=2; shift 2
  if [[ -e "$O/$n.txt" ]]; then while [[ -e "$O/${n}_$k.txt" ]]; do k=$((k + 1)); done; n="${n}_$k"; fi
  timeout -k 10 "$t" python bench.py "$@" > "$O/$n.txt" 2>&1 || { echo "FAIL $n"; tail -20 "$O/$n.txt"; exit 1; }
  summ "$O/$n.txt" "$n"
}
reps() { local s="$1"; [[ "$s" == *x* ]] && echo "${s##*x}" || echo 1; }

for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/tests.txt" 2>&1 \
        || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error|assert" "$O/tests.txt" | tail -20; exit 1; }
      echo "gpu tests: $(tail -1 "$O/tests.txt")" ;;
    test:*)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread -k "${step#test:}" \
        > "$O/test_${step#test:}.txt" 2>&1 || { echo "GPU TEST FAILED"; tail -40 "$O/test_${step#test:}.txt"; exit 1; }
      echo "test ${step#test:}: $(tail -1 "$O/test_${step#test:}.txt")" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.txt" 2>&1 \
        || { echo "SMOKE FAILED"; tail -20 "$O/smoke.txt"; exit 1; }
      tail -1 "$O/smoke.txt" ;;
    b1*)
      for i in $(seq 1 "$(reps "$step")"); do bench "b1_s$i" 300 --steps 20 --warmup 5; done ;;
    long)
      bench b1_long 400 --steps 200 --warmup 10 ;;
    emu*)
      s="${step#emu}"; n="${s%%x*}"
      for i in $(seq 1 "$(reps "$step")"); do bench "emu${n}_s$i" 300 --emulate-world "$n" --steps 20 --warmup 5; done ;;
    reh*)
      s="${step#reh}"; n="${s%%:*}"; r=60; [[ "$s" == *:* ]] && r="${s#*:}"
      BISCOTTI_RCCL_SHARED_DEVICE=1 bench "reh${n}" 600 --gpus "$n" --steps "$r" --warmup 5 --set ablation=spec_head_shared ;;
    bench:*)
      s="${step#bench:}"; tag="${s%%:*}"; IFS='+' read -ra args <<< "${s#*:}"
      bench "$tag" 900 "${args[@]}" ;;
    cfg:*)
      s="${step#cfg:}"; name="${s%%:*}"; st=20; [[ "$s" == *:* ]] && st="${s#*:}"
      bench "cfg_$name" 900 --config "$name" --steps "$st" --warmup 5 ;;
    set:*)
      s="${step#set:}"; kv="${s%%x*}"; args=()
      IFS=',' read -ra kvs <<< "$kv"; for x in "${kvs[@]}"; do args+=(--set "$x"); done
      for i in $(seq 1 "$(reps "$step")"); do bench "set_${kv//[=,]/_}_s$i" 300 --steps 20 --warmup 5 "${args[@]}"; done ;;
    seeds:*)
      s="${step#seeds:}"; name="${s%%:*}"; k="${s#*:}"
      timeout -k 10 1100 python bench.py --config "$name" --seeds "$k" > "$O/seeds_$name.txt" 2>&1 \
        || { echo "FAIL seeds $name"; tail -20 "$O/seeds_$name.txt"; exit 1; }
      grep '^{' "$O/seeds_$name.txt" | tail -1 | head -c 600; echo ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python bench.py --steps 20 --warmup 5 \
        > "$O/prof_bench.txt" 2>&1 || { echo "PROF FAILED"; tail -20 "$O/prof_bench.txt"; exit 1; }
      echo "profiled: $(grep '^{' "$O/prof_bench.txt" | tail -1 | head -c 160)" ;;
    hosttl*)
      e="${step#hosttl}"; ea=(); [[ -n "$e" ]] && ea=(--emulate-world "${e#:}")
      # hosttlw:N -- weak scaling: 100 peers per emulated rank (bench.py's scale_weak)
      [[ "$e" == w:* ]] && { e="${e#w}"; ea=(--emulate-world "${e#:}" --set "num_nodes=$((100 * ${e#:}))"); e="w${e#:}"; }
      timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true "${ea[@]}" \
        --wrap _early_vrf_submit,_spec_head_launch,_spec_front_launch,_adopt_spec_front,_prepare_next_in_wait,_open_round,_select_noisers,_launch_krum,native.spec_msm,native.after_select,native.agg_multi,_gather_verify_inputs,_finish_secagg,_secure_aggregation,_round_front,_finish_verification \
        > "$O/host_tl${e#:}.json" \
        2> "$O/host_tl${e#:}.err" || { echo "HOST TL FAILED"; tail -20 "$O/host_tl${e#:}.err"; exit 1; }
      echo "host timeline: $O/host_tl${e#:}.json" ;;
    mrprof:*)
      n="${step#mrprof:}"
      timeout -k 10 300 python scripts/prof_rounds.py --emulate-world "$n" -o "$O/mrprof_${n}_full.txt" > "$O/mrprof_$n.txt" 2>&1 \
        || { echo "MRPROF FAILED"; tail -20 "$O/mrprof_$n.txt"; exit 1; }
      head -40 "$O/mrprof_$n.txt" ;;
    kt:*)
      s="${step#kt:}"; tag="${s%%:*}"; IFS='+' read -ra args <<< "${s#*:}"
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/kt_$tag" -o run -- python bench.py "${args[@]}" \
        > "$O/kt_$tag.txt" 2>&1 || { echo "KT FAILED"; tail -20 "$O/kt_$tag.txt"; exit 1; }
      summ "$O/kt_$tag.txt" "kt_$tag"
      # the timeline as text (the trace database is tens of MB: gpurun copies back at most 64 MiB)
      python scripts/kt_timeline.py "$(ls "$O"/kt_$tag/*.db | head -1)" 30 34 > "$O/kt_${tag}_timeline.txt" 2>&1 || true
      rm -rf "$O/kt_$tag" ;;
    ht:*)
      s="${step#ht:}"; tag="${s%%:*}"; IFS='+' read -ra args <<< "${s#*:}"
      timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d "$O/ht_$tag" -o run -- python bench.py "${args[@]}" \
        > "$O/ht_$tag.txt" 2>&1 || { echo "HT FAILED"; tail -20 "$O/ht_$tag.txt"; exit 1; }
      summ "$O/ht_$tag.txt" "ht_$tag"
      python scripts/hip_api_costs.py "$(ls "$O"/ht_$tag/*.db | head -1)" > "$O/ht_${tag}_api.txt" 2>&1 || true
      python scripts/kt_timeline.py "$(ls "$O"/ht_$tag/*.db | head -1)" 30 34 > "$O/ht_${tag}_timeline.txt" 2>&1 || true
      python scripts/launch_gap.py "$(ls "$O"/ht_$tag/*.db | head -1)" > "$O/ht_${tag}_launch.txt" 2>&1 || true
      rm -rf "$O/ht_$tag" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done

#!/usr/bin/env bash
# DistSys/localTest.sh equivalent: generate keys, launch N peer processes on 127.0.0.1:8000+i,
# wait, and check that every peer printed a byte-identical chain.
#   scripts/local_test.sh [N=4] [dataset=creditcard] [rounds=5]
set -euo pipefail
N=${1:-4}
DS=${2:-creditcard}
ROUNDS=${3:-5}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WORK=$(mktemp -d)
DIMS=$([ "$DS" = "mnist" ] && echo 7850 || echo 25)
python -m biscotti_amd.keygen -n "$N" -d "$DIMS" -o "$WORK" > /dev/null
mkdir -p "$WORK/LogFiles"
for ((i = 0; i < N; i++)); do
  (cd "$ROOT" && python -m biscotti_amd.peer -i="$i" -t="$N" -d="$DS" -na=1 -nv=1 -nn=1 \
      --device cpu --rounds "$ROUNDS" --print-chain all --deterministic-time \
      --commit-key "$WORK/commitKey.json" --pkey-file "$WORK/pKeyG1.json" \
      > "$WORK/LogFiles/test1_${i}_${N}.log" 2> "$WORK/LogFiles/log_${i}_${N}.log") &
done
wait
cd "$WORK/LogFiles"
for ((i = 0; i < N; i++)); do grep -v '^\[Gloo\]' "test1_${i}_${N}.log" > "chain_${i}.txt"; done
for ((i = 1; i < N; i++)); do
  if ! cmp -s chain_0.txt "chain_${i}.txt"; then
    echo "FAILURE: peer $i holds a different chain (logs in $WORK/LogFiles)"
    exit 1
  fi
done
echo "SUCCESS! Nodes have same blockchain ($N peers, $(grep -c 'Hash: ' chain_0.txt) blocks)"
rm -rf "$WORK"

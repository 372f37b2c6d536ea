# Build a copy of commit ${1:-HEAD~1}'s package, bench.py and scripts/ with its own native libraries in
# ${2:-ab_base}/, for same-box A/B runs (scripts/gpu_ab_tree.sh, poisoning comparisons across commits).
set -e
REV=${1:-HEAD~1}
DIR=${2:-ab_base}
rm -rf "$DIR" && mkdir -p "$DIR"
git archive "$REV" biscotti_amd bench.py scripts | tar -x -C "$DIR"
rm -rf "$DIR/biscotti_amd/data/files/creditcard.csv"
(cd "$DIR" && python -m biscotti_amd._build > /dev/null)
ls "$DIR"/biscotti_amd/*.so

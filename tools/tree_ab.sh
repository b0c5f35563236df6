#!/bin/bash
# A/B of the working tree against a second checkout (abtree/, e.g. a git
# worktree of HEAD built in place): step and kernel times of cfg2 and cfg4,
# alternating.  Usage: tools/tree_ab.sh [reps]
set -uo pipefail
OUT=gpurun_out/tree_ab.txt
REPS=${1:-2}
: > "$OUT"
run() {
  local label=$1 dir=$2 n=$3 steps=$4
  local line
  line=$(cd "$dir" && timeout -k 10 150 python3 bench.py --samples $n --features $n --steps $steps --warmup 3 \
           --no-fit --no-cpu-baseline 2>/dev/null) || { echo "$label FAILED" >> "$OUT"; return 1; }
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in r['kernel_ms'].items()})" "$label" "$line" >> "$OUT"
}
for rep in $(seq $REPS); do
  run cfg2_new . 5000 20 && run cfg2_old abtree 5000 20 || exit 1
done
for rep in $(seq $REPS); do
  run cfg4_new . 20000 5 && run cfg4_old abtree 20000 5 || exit 1
done
cat "$OUT"

#!/bin/bash
# Mean correction (k_colrank + k_rowcorr) beside k_dist or before it
# (FS_SIDE), working tree against abtree/, cfg4 and cfg2, alternating.
set -uo pipefail
OUT=gpurun_out/side_ab.txt
: > "$OUT"
run() {
  local label=$1 dir=$2 n=$3 steps=$4; shift 4
  local line
  line=$(cd "$dir" && env "$@" timeout -k 10 150 python3 bench.py --samples $n --features $n --steps $steps \
           --warmup 3 --no-fit --no-cpu-baseline 2>/dev/null) || { echo "$label FAILED" >> "$OUT"; return 1; }
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in r['kernel_ms'].items()})" "$label" "$line" >> "$OUT"
}
for rep in 1 2; do
  run cfg4_new_side1 . 20000 5 FS_NOOP=1 && run cfg4_new_side0 . 20000 5 FS_SIDE=0 \
    && run cfg4_old_side1 abtree 20000 5 FS_NOOP=1 || exit 1
done
for rep in 1 2; do
  run cfg2_new_side1 . 5000 20 FS_NOOP=1 && run cfg2_new_side0 . 5000 20 FS_SIDE=0 \
    && run cfg2_old_side1 abtree 5000 20 FS_NOOP=1 || exit 1
done
cat "$OUT"

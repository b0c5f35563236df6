#!/bin/bash
# Tail K-split of pass 1 (automatic) against no split (FS_KSPLIT=1), cfg2 and
# cfg4 step times and kernel times, alternating twice.
set -uo pipefail
OUT=gpurun_out/ksplit_tail_ab.txt
: > "$OUT"
run() {
  local label=$1 n=$2 steps=$3; shift 3
  local line
  line=$(env "$@" timeout -k 10 150 python3 bench.py --samples $n --features $n --steps $steps --warmup 3 \
           --no-fit --no-cpu-baseline 2>/dev/null) || { echo "$label FAILED" >> "$OUT"; return 1; }
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in r['kernel_ms'].items()})" "$label" "$line" >> "$OUT"
}
for rep in 1 2; do
  run cfg2_tail 5000 20 FS_NOOP=1 && run cfg2_nosplit 5000 20 FS_KSPLIT=1 || exit 1
done
for rep in 1 2; do
  run cfg4_tail 20000 5 FS_NOOP=1 && run cfg4_nosplit 20000 5 FS_KSPLIT=1 || exit 1
done
cat "$OUT"

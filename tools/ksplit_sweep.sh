#!/bin/bash
# Pass-1 K-split choices at cfg2 (and cfg4): automatic vs FS_KSPLIT=s
# (every tile split into s parts), step and kernel times.
set -uo pipefail
OUT=gpurun_out/ksplit_sweep.txt
: > "$OUT"
run() {
  local label=$1 n=$2 steps=$3; shift 3
  local line
  line=$(env "$@" timeout -k 10 150 python3 bench.py --samples $n --features $n --steps $steps --warmup 3 \
           --no-fit --no-cpu-baseline 2>/dev/null) || { echo "$label FAILED" >> "$OUT"; return 1; }
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in r['kernel_ms'].items()})" "$label" "$line" >> "$OUT"
}
for rep in 1 2; do
  run cfg2_auto 5000 20 FS_NOOP=1 || exit 1
  for s in 1 4 6 8; do run cfg2_s$s 5000 20 FS_KSPLIT=$s || exit 1; done
done
run cfg4_auto 20000 5 FS_NOOP=1 || exit 1
run cfg4_auto 20000 5 FS_NOOP=1 || exit 1
cat "$OUT"

#!/bin/bash
# cfg2 (MultiSURF 5000 x 5000) step time under pass-2 grid sizes and pass-1
# K-split choices (fill the chip at small sizes).
set -uo pipefail
OUT=gpurun_out/cfg2_sweep.txt
: > "$OUT"
run() {
  local label=$1; shift
  local line
  line=$(env "$@" timeout -k 10 120 python3 bench.py --samples 5000 --features 5000 --steps 20 --warmup 3 \
           --no-fit --no-cpu-baseline 2>/dev/null) || { echo "$label FAILED" >> "$OUT"; return 1; }
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in r['kernel_ms'].items()})" "$label" "$line" >> "$OUT"
}
run default FS_NOOP=1
for s in 1 2 4; do run ksplit$s FS_KSPLIT=$s; done
cat "$OUT"

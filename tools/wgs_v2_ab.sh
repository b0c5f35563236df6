#!/bin/bash
# Pass-2 workgroup count (segment length) A/B for the v2 sparse kernel.
set -euo pipefail
OUT=gpurun_out/wgs_v2
mkdir -p "$OUT"
for round in 1 2; do
  for w in 32768 16384 65536 131072; do
    FS_PASS2_WGS=$w timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-fit > "$OUT/$w.$round.json" 2> "$OUT/$w.$round.err"
    python3 -c "import json; d=json.loads(open('$OUT/$w.$round.json').read().strip().splitlines()[-1]); print('$w', $round, round(d['ms_per_step'],2), {k: round(x,2) for k,x in d['roofline']['kernel_ms'].items()})"
  done
done

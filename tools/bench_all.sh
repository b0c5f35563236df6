#!/bin/bash
# Every BASELINE config through bench.py on one GPU (round 3), one JSON line
# each under gpurun_out/$1/.
set -euo pipefail
OUT=gpurun_out/${1:-r03_configs}
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py > "$OUT/cfg4.json" 2> "$OUT/cfg4.err"
for c in cfg2 cfg3 cfg5s cfg5m; do
  timeout -k 10 300 python3 bench.py --config $c --no-fit > "$OUT/$c.json" 2> "$OUT/$c.err"
done

#!/bin/bash
# fit() of cfg4 from float64 and from float32 X: working tree against abtree/,
# alternating (tools/fit_time.py prints one JSON line per run).
set -uo pipefail
OUT=gpurun_out/fit_ab.txt
: > "$OUT"
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=abtree
    line=$(cd $d && timeout -k 10 300 python3 "$OLDPWD/tools/fit_time.py" 2>/dev/null) || exit 1
    echo "$t $line" >> "$OUT"
  done
done
cat "$OUT"

#!/bin/bash
# Diagnostic: k_score_sparse with half the LDS bytes per entry (ds_read_b64,
# wrong scores) against the shipped loop, alternating -- is the loop bound by
# the LDS traffic of the row reads?
set -uo pipefail
OUT=gpurun_out/half_lds_ab.txt
: > "$OUT"
for r in 1 2; do
  for w in 1 2; do
    line=$(FS_SPARSE_JIT=$w timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fit 2>/dev/null) || { echo "jit=$w FAILED" >> "$OUT"; cat "$OUT"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('variant', sys.argv[1], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['roofline']['kernel_ms'].items()})" "$w" "$line" >> "$OUT"
  done
done
cat "$OUT"

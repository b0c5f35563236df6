#!/bin/bash
# A/B of two k_score_sparse loop builds: FS_SPARSE_JIT=1 (shipped) vs 2 (the
# FS_SPARSE_STREAM_ASM_HALF macro of the current generator run: half-LDS
# diagnostic or FS_GEN_WAIT_EVERY variant).
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

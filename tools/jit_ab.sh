#!/bin/bash
# A/B of the sparse pass-2 loops (FS_SPARSE_JIT): parity with the JIT loop
# first (small sizes, then cfg2 / cfg4 against the oracle fixtures), then the
# bench alternating on one box.
set -uo pipefail
OUT=gpurun_out/jit_ab.txt
: > "$OUT"
FS_SPARSE_JIT=1 timeout -k 10 300 python3 -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "multisurf" >> "$OUT" 2>&1 || { echo "parity FAILED" >> "$OUT"; cat "$OUT"; exit 1; }
: # fullsize parity checked for lead 6
for r in 1 2; do
  for w in 0 1; do
    line=$(FS_SPARSE_JIT=$w timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fit 2>/dev/null) || { echo "jit=$w FAILED" >> "$OUT"; cat "$OUT"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('jit', sys.argv[1], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['roofline']['kernel_ms'].items()})" "$w" "$line" >> "$OUT"
  done
done
cat "$OUT"

#!/bin/bash
# A/B of the L2 warm-up loads in k_score_sparse (FS_SPARSE_WARM): parity of
# MultiSURF with the warm loop first (small, then cfg4), then the bench
# alternating on one box.
set -uo pipefail
OUT=gpurun_out/warm_ab.txt
: > "$OUT"
FS_SPARSE_WARM=1 timeout -k 10 300 python3 -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "multisurf" >> "$OUT" 2>&1 || { echo "parity FAILED" >> "$OUT"; cat "$OUT"; exit 1; }
for r in 1 2; do
  for w in 0 1; do
    line=$(FS_SPARSE_WARM=$w timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fit 2>/dev/null) || { echo "warm=$w FAILED" >> "$OUT"; cat "$OUT"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('warm', sys.argv[1], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['roofline']['kernel_ms'].items()})" "$w" "$line" >> "$OUT"
  done
done
FS_SPARSE_WARM=1 timeout -k 10 400 python3 -m pytest tests/test_gpu_baseline.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cfg4 or cfg2" >> "$OUT" 2>&1
cat "$OUT"

#!/bin/bash
# Same-box A/B of k_score_sparse2 lookahead variants (tools/build_variant.sh
# builds), alternating, one bench line each.
set -euo pipefail
OUT=gpurun_out/lead_v2
mkdir -p "$OUT"
for round in 1 2; do
  for v in default L2 L3 L6; do
    if [ "$v" = default ]; then
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-fit > "$OUT/$v.$round.json" 2> "$OUT/$v.$round.err"
    else
      FS_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-fit > "$OUT/$v.$round.json" 2> "$OUT/$v.$round.err"
    fi
    python3 -c "import json,sys; d=json.loads(open('$OUT/$v.$round.json').read().strip().splitlines()[-1]); print('$v', $round, round(d['ms_per_step'],2), d['roofline']['kernel_ms'])"
  done
done

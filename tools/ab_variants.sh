#!/bin/bash
# Same-box A/B of library variants (tools/build_variant.sh builds; "default"
# = the in-tree library), alternating over rounds, one bench line each.
#   tools/ab_variants.sh <tag> <rounds> <variant>... [-- extra bench args]
set -euo pipefail
TAG=$1; ROUNDS=$2; shift 2
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
EXTRA="$*"
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
for round in $(seq 1 "$ROUNDS"); do
  for v in "${VARS[@]}"; do
    if [ "$v" = default ]; then unset FS_LIB_VARIANT; else export FS_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-fit $EXTRA > "$OUT/$v.$round.json" 2> "$OUT/$v.$round.err"
    python3 -c "import json,sys; d=json.loads(open('$OUT/$v.$round.json').read().strip().splitlines()[-1]); print('$v', $round, round(d['ms_per_step'],2), {k: round(x, 2) for k, x in d['roofline']['kernel_ms'].items()})"
  done
done
unset FS_LIB_VARIANT

#!/bin/bash
# L2 / fabric counters of the pass-2 kernels for a library variant:
#   pass fetch: FETCH_SIZE (3 TCC slots) + TCC_HIT_sum
#   pass miss : TCC_MISS_sum, TCC_REQ_sum
# $1 = tag, $2 = FS_LIB_VARIANT (or "default"), $3 = extra env (e.g. FS_SPARSE_V=1)
set -euo pipefail
TAG=$1; VAR=${2:-default}; EXTRA=${3:-}
OUT=gpurun_out/pmc_l2_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$VAR" != default ]; then export FS_LIB_VARIANT=$VAR; fi
if [ -n "$EXTRA" ]; then export "$EXTRA"; fi
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-fit"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -f csv -d "$OUT/fetch" -o run -- \
    python3 bench.py $ARGS > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -s KILL 150 rocprofv3 --pmc TCC_MISS_sum TCC_REQ_sum -f csv -d "$OUT/miss" -o run -- \
    python3 bench.py $ARGS > "$OUT/miss.json" 2> "$OUT/miss.err"
python3 tools/pmc_table.py "$OUT" > "$OUT/table.txt"

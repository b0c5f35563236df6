#!/bin/bash
# SQ stall / issue, LDS and clock counters of the pass-2 kernels (round 3:
# k_score_sparse2 vs k_score_sparse).  One PMC pass per group (<= 8 SQ,
# <= 2 GRBM counters), kernel-trace only.  $1 = tag, $2 = extra bench args.
set -euo pipefail
TAG=${1:-v2}
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-fit ${2:-}"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d "$OUT/sq" -o run -- \
    python3 bench.py $ARGS > "$OUT/sq.json" 2> "$OUT/sq.err"
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES -f csv -d "$OUT/lds" -o run -- \
    python3 bench.py $ARGS > "$OUT/lds.json" 2> "$OUT/lds.err"
python3 tools/pmc_table.py "$OUT" > "$OUT/table.txt"

#!/bin/bash
# LDS and scalar-cache counters of the bench kernels (name the
# binding wait of k_score_sparse).  Two PMC passes (8 SQ counters at most
# each), kernel-trace only; tools/pmc_table.py prints per-kernel averages.
#   pass lds : LDS instructions, bank conflicts, LDS-busy cycles, LDS issue
#              stalls, scalar-cache hits / misses, SMEM cycles
#   pass lvl : in-flight levels of LDS / SMEM instructions (level / insts =
#              average latency in cycles)
set -euo pipefail
TAG=${1:-lds}
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-fit ${2:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INST_CYCLES_SMEM SQ_WAVE_CYCLES -f csv -d "$OUT/lds" -o run -- \
    python3 bench.py $ARGS > "$OUT/lds.json" 2> "$OUT/lds.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES -f csv -d "$OUT/lvl" -o run -- \
    python3 bench.py $ARGS > "$OUT/lvl.json" 2> "$OUT/lvl.err"
python3 tools/pmc_table.py "$OUT" > "$OUT/table.txt"

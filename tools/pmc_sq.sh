#!/bin/bash
# SQ occupancy/stall counters + GRBM clock for the bench kernels (one PMC pass
# per counter group, kernel-trace only; see the gpurun rules).
set -euo pipefail
TAG=${1:-sq}
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d "$OUT/sq" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${2:-} > "$OUT/sq.json" 2> "$OUT/sq.err"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES -f csv -d "$OUT/grbm" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${2:-} > "$OUT/grbm.json" 2> "$OUT/grbm.err"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS -f csv -d "$OUT/lds" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${2:-} > "$OUT/lds.json" 2> "$OUT/lds.err"
python3 tools/pmc_table.py "$OUT" | tee "$OUT/table.txt"

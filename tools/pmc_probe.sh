#!/bin/bash
# Kernel trace + SQ / GRBM / LDS counter passes over any python command (one
# PMC pass per counter group, kernel-trace only; see the gpurun rules):
#   bash tools/pmc_probe.sh <tag> tools/chains_probe.py --n 8192 --p 8192
set -euo pipefail
TAG=$1
shift
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 "$@" > "$OUT/trace.out" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d "$OUT/sq" -o run -- \
    python3 "$@" > "$OUT/sq.out" 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES -f csv -d "$OUT/grbm" -o run -- \
    python3 "$@" > "$OUT/grbm.out" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS -f csv -d "$OUT/lds" -o run -- \
    python3 "$@" > "$OUT/lds.out" 2>&1
python3 tools/pmc_table.py "$OUT" > "$OUT/table.txt"

#!/bin/bash
# PMC passes over the mean-correction kernels (tools/colsort_bench.py)
out=$GRAFT_REPO_ROOT/gpurun_out/r04e
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/tools/colsort_bench.py 20000 2048 2 gauss"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o run -- $B > "$out/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -f csv -d "$out/pmc1" -o run -- $B > "$out/pmc1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -f csv -d "$out/pmc2" -o run -- $B > "$out/pmc2.log" 2>&1 || exit $?
echo ok

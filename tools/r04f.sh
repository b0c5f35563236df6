#!/bin/bash
# Mean-correction check: the GPU mean-correction / family tests, the default
# bench with a kernel trace (tools/r04_check.sh), then one PMC pass over the
# mean-correction kernels alone (tools/colsort_bench.py, dispatches
# serialised by the profiler: GRBM_GUI_ACTIVE is the standalone time).
tag=${1:-r04f}
bash tools/r04_check.sh "$tag" tests/test_gpu_meancorr.py tests/test_gpu_families.py || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/tools/colsort_bench.py 20000 2048 2 gauss"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d "$out/pmc1" -o run -- $B > "$out/pmc1.log" 2>&1 || exit $?

cd "$GRAFT_REPO_ROOT" || exit 1
FAM=uniform_16k,lognormal_16k,mixed_16k timeout -k 10 600 python -u tools/family_diag.py > "$out/families.txt" 2>&1 || exit $?
cat "$out/families.txt"

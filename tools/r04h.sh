#!/bin/bash
# Round-4 diagnostics on one MI355X (results under gpurun_out/r04h/):
#  1. cfg2 bench line + rocprofv3 kernel trace
#  2. pair-weight density per tile at cfg4 (next #4: dense/sparse split?)
#  3. devices= phase log at cfg4 (next #5: X over the host link once)
#  4. mean-correction kernels standalone, one PMC pass (next #7)
out=$GRAFT_REPO_ROOT/gpurun_out/r04h
mkdir -p "$out"
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 20 --warmup 3 --no-fit \
  > "$out/cfg2_bench.json" 2> "$out/cfg2_bench.err" || exit $?
cat "$out/cfg2_bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$out/cfg2_prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-fit \
  > "$out/cfg2_prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python3 -u tools/tile_density.py 20000 20000 12 > "$out/tile_density.json" 2> "$out/tile_density.err" || exit $?
cat "$out/tile_density.json"
timeout -k 10 600 python3 -u tools/devices_trace.py > "$out/devices_trace.txt" 2>&1 || exit $?
tail -3 "$out/devices_trace.txt"
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/tools/colsort_bench.py 20000 2048 2 gauss"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$out/colsort_trace" -o run -- $B > "$out/colsort_trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d "$out/colsort_pmc1" -o run -- $B > "$out/colsort_pmc1.log" 2>&1 || exit $?
echo r04h done

#!/bin/bash
# Round-4 check after the tiled exact-row kernel: the parity tests it
# touches, cfg2 bench + kernel trace, and the mean correction alone
# (mcmain variant: on the main stream, so the trace shows its own time) with
# one SQ counter pass.
out=gpurun_out/r04m
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_exact_thresholds.py tests/test_gpu_families.py tests/test_gpu_meancorr.py \
  tests/test_gpu_dist.py tests/test_gpu_baseline.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/tests.log"; tail -4 "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 20 --warmup 3 --no-fit \
  > "$out/cfg2_bench.json" 2> "$out/cfg2_bench.err" || exit $?
python3 -c "import json; d=json.load(open('$out/cfg2_bench.json')); print('cfg2', d['ms_per_step'], d['roofline']['kernel_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/cfg2_prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-fit \
  > "$GRAFT_REPO_ROOT/$out/cfg2_prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
lib=fastselect_amd/libfastselect_amd.so
cp $lib "$out/.product.so" && cp fastselect_amd/libfastselect_amd_mcmain.so $lib || exit 1
cd /tmp
B="python3 $GRAFT_REPO_ROOT/tools/colsort_bench.py 20000 2048 2 gauss"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/colsort_trace" -o run -- $B > "$GRAFT_REPO_ROOT/$out/colsort_trace.log" 2>&1
r1=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -f csv -d "$GRAFT_REPO_ROOT/$out/colsort_pmc1" -o run -- $B > "$GRAFT_REPO_ROOT/$out/colsort_pmc1.log" 2>&1
r2=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_INSTS_VMEM -f csv -d "$GRAFT_REPO_ROOT/$out/colsort_pmc2" -o run -- $B > "$GRAFT_REPO_ROOT/$out/colsort_pmc2.log" 2>&1
r3=$?
cd "$GRAFT_REPO_ROOT" && cp "$out/.product.so" $lib && rm -f "$out/.product.so"
echo "colsort rc $r1 $r2 $r3"

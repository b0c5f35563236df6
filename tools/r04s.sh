#!/bin/bash
# k_colsort on 8192 bins (colsort_bin_bits) vs 4096 (FS_COLSORT_BINS12=1):
# the mean-correction tests, then cfg4 bench lines alternating the two and a
# kernel trace of each.
out=gpurun_out/r04s
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_meancorr.py tests/test_exact_thresholds.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/tests.log"; tail -3 "$out/tests.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 13 12 13 12; do
  if [ $v = 12 ]; then export FS_COLSORT_BINS12=1; else unset FS_COLSORT_BINS12; fi
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fit \
    > "$out/bench_$v.json" 2> "$out/bench_$v.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/bench_$v.json')); print('bins$v', round(d['ms_per_step'],3))" | tee -a "$out/ab.txt"
done
cd /tmp && export TMPDIR=/tmp
for v in 13 12; do
  if [ $v = 12 ]; then export FS_COLSORT_BINS12=1; else unset FS_COLSORT_BINS12; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/prof$v" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-q32 --no-fit \
    > "$GRAFT_REPO_ROOT/$out/prof$v.log" 2>&1 || exit $?
done
cd "$GRAFT_REPO_ROOT" || exit 1
unset FS_COLSORT_BINS12
timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 20 --warmup 3 --no-fit \
  > "$out/cfg2_bench.json" 2> "$out/cfg2_bench.err" || exit $?
python3 -c "import json; d=json.load(open('$out/cfg2_bench.json')); print('cfg2', d['ms_per_step'], d['roofline']['kernel_ms'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/cfg2_prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-fit \
  > "$GRAFT_REPO_ROOT/$out/cfg2_prof.log" 2>&1 || exit $?

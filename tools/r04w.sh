#!/bin/bash
# k_rowcorr over column slices: the mean-correction and MultiSURF parity
# tests, cfg2 and cfg4 bench lines and a cfg2 kernel trace.
out=gpurun_out/r04w
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_meancorr.py tests/test_exact_thresholds.py tests/test_gpu_families.py \
  tests/test_gpu_baseline.py tests/test_gpu_dist.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/tests.log"; tail -3 "$out/tests.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for c in cfg2 cfg4 cfg2 cfg4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-fit \
    > "$out/$c.json" 2> "$out/$c.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/$c.json')); print('$c', round(d['ms_per_step'],3), {k: round(v,2) for k,v in d['roofline']['kernel_ms'].items()})" | tee -a "$out/bench.txt"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/cfg2_prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-fit \
  > "$GRAFT_REPO_ROOT/$out/cfg2_prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
# A/B: short-column k_colsort at two workgroups per CU (<= 64 VGPRs)
bash tools/variant_ab.sh r04w_cswpe8 2 default cswpe8 -- --config cfg2

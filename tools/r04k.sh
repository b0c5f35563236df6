#!/bin/bash
# Decision flips on the families (tools/flip_diag.py) per operand width, the
# two GPU tests that failed in r04j, then an A/B of the pass-2 library
# variants.
out=gpurun_out/r04k
mkdir -p "$out"
for fam in lognormal_16k uniform_16k; do
  for mode in default q16; do
    FS_TRACE=1 timeout -k 10 240 python3 -u tools/flip_diag.py $fam $mode > "$out/flip_${fam}_$mode.json" 2> "$out/flip_${fam}_$mode.err" || exit $?
    cat "$out/flip_${fam}_$mode.json"; grep "exact thresholds\|too many" "$out/flip_${fam}_$mode.err" | head -3
  done
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_meancorr.py tests/test_gpu_families.py tests/test_exact_thresholds.py -m gpu \
  > "$out/tests.log" 2>&1
rc=$?; tail -3 "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/variant_ab.sh r04k_ab 2 default prio old || exit $?
bash tools/sp2_prof.sh r04k_sp2 prioprof || exit $?
bash tools/sp2_prof.sh r04k_sp2 sp2prof2 || exit $?

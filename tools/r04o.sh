#!/bin/bash
# exact-threshold kernel (16-sample chunks) re-checked, then pass-2 segment
# length A/B at cfg2 and cfg4
out=gpurun_out/r04o
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_exact_thresholds.py tests/test_gpu_families.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/tests.log"; tail -3 "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/variant_ab.sh r04o_ab_cfg2 2 default segmul2 segmul4 -- --config cfg2 || exit $?
bash tools/variant_ab.sh r04o_ab_cfg4 1 default segmul2 || exit $?

#!/bin/bash
# Segment-walk variant (FS_SP2_SEG): parity with the variant swapped in, then
# an A/B against the product at cfg4 and cfg2.
out=gpurun_out/r04p
mkdir -p "$out"
lib=fastselect_amd/libfastselect_amd.so
cp $lib "$out/.product.so" && cp fastselect_amd/libfastselect_amd_seg.so $lib || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_baseline.py tests/test_gpu.py tests/test_exact_thresholds.py -m gpu > "$out/tests_seg.log" 2>&1
rc=$?
cp "$out/.product.so" $lib && rm -f "$out/.product.so"
echo "pytest (seg variant) rc=$rc" >> "$out/tests_seg.log"; tail -3 "$out/tests_seg.log"
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/variant_ab.sh r04p_ab 2 default seg || exit $?
bash tools/variant_ab.sh r04p_ab2 1 default seg -- --config cfg2 || exit $?

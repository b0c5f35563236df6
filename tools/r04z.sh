#!/bin/bash
# The mean-correction agreement tests, bin-bit edge cases included.
out=gpurun_out/r04z
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_meancorr.py -m gpu -k "corrections_agree" > "$out/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/tests.log"; tail -14 "$out/tests.log"
exit $rc

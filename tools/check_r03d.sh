#!/bin/bash
# The 16-bit decision check at cfg4 / cfg2, data-family parity on the default
# path, then the whole GPU suite (run via gpurun).
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r03d}
mkdir -p $out
PYTHONPATH=. timeout -k 10 300 python3 -u tools/guard_probe.py > $out/guard_probe.txt 2>&1
timeout -k 10 400 python3 -u -m pytest -v -rxs --timeout 250 --timeout-method thread -m gpu tests/test_gpu_families.py > $out/families.txt 2>&1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests > $out/gpu_tests.txt 2>&1
echo done

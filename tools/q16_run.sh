#!/bin/bash
# GPU suite (incl. the 16-bit pass-1 tests) + a kernel trace of the bench.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -m pytest tests -m gpu -q -x > gpurun_out/q16_tests.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_q16/trace -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/q16_bench.json 2> gpurun_out/q16_bench.err

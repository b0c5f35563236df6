#!/bin/bash
# End-of-round-3 kernel traces (run via gpurun) of the shipped tree: cfg4
# (default bench line), cfg3 and cfg2, rocprofv3 --kernel-trace --stats each.
set -euo pipefail
export TMPDIR=/tmp
for c in cfg4 cfg3 cfg2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03c_$c/trace -o run -- \
    python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r03c_$c.json 2> gpurun_out/prof_r03c_$c.err
done
echo done

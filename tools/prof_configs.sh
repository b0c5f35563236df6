#!/bin/bash
# rocprofv3 kernel statistics of the other BASELINE configs (one-shot call + fit
# of each, tools/bench_configs.py): cfg3 ReliefF, cfg5 SURF* and MultiSURF*, cfg2.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in cfg2 cfg3 cfg5s cfg5m; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$c/trace -o run -- \
    python3 tools/bench_configs.py --only $c --repeat 1 > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err
  echo "$c done"
done

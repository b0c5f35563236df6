#!/bin/bash
# End-of-round-3 measurement set (run via gpurun): the default cfg4 workload's
# kernel trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh, no
# 32-bit comparison job), every BASELINE config through bench.py
# (tools/bench_all.sh), and kernel traces of cfg2 / cfg3.
set -euo pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r03
bash tools/bench_all.sh r03_configs
for c in cfg2 cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03_$c/trace -o run -- \
    python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-q32 > gpurun_out/prof_r03_$c.json 2> gpurun_out/prof_r03_$c.err
done
echo done

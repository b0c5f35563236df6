#!/bin/bash
# Round-3 profile set (run via gpurun): the default cfg4 workload's kernel
# trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh), the SQ
# busy/wait counters of the round-2 sparse pass 2 (FS_SPARSE_V=1) for the
# v1 -> v2 table beside gpurun_out/pmc_v2, and kernel traces of cfg2 / cfg3.
set -euo pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r03
FS_SPARSE_V=1 bash tools/pmc_v2.sh v1
for c in cfg2 cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03_$c/trace -o run -- \
    python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r03_$c.json 2> gpurun_out/prof_r03_$c.err
done
echo done

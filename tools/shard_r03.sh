#!/bin/bash
# One rank's share of cfg4 at N = 2, 4, 8 (tools/shard_profile.py) beside the
# N = 1 bench step on the same box, and the N = 8 share's kernel statistics.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/shard_r03
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fit --no-q32 > "$OUT/bench_w1.json" 2> "$OUT/bench_w1.err"
for w in 2 4 8; do
  timeout -k 10 300 python3 tools/shard_profile.py --world $w --steps 5 > "$OUT/w$w.json" 2> "$OUT/w$w.err"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/w8_trace" -o run -- \
  python3 tools/shard_profile.py --world 8 --steps 3 > "$OUT/w8_prof.json" 2> "$OUT/w8_prof.err"
echo done

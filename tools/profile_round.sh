#!/bin/bash
# Profile the default bench workload on the GPU box (run via gpurun).
#   1. kernel trace + stats (durations, agrees with bench's HIP-event timing)
#   2. PMC pass FETCH_SIZE, 3. PMC pass WRITE_SIZE (separate passes, no
#      sys/runtime trace: see the gpurun rules), 1 timed step each.
# Summaries land in gpurun_out/prof_<tag>/ ; copy the ones to keep into profiles/.
set -euo pipefail
TAG=${1:-r01}
ARGS=${2:-"--steps 3 --warmup 1 --no-cpu-baseline --no-fit --no-q32 --no-ref"}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fit --no-q32 --no-ref > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fit --no-q32 --no-ref > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
find "$OUT" -name "*.csv" | head -20

#!/bin/bash
# Full GPU suite, then the round profile (trace + FETCH/WRITE + SQ) and one bench line.
set -euo pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests_${TAG}.log 2>&1
bash tools/profile_round.sh "$TAG"
bash tools/pmc_sq.sh "$TAG"
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err

#!/bin/bash
# GPU suite subset touching row statistics / neighbour counts, then a traced bench.
set -euo pipefail
mkdir -p gpurun_out/prof_sk
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sk_tests.log 2>&1
tail -1 gpurun_out/sk_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_sk/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sk/bench.json 2> gpurun_out/prof_sk/bench.err
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_sk/trace/run_kernel_stats.csv')):
    print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6,3))
" | head -14

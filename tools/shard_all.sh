#!/bin/bash
# One rank's share at world 2/4/8 (cfg4), then every BASELINE config.
set -euo pipefail
mkdir -p gpurun_out
for w in 2 4 8; do
  timeout -k 10 300 python3 tools/shard_profile.py --world $w > gpurun_out/shard_w$w.json 2> gpurun_out/shard_w$w.err
done
timeout -k 10 900 python3 tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err

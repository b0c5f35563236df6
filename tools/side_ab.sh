#!/bin/bash
# Mean correction beside k_dist (side stream) or before it (FS_SIDE=0): cfg4 world 1 and 8, cfg5 MultiSURF*.
set -euo pipefail
mkdir -p gpurun_out
for side in 1 0 1 0; do
  for w in 1 8; do
    FS_SIDE=$side timeout -k 10 120 python3 tools/shard_profile.py --world $w > gpurun_out/side.json 2> gpurun_out/side.err
    echo "side=$side $(cut -c1-150 gpurun_out/side.json)"
  done
done
for side in 1 0; do
  FS_SIDE=$side timeout -k 10 200 python3 tools/bench_configs.py --only cfg5m > gpurun_out/side5.json 2> gpurun_out/side5.err
  echo "side=$side cfg5m $(python3 -c "import json;d=json.loads(open('gpurun_out/side5.json').read().splitlines()[-1]);print(d['step_s']*1e3, d['k_dist_ms'], d['k_score_ms'])")"
done

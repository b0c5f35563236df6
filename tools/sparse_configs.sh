#!/bin/bash
# Per-config timings with the default pass 2, then the dense / sparse pass 2
# forced (FS_SPARSE=0/1) on the configs where the choice is close, and one
# rank's share at world 2/4/8 (cfg4).  Run on the GPU box via gpurun.
set -euo pipefail
mkdir -p gpurun_out
for w in 2 4 8; do
  timeout -k 10 300 python3 tools/shard_profile.py --world $w > gpurun_out/shard_w$w.json 2> gpurun_out/shard_w$w.err
done
timeout -k 10 900 python3 tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
FS_SPARSE=0 timeout -k 10 600 python3 tools/bench_configs.py --only cfg2,cfg4,cfg5m,cfg5surf \
  > gpurun_out/configs_dense.jsonl 2>> gpurun_out/configs.err
FS_SPARSE=1 timeout -k 10 600 python3 tools/bench_configs.py --only cfg5s \
  > gpurun_out/configs_sparse.jsonl 2>> gpurun_out/configs.err

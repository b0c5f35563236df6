#!/bin/bash
# Sparse pass-2 grid size (FS_PASS2_WGS) against one rank's step at world 1 and 8 (cfg4).
set -euo pipefail
mkdir -p gpurun_out
for wgs in ${WGS_LIST:-65536 131072}; do
  for w in 1 8; do
    FS_PASS2_WGS=$wgs timeout -k 10 120 python3 tools/shard_profile.py --world $w > gpurun_out/wgs_${wgs}_w$w.json 2> gpurun_out/wgs_${wgs}_w$w.err
    echo "wgs=$wgs $(cat gpurun_out/wgs_${wgs}_w$w.json)"
  done
done

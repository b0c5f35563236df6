#!/bin/bash
# K-split of pass 1 (FS_KSPLIT) against one rank's step, world 1 and 8 (cfg4).
set -euo pipefail
mkdir -p gpurun_out
for spec in "1 1" "1 2" "1 3" "1 1" "1 2" "8 0" "8 4" "8 6" "8 8"; do
  set -- $spec
  if [ "$2" = "0" ]; then unset FS_KSPLIT; else export FS_KSPLIT=$2; fi
  timeout -k 10 120 python3 tools/shard_profile.py --world $1 > gpurun_out/ks.json 2> gpurun_out/ks.err
  echo "world=$1 ksplit=$2 $(cut -c1-170 gpurun_out/ks.json)"
done

#!/bin/bash
# Quantisation split (xqT first, xs + eps beside k_dist) against one quantize (FS_QSPLIT=0).
# (FS_QSPLIT existed only in the A/B build; the split was not kept: DESIGN.md, profiles/r01l_qsplit_ab.txt)
set -euo pipefail
mkdir -p gpurun_out
for q in 1 0 1 0 1 0; do
  for w in 1 8; do
    FS_QSPLIT=$q timeout -k 10 120 python3 tools/shard_profile.py --world $w > gpurun_out/qs.json 2> gpurun_out/qs.err
    echo "qsplit=$q $(cut -c1-110 gpurun_out/qs.json)"
  done
done

#!/bin/bash
# A/B of the LDS row-read lead of the sparse loop (FS_SPARSE_LEAD, A/B build).
# (FS_SPARSE_LEAD selected variants only in A/B builds made with FS_GEN_LEAD_VARIANTS=1; see tools/gen_sparse_asm.py)
set -euo pipefail
mkdir -p gpurun_out
for v in ${LEADS:-2 1 0 -1 2 1 0 -1}; do
  FS_SPARSE_LEAD=$v timeout -k 10 120 python3 tools/shard_profile.py --world 1 > gpurun_out/lead.json 2> gpurun_out/lead.err
  echo "lead=$v $(cut -c1-150 gpurun_out/lead.json)"
done

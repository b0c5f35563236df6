#!/bin/bash
# Sparse pass-2 loop variants A/B on one box: FS_SPARSE_PK=0/1, correctness
# (FS_SPARSE_PK existed only in the A/B build; not kept: tools/gen_sparse_asm.py docstring)
# (sparse tests with the packed loop) then alternating world-1 cfg4 steps.
set -euo pipefail
mkdir -p gpurun_out
FS_SPARSE_PK=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -q -x --timeout 120 --timeout-method thread \
  -k "sparse or cfg1 or multisurf_sizes or mixed or device_cache" > gpurun_out/pk_tests.log 2>&1
tail -1 gpurun_out/pk_tests.log
for pk in 0 1 0 1; do
  FS_SPARSE_PK=$pk timeout -k 10 120 python3 tools/shard_profile.py --world 1 > gpurun_out/pk_$pk.json 2> gpurun_out/pk_$pk.err
  echo "pk=$pk $(cut -c1-200 gpurun_out/pk_$pk.json)"
done

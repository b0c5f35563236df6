#!/bin/bash
# k_exact_pairs_rows change: one rank's share at N=8 and the N=1 step,
# working tree against abtree/, alternating.
set -uo pipefail
OUT=gpurun_out/exact_ab.txt
: > "$OUT"
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=abtree
    (cd $d && timeout -k 10 200 python3 tools/shard_profile.py --world 8) > gpurun_out/w8_$t.json 2>/dev/null || exit 1
    echo "w8 $t $(cut -c1-200 gpurun_out/w8_$t.json)" >> "$OUT"
  done
done
cat "$OUT"

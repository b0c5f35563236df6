#!/bin/bash
# What the mean correction beside k_dist costs (FS_MEANCORR=0 skips
# k_colrank / k_rowcorr: a diagnostic, scores change), cfg2 and cfg4,
# alternating.
set -euo pipefail
OUT=gpurun_out/meancorr_ab.txt
: > "$OUT"
for rep in 1 2; do
  for v in 0 1; do
    for c in cfg2 cfg4; do
      if [ $v = 1 ]; then export FS_MEANCORR=0; else export FS_MEANCORR=1; fi
      line=$(timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-q32 --no-fit 2>/dev/null)
      python3 -c "import json,sys; d=json.loads(sys.argv[3]); print(sys.argv[1], 'nocorr=' + sys.argv[2], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})" $c $v "$line" >> "$OUT"
    done
  done
done
unset FS_MEANCORR

#!/bin/bash
# k_rf_select phase timing (cfg3): the first launch whole, up to the row
# load (FS_RF_DIAG=1 variant), up to the radix select (=2); the first
# launch's HIP-event time is kernel_ms k_rf_select in the bench line.
set -uo pipefail
OUT=gpurun_out/rf_phase_ab.txt
: > "$OUT"
for rep in 1 2; do
  for v in default rfd1 rfd2; do
    if [ $v = default ]; then unset FS_LIB_VARIANT; else export FS_LIB_VARIANT=$v; fi
    line=$(timeout -k 10 200 python3 bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null) || { echo "$v FAILED" >> "$OUT"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})" $v "$line" >> "$OUT"
  done
done

#!/bin/bash
# Pass-2 (v2) workgroup target (FS_PASS2_WGS) for one rank of N = 8
# (tools/shard_profile.py) and for the whole cfg4 step, alternating.
set -uo pipefail
OUT=gpurun_out/pass2_wgs_v2.txt
: > "$OUT"
for rep in 1 2; do
  for w in default 4096 8192 16384; do
    if [ $w = default ]; then unset FS_PASS2_WGS; else export FS_PASS2_WGS=$w; fi
    line=$(timeout -k 10 200 python3 tools/shard_profile.py --world 8 --steps 5 2>/dev/null) || { echo "w8 $w FAILED" >> "$OUT"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('w8', sys.argv[1], round(d['step_ms'],3), round(d['k_dist_ms'],3), round(d['k_score_ms'],3))" $w "$line" >> "$OUT"
  done
  for w in default 16384 65536; do
    if [ $w = default ]; then unset FS_PASS2_WGS; else export FS_PASS2_WGS=$w; fi
    line=$(timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-q32 --no-fit 2>/dev/null) || { echo "w1 $w FAILED" >> "$OUT"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('w1', sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})" $w "$line" >> "$OUT"
  done
done
unset FS_PASS2_WGS
bash tools/rf_phase_ab.sh

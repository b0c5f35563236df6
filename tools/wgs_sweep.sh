#!/bin/bash
# Pass-2 grid size (FS_PASS2_WGS) at cfg4, alternating with the default.
set -uo pipefail
OUT=gpurun_out/wgs_sweep.txt
: > "$OUT"
run() {
  local label=$1; shift
  local line
  line=$(env "$@" timeout -k 10 150 python3 bench.py --steps 5 --warmup 2 --no-fit --no-cpu-baseline 2>/dev/null) \
    || { echo "$label FAILED" >> "$OUT"; return 1; }
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],3), {k: round(v,3) for k,v in r['kernel_ms'].items()})" "$label" "$line" >> "$OUT"
}
for rep in 1 2; do
  run default FS_NOOP=1 || exit 1
  for w in 16384 24576 49152 65536; do run wgs$w FS_PASS2_WGS=$w || exit 1; done
done
cat "$OUT"

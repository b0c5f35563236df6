#!/bin/bash
# Every BASELINE config through bench.py at the end of round 4 (one line each)
out=gpurun_out/r04r
mkdir -p "$out"
for c in cfg2 cfg3 cfg5m cfg5s; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-fit \
    > "$out/$c.json" 2> "$out/$c.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],3), r.get('kernel'), round(r['frac'],3), {k: round(v,2) for k,v in r.get('kernel_ms',{}).items()}, d.get('cpu_baseline',{}).get('value'))"
done

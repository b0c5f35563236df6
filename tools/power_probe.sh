#!/bin/bash
# Board power and clocks while bench.py runs (is pass 2 power-limited?).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --steps 40 --warmup 2 --no-cpu-baseline > gpurun_out/power_bench.json 2> gpurun_out/power_bench.err &
BP=$!
for i in $(seq 1 40); do
  echo "t=$i $(date +%s.%N)"
  timeout 10 amd-smi metric -p -c 2>/dev/null | grep -iE "socket_power|gfx_0|SOCKET|POWER|CLK" | head -8
  sleep 0.4
done > gpurun_out/power_probe.txt 2>&1
wait $BP
echo "bench rc=$?"

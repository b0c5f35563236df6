#!/bin/bash
# End-of-round check (run via gpurun): the GPU suite, smoke(), the parity
# report over every fixture, the default bench line.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final_r03
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests > gpurun_out/final_r03/gpu_tests.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_r03/smoke.txt 2>&1
timeout -k 10 600 python3 -u tools/parity_report.py > gpurun_out/final_r03/parity_report.txt 2> gpurun_out/final_r03/parity_report.err
timeout -k 10 400 python3 bench.py > gpurun_out/final_r03/bench.json 2> gpurun_out/final_r03/bench.err
echo done

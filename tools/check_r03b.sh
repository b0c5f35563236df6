#!/bin/bash
# Re-entry check (run via gpurun): the GPU suite, smoke(), default bench and
# the cfg3 bench line on the current tree.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r03b}
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests > $out/gpu_tests.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err
timeout -k 10 300 python3 bench.py --config cfg3 > $out/bench_cfg3.json 2> $out/bench_cfg3.err
echo done

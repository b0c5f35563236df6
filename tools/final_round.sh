#!/bin/bash
# End-of-session check on one MI355X: smoke, the whole GPU suite, the default
# bench line (with CPU baseline and fit_ms), then the profile set of the
# round: kernel trace + FETCH/WRITE (tools/profile_round.sh), SQ counters
# (tools/pmc_sq.sh), LDS / scalar-cache counters (tools/pmc_lds.sh).
set -uo pipefail
TAG=${1:-r02z}
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo smoke FAILED; cat gpurun_out/${TAG}_smoke.txt; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo tests FAILED; tail -20 gpurun_out/${TAG}_tests.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo bench FAILED; tail gpurun_out/${TAG}_bench.err; exit 1; }
bash tools/profile_round.sh "$TAG" > /dev/null || { echo profile FAILED; exit 1; }
bash tools/pmc_sq.sh "$TAG" "--no-fit" > /dev/null || { echo pmc_sq FAILED; exit 1; }
bash tools/pmc_lds.sh "${TAG}l" > /dev/null || { echo pmc_lds FAILED; exit 1; }
cat gpurun_out/${TAG}_smoke.txt; tail -1 gpurun_out/${TAG}_tests.log; cut -c1-400 gpurun_out/${TAG}_bench.json

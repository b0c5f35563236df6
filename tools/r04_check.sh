#!/bin/bash
# Round-4 GPU check: selected GPU tests, then (unless a test run faulted or
# timed out) the default bench and a rocprofv3 kernel trace of it.
#   tools/r04_check.sh <tag> [pytest targets...]
# Results under gpurun_out/<tag>/.
tag=${1:?tag}
shift
out=gpurun_out/$tag
mkdir -p "$out"
targets=${*:-tests -m gpu}
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread $targets \
  > "$out/tests.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$out/tests.log"
tail -3 "$out/tests.log"
# 0 passed, 1 test failures: the GPU is fine, go on; anything else: stop
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > "$out/bench.json" 2> "$out/bench.err" || exit $?
cat "$out/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-q32 --no-fit \
  > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1 || exit $?
find "$GRAFT_REPO_ROOT/$out/prof" -name "*kernel_stats.csv" -exec head -25 {} \;

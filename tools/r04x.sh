#!/bin/bash
# Final tree of round 4: smoke, the whole GPU suite, the default bench line.
out=gpurun_out/r04x
mkdir -p "$out"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit $?
cat "$out/smoke.txt"
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu \
  > "$out/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/tests.log"; tail -3 "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
cat "$out/bench.json"

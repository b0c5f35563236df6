#!/bin/bash
# Round-4 verification of the tree: smoke, the whole GPU suite, the default
# bench line and a rocprofv3 kernel trace of it.
out=gpurun_out/r04q
mkdir -p "$out"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit $?
cat "$out/smoke.txt"
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu \
  > "$out/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/tests.log"; tail -3 "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > "$out/bench.json" 2> "$out/bench.err" || exit $?
cat "$out/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-q32 --no-fit \
  > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1 || exit $?

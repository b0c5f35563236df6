#!/bin/bash
# Kernel traces of the other BASELINE configs on the final tree (cfg3, cfg5m, cfg5s).
out=gpurun_out/r04y
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for c in cfg3 cfg5m cfg5s; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/$c" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-fit \
    > "$GRAFT_REPO_ROOT/$out/$c.json" 2> "$GRAFT_REPO_ROOT/$out/$c.err" || exit $?
done

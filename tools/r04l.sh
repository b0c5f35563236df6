#!/bin/bash
# Round-4 measurements on one MI355X:
#  1. mean-correction cost at cfg4: product (side stream) vs none (nomc,
#     wrong thresholds) vs on the main stream before k_dist (mcmain)
#  2. the round's profile set: kernel trace + FETCH_SIZE / WRITE_SIZE passes
#     (tools/profile_round.sh r04l)
#  3. cfg2 bench line + kernel trace
#  4. devices= phase log at cfg4 (X over the host link once)
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/variant_ab.sh r04l_ab 2 default nomc mcmain || exit $?
bash tools/profile_round.sh r04l || exit $?
out=gpurun_out/r04l
mkdir -p "$out"
timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 20 --warmup 3 --no-fit \
  > "$out/cfg2_bench.json" 2> "$out/cfg2_bench.err" || exit $?
cat "$out/cfg2_bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/cfg2_prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --no-fit \
  > "$GRAFT_REPO_ROOT/$out/cfg2_prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u tools/devices_trace.py > "$out/devices_trace.txt" 2>&1 || exit $?
tail -4 "$out/devices_trace.txt"

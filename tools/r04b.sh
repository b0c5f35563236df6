set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 300 python -u tools/colsort_debug.py 3000 64 > gpurun_out/r04b/dbg.txt 2>&1 || exit $?
FS_COLSORT_GLOBAL=1 timeout -k 10 300 python -u tools/colsort_debug.py 3000 64 >> gpurun_out/r04b/dbg.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/colsort_debug.py 25000 64 >> gpurun_out/r04b/dbg.txt 2>&1 || exit $?
cat gpurun_out/r04b/dbg.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04b/prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-q32 --no-fit \
  > "$GRAFT_REPO_ROOT/gpurun_out/r04b/prof.log" 2>&1 || exit $?
find "$GRAFT_REPO_ROOT/gpurun_out/r04b/prof" -name "*kernel_stats.csv" -exec head -30 {} \;

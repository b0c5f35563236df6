#!/bin/bash
# Mean-correction kernel A/B: the binned k_colsort (mcmain: on the main
# stream, so its own time shows) against every column through the block
# radix sort k_colsort_full (fullall), at n = 20000 and n = 5000; then the
# exact-threshold row count at cfg2.
out=gpurun_out/r04n
mkdir -p "$out"
lib=fastselect_amd/libfastselect_amd.so
cp $lib "$out/.product.so" || exit 1
for v in mcmain fullall; do
  cp fastselect_amd/libfastselect_amd_$v.so $lib || exit 1
  for n in 20000 5000; do
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv \
       -d "$GRAFT_REPO_ROOT/$out/${v}_$n" -o run -- python3 "$GRAFT_REPO_ROOT/tools/colsort_bench.py" $n 2048 2 gauss \
       > "$GRAFT_REPO_ROOT/$out/${v}_$n.log" 2>&1) || { cp "$out/.product.so" $lib; exit 1; }
    grep -h "colsort" "$out/${v}_$n/run_kernel_stats.csv" | cut -c1-160
  done
done
cp "$out/.product.so" $lib && rm -f "$out/.product.so"
FS_TRACE=1 timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 1 --warmup 0 --no-fit --no-cpu-baseline --no-q32 \
  > "$out/cfg2_trace.json" 2> "$out/cfg2_trace.err" || exit $?
grep "rows near" "$out/cfg2_trace.err" | head -3

#!/bin/bash
# Every BASELINE config through bench.py (tools/r04r.sh), then the mean
# correction alone at cfg4's n: the mcmain build (k_colsort + k_rowcorr on
# the main stream, so the trace shows their own time), 8192 vs 4096 bins.
bash tools/r04r.sh || exit $?
out=gpurun_out/r04t
mkdir -p "$out"
lib=fastselect_amd/libfastselect_amd.so
cp $lib "$out/.product.so" && cp fastselect_amd/libfastselect_amd_mcmain.so $lib || exit 1
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/tools/colsort_bench.py 20000 2048 2 gauss"
for v in 13 12; do
  if [ $v = 12 ]; then export FS_COLSORT_BINS12=1; else unset FS_COLSORT_BINS12; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$out/cs$v" -o run -- $B \
    > "$GRAFT_REPO_ROOT/$out/cs$v.log" 2>&1 || exit $?
  python3 -c "
import csv
for r in csv.DictReader(open('$GRAFT_REPO_ROOT/$out/cs$v/run_kernel_stats.csv')):
    if 'colsort' in r['Name'] or 'rowcorr' in r['Name']: print('bins$v', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
" | tee -a "$GRAFT_REPO_ROOT/$out/cs_ab.txt"
done
cp "$GRAFT_REPO_ROOT/$out/.product.so" "$GRAFT_REPO_ROOT/$lib"
cd "$GRAFT_REPO_ROOT" || exit 1
unset FS_COLSORT_BINS12
# cfg2: is the mean correction on the step's critical path (beside k_dist)?
bash tools/variant_ab.sh r04t_cfg2 2 default mcmain nomc sideprio -- --config cfg2 && bash tools/variant_ab.sh r04t_cfg4 2 default sideprio

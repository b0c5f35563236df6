#!/bin/bash
# k_colsort timed alone (the row guard's launch of tools/colsort_bench.py,
# before any k_dist) for the product library and variant builds:
#   tools/colsort_phase_ab.sh <tag> <variant>...   (variant "default" = product)
# Round 5 used it with builds that stop after phase k (wrong results) to
# price the phases, and to A/B the phase-4 bin-bound rewrite.
set -u
tag=${1:?tag}; shift
out=gpurun_out/$tag
mkdir -p $out
lib=fastselect_amd/libfastselect_amd.so
cp $lib $out/.product.so
export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = default ]; then cp $out/.product.so $lib; else cp fastselect_amd/libfastselect_amd_$v.so $lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/$v -o run -- python3 tools/colsort_bench.py 20000 2048 2 gauss > $out/$v.log 2>&1 || { cp $out/.product.so $lib; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$out/$v/**/run_kernel_trace.csv', recursive=True)[0]
rows=sorted((r for r in csv.DictReader(open(f)) if 'k_colsort<' in r['Kernel_Name']), key=lambda r: int(r['Start_Timestamp']))
print('$v', 'k_colsort us per launch (first = alone):', [round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3,1) for r in rows])
" | tee -a $out/ab.txt
done
cp $out/.product.so $lib
rm -f $out/.product.so

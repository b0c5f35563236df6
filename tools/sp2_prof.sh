#!/bin/bash
# Pass-2 walk clock stamps (a -DFS_SP2_PROF variant: make -C
# fastselect_amd/csrc variant V=sp2prof DEFS=-DFS_SP2_PROF): the variant
# replaces the product library inside this GPU-box snapshot for one short
# cfg4 bench (restored afterwards), which prints, per wave and tile, the
# shader clocks of the tile start (first entries + B rows landing), the
# stream walk and everything outside it.
#   tools/sp2_prof.sh <tag> [variant, default sp2prof]
tag=${1:?tag}
v=${2:-sp2prof}
out=gpurun_out/$tag
mkdir -p "$out"
lib=fastselect_amd/libfastselect_amd.so
cp "$lib" "$out/.product.so" || exit 1
cp "fastselect_amd/libfastselect_amd_$v.so" "$lib" || exit 1
FS_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-q32 --no-fit \
  > "$out/$v.json" 2> "$out/$v.err"
rc=$?
cp "$out/.product.so" "$lib"
rm -f "$out/.product.so"
[ $rc -eq 0 ] || exit $rc
echo "== $v"; grep "k_score_sparse2" "$out/$v.err"

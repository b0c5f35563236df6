#!/bin/bash
# A/B of library variants on one GPU box (make -C fastselect_amd/csrc variant
# V=<name> DEFS=...): each round runs the cfg4 bench once per variant, in turn
# (default = the product library), so box drift hits every variant alike.
#   tools/variant_ab.sh <tag> <rounds> <variant>... [-- bench args]
# Each variant's library replaces the product one inside this snapshot only;
# the product library is restored afterwards.  One line per run in
# gpurun_out/<tag>/ab.txt: variant, round, ms per step, kernel ms.
tag=${1:?tag}; rounds=${2:?rounds}; shift 2
vars=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ "$1" = "--" ] && shift
out=gpurun_out/$tag
mkdir -p "$out"
lib=fastselect_amd/libfastselect_amd.so
cp "$lib" "$out/.product.so" || exit 1
for r in $(seq 1 "$rounds"); do
  for v in "${vars[@]}"; do
    if [ "$v" = default ]; then cp "$out/.product.so" "$lib"; else cp "fastselect_amd/libfastselect_amd_$v.so" "$lib"; fi || exit 1
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-q32 --no-fit "$@" \
      > "$out/$v.$r.json" 2> "$out/$v.$r.err" || { cp "$out/.product.so" "$lib"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['roofline']['kernel_ms'].items()})" \
      "$out/$v.$r.json" "$v" "$r" | tee -a "$out/ab.txt"
  done
done
cp "$out/.product.so" "$lib"
rm -f "$out/.product.so"

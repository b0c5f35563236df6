#!/bin/bash
# Kernel stats of library variants (make -C fastselect_amd/csrc variant
# V=<name> DEFS=...) on one GPU box: each variant's library replaces the
# product one inside this snapshot, the bench runs under rocprofv3
# --kernel-trace --stats, and the rows of the kernels matching <pattern> are
# printed per variant; the product library is restored afterwards.
#   tools/variant_prof.sh <tag> <pattern> <variant>... [-- bench args]
tag=${1:?tag}; pat=${2:?pattern}; shift 2
vars=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ "$1" = "--" ] && shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
lib=fastselect_amd/libfastselect_amd.so
cp "$lib" "$out/.product.so" || exit 1
for v in "${vars[@]}"; do
  if [ "$v" = default ]; then cp "$out/.product.so" "$lib"; else cp "fastselect_amd/libfastselect_amd_$v.so" "$lib"; fi || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$out/$v" -o run -- \
    python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-q32 --no-fit --no-ref "$@" \
    > "$out/$v.json" 2> "$out/$v.err" || { cp "$out/.product.so" "$lib"; exit 1; }
  stats=$(find "$out/$v" -name "*kernel_stats.csv" | head -1)
  python3 - "$stats" "$pat" "$v" "$out/$v.json" <<'PY' | tee -a "$out/prof.txt"
import csv, json, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms_per_step", round(d["ms_per_step"], 2))
for r in rows:
    if re.search(sys.argv[2], r["Name"]):
        print("  ", r["Name"][:60], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1),
              "total_ms", round(float(r["TotalDurationNs"]) / 1e6, 2))
PY
done
cp "$out/.product.so" "$lib"
rm -f "$out/.product.so"

"""Per-kernel table of the counters collected by tools/pmc_sq.sh."""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            k = k.split("(")[0].replace("fs::gpu::", "").replace("refacc::", "")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in vals.items():
        if not k.startswith("k_"):
            continue
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        print(k)
        for n in sorted(avg):
            print(f"   {n:24s} {avg[n]:.4g}")
        if "SQ_WAVE_CYCLES" in avg:
            w = avg["SQ_WAVE_CYCLES"]
            print(f"   wait_any {avg.get('SQ_WAIT_ANY', 0) / w:.3f}  wait_inst {avg.get('SQ_WAIT_INST_ANY', 0) / w:.3f}"
                  f"  active_inst {avg.get('SQ_ACTIVE_INST_ANY', 0) / w:.3f}  active_valu {avg.get('SQ_ACTIVE_INST_VALU', 0) / w:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])

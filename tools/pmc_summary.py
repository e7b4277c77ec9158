"""Average rocprofv3 PMC counters per kernel over dispatches (our nslam kernels by default).

usage: python tools/pmc_summary.py gpurun_out/pmc/p1 [gpurun_out/pmc/p2 ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            seen = set()
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "nslam" not in name and "anonymous namespace)::k_" not in name:
                    continue
                short = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
                short = name[name.find("k_"):name.find("((")] if "k_" in name else short
                acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (r["Dispatch_Id"], short)
                if key not in seen:
                    seen.add(key)
                    dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in sorted(acc):
        d = sum(dur[k]) / max(len(dur[k]), 1)
        print(f"== {k}  (avg {d:.1f} us over {len(dur[k])} dispatch-passes)")
        for c, v in sorted(acc[k].items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()

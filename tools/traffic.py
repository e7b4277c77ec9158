"""HBM traffic per launch of each nslam kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/traffic.py FETCH_DIR WRITE_DIR CMD > profiles/r01_traffic.json

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced read (128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE is exact for 16-B
stores and float atomics.  Both are in KiB per dispatch.  Kernels are serialised under --pmc.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if r["Counter_Name"] != counter or "k_" not in name:
                continue
            if "nslam" not in name and "anonymous namespace)::k_" not in name:
                continue
            k0 = name.find("k_")
            short = name[k0:name.find("(", k0)].strip()
            vals[short].append(float(r["Counter_Value"]))
    return vals


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else ""
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch[k]) / len(fetch[k]) if fetch[k] else None
        w = sum(write[k]) / len(write[k]) if write[k] else None
        tot = None if f is None or w is None else (2 * f + w) * 1024
        out[k] = {"fetch_size_kib_raw": f, "write_size_kib": w, "dispatches": max(len(fetch[k]), len(write[k])),
                  "hbm_bytes_per_launch": tot}
    print(json.dumps({"command": cmd, "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B), gfx950",
                      "kernels": out}, indent=1))


if __name__ == "__main__":
    main()

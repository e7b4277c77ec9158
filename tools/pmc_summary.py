"""Average rocprofv3 PMC counters per kernel over dispatches (our nslam kernels by default).

usage: python tools/pmc_summary.py gpurun_out/pmc/p1 [gpurun_out/pmc/p2 ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 1024  # MI355X: 256 CUs x 4 SIMDs
F_MAX_GHZ = 2.4  # MI355X peak engine clock


def main():
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
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
        m = {c: sum(v) / len(v) for c, v in acc[k].items()}
        for c, v in sorted(m.items()):
            print(f"   {c:28s} {v:16.1f}")
        # derived (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE sums the 8 XCDs' cycles; SQ_WAVE_CYCLES and
        # SQ_ACTIVE_INST_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles; 1024 SIMDs).
        # SIMD-cycles = the kernel's own rocprof duration x its clock: GRBM_GUI_ACTIVE / 8 over the
        # duration when that is a clock the part can run (<= 2.4 GHz), else 2.4 GHz — a GRBM window
        # that yields more also counted other work (launch overhead of a short kernel, or a kernel
        # beside it), and normalising by it would understate every fraction.
        if "GRBM_GUI_ACTIVE" in m and d > 0:
            ghz_grbm = m["GRBM_GUI_ACTIVE"] / 8 / (d * 1e3)
            ghz = min(ghz_grbm, F_MAX_GHZ)
            simd_cyc = d * 1e3 * ghz * SIMDS
            flag = "" if ghz_grbm <= F_MAX_GHZ else f"   (GRBM window {ghz_grbm:.2f} GHz: capped)"
            print(f"   {'(clock GHz)':28s} {ghz:16.3f}{flag}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                print(f"   {'(MFMA busy / SIMD-cycles)':28s} {m['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cyc:16.3f}")
            if "SQ_WAVE_CYCLES" in m:
                print(f"   {'(resident waves / SIMD)':28s} {4 * m['SQ_WAVE_CYCLES'] / simd_cyc:16.3f}")
            if "SQ_ACTIVE_INST_VALU" in m:
                print(f"   {'(VALU issue / SIMD-cycles)':28s} {4 * m['SQ_ACTIVE_INST_VALU'] / simd_cyc:16.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("SQ_INSTS_MFMA"):
            print(f"   {'(MFMA busy cycles / instr)':28s} {m['SQ_VALU_MFMA_BUSY_CYCLES'] / m['SQ_INSTS_MFMA']:16.1f}")
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if c in m and m.get("SQ_WAVE_CYCLES"):
                print(f"   {'(' + c + ' / WAVE_CYCLES)':28s} {m[c] / m['SQ_WAVE_CYCLES']:16.3f}")


if __name__ == "__main__":
    main()

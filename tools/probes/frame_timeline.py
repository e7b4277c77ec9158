"""One tracked frame's dispatch timeline from a rocprofv3 kernel trace: the dispatches between two
consecutive k_cam_vector_batch launches (the first node of a frame's graph), with queue, start offset,
duration and the gap since the previous dispatch ended.  usage: python frame_timeline.py <rocprof dir> [k]"""
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name.replace("void ", ""))
    return name.split("<")[0].split("::")[-1][:48]


def main():
    path = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_cam_vector_batch" in r["Kernel_Name"]]
    if len(starts) < k + 2:
        k = len(starts) - 2
    a, b = starts[k], starts[k + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    print(f"frame {k}: {b - a} dispatches, {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us to the next frame")
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        print(f"q{r['Queue_Id']:>2} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {(s - prev_end) / 1e3:6.1f}  "
              f"grid {r['Grid_Size_X']:>7}  {short(r['Kernel_Name'])}")
        prev_end = max(prev_end, e)
    print(f"busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()

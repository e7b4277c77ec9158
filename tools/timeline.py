"""Print the kernel timeline of one mapping iteration (the last k_gather_rays .. next) from a
rocprofv3 kernel_trace.csv: start offset, duration, queue, kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "k_gather_rays" in r["Kernel_Name"]]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3   # which iteration, counted from the end
i0, i1 = (marks[-back], marks[-back + 1]) if len(marks) >= back else (0, len(rows))
t0 = int(rows[i0]["Start_Timestamp"])
end = t0
busy = []
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:70]
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{r['Queue_Id']:>3}  {name}")
    end = max(end, e)
print(f"iteration span {(end - t0) / 1e3:.1f} us")

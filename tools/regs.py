"""Per-kernel register / spill / LDS usage of one csrc file (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python tools/regs.py nslam_query.hip [name-filter] [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = sys.argv[3:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-munsafe-fp-atomics", "-I../../include", "--cuda-device-only", "-c", src, "-o", "/tmp/regs.o",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True, cwd="nice-slam_amd/csrc").stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (?:\S+: )?\s*(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|SGPRs Spill|VGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:70]:70s} V{r.get('VGPRs')} A{r.get('AGPRs')} spill{r.get('VGPRs Spill')} "
              f"scratch{r.get('ScratchSize [bytes/lane]')} occ{r.get('Occupancy [waves/SIMD]')} lds{r.get('LDS Size [bytes/block]')}")

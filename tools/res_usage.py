#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of a HIP source file for
gfx950 (hipcc -Rpass-analysis=kernel-resource-usage), to catch spills before
a GPU run. Usage: tools/res_usage.py SRC.hip [-Dflags...] [--filter substr]"""
import re
import subprocess
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--filter")]
filt = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--filter=")), "")
src, flags = args[0], args[1:]
R = __file__.rsplit("/tools/", 1)[0]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
       "-Wno-unused-function", f"-I{R}/include",
       f"-I{R}/real-time-recommendation-system-with-feature-store_amd/csrc",
       "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"] + flags
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)",
                  line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
for r in rows:
    if filt and filt not in r["name"]:
        continue
    dm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    print(f"{r.get('VGPRs', 0):4d} vgpr {r.get('AGPRs', 0):4d} agpr {r.get('ScratchSize', 0):5d} scratch "
          f"{r.get('Occupancy', 0):2d} occ {r.get('LDS', 0):6d} lds  {dm[:110]}")

"""Per-kernel VGPR/AGPR/scratch/occupancy of libmpcx (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/resource_usage.py [filter]
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "mpc-verde_amd"), "-j8", "resource-usage"],
                     capture_output=True, text=True)
out = out.stdout + out.stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)",
                  line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"fn": v}
        rows.append(cur)
    else:
        cur[k.split()[0]] = v
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    name = subprocess.run(["c++filt", r["fn"]], capture_output=True, text=True).stdout.strip()
    if flt in name:
        print(f"{r.get('VGPRs', '?'):>4} {r.get('AGPRs', '?'):>4} scratch {r.get('ScratchSize', '?'):>5} "
              f"occ {r.get('Occupancy', '?')}  {name}")

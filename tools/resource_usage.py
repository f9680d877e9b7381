"""Per-kernel VGPR/AGPR/scratch/occupancy of libmpcx (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/resource_usage.py [filter] [--units unicycle,dyn_bicycle] [-D...]

Each model unit (csrc/solve_<model>.hip) is compiled for the device only, in parallel, with its
remarks captured separately (so the rows of different units never interleave).
"""
import concurrent.futures
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "mpc-verde_amd")


def unit_rows(path, defines):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I../include", "-Icsrc",
           "--cuda-device-only", "-c", path, "-o", f"/tmp/ru_{os.path.basename(path)}.o",
           "-Rpass-analysis=kernel-resource-usage"] + defines
    out = subprocess.run(cmd, capture_output=True, text=True, cwd=SRC)
    rows, cur = [], None
    for line in (out.stdout + out.stderr).splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): "
                      r"(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"fn": v}
            rows.append(cur)
        else:
            cur[k.split()[0]] = v
    return rows


def main():
    args = sys.argv[1:]
    defines = [a for a in args if a.startswith("-D")]
    units = None
    flt = ""
    for i, a in enumerate(args):
        if a == "--units":
            units = args[i + 1].split(",")
        elif not a.startswith("-") and (i == 0 or args[i - 1] != "--units"):
            flt = a
    paths = sorted(glob.glob(os.path.join(SRC, "csrc", "solve_*.hip")))
    if units:
        paths = [p for p in paths if os.path.basename(p)[6:-4] in units]
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        results = list(ex.map(lambda p: unit_rows(p, defines), paths))
    for rows in results:
        for r in rows:
            name = subprocess.run(["c++filt", r["fn"]], capture_output=True, text=True).stdout.strip()
            if flt in name:
                print(f"{r.get('VGPRs', '?'):>4} {r.get('AGPRs', '?'):>4} scratch {r.get('ScratchSize', '?'):>5} "
                      f"occ {r.get('Occupancy', '?')}  {name}")


if __name__ == "__main__":
    main()

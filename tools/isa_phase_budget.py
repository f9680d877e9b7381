#!/usr/bin/env python3
"""Static per-phase instruction budget of the fused solve kernel from its ISA.

    hipcc ... --cuda-device-only -S -DMPCX_STAMPS -o k.s csrc/solve_unicycle_xfree.hip
    python tools/isa_phase_budget.py k.s SYMBOL [--trips loopheader=count ...]

The diagnostic build (-DMPCX_STAMPS) fences every solver phase with an `s_memtime` (kernels.h
STAMP), so the kernel's code between two consecutive s_memtime instructions, in program order,
is one phase of the IPM iteration.  For each phase this counts the VALU instructions (and the
FP64 ones among them), the SALU, LDS and global/scratch memory instructions, split into the
straight-line part and the bodies of the loops nested in the phase (LLVM's `Loop Header` block
comments; depth relative to the solve loop).  Dynamic counts per IPM iteration follow by
multiplying each loop body with its trip count (e.g. the Riccati chain: N steps at the loop's
unroll factor), given with --trips; blocks laid out cold (restoration, soft restoration) are
reported as such and not counted.
"""
import argparse
import json
import re
import sys

F64 = re.compile(r"^v_\w*f64")


def kernel_lines(path, sym):
    out, on = [], False
    with open(path) as f:
        for ln in f:
            if ln.startswith(sym + ":"):
                on = True
                continue
            if on:
                out.append(ln.rstrip("\n"))
                if "s_endpgm" in ln:
                    break
    if not out:
        raise SystemExit(f"{sym} not found in {path}")
    return out


def classify(mn):
    if mn.startswith("v_"):
        return "valu_f64" if F64.match(mn) else "valu_other"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def parse(lines):
    """Blocks in program order: (label, loop header of the block or None, depth, instrs)."""
    blocks = []
    cur = {"label": "entry", "header": None, "depth": 0, "ins": []}
    for ln in lines:
        m = re.match(r"^(\.LBB\w+):\s*(;.*)?$", ln)
        if m:
            blocks.append(cur)
            com = m.group(2) or ""
            depth = int(re.search(r"Depth=(\d+)", com).group(1)) if "Depth=" in com else 0
            hdr = None
            h = re.search(r"Header=(BB\w+)", com)
            if h:
                hdr = h.group(1)
            elif "Loop Header" in com:
                hdr = m.group(1).lstrip(".L")
            cur = {"label": m.group(1), "header": hdr, "depth": depth, "ins": []}
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            if "Loop Header" in s and cur["ins"] == []:  # header comment on its own line
                d = re.search(r"Depth=(\d+)", s)
                cur["depth"] = int(d.group(1)) if d else cur["depth"]
                cur["header"] = cur["label"].lstrip(".L")
            continue
        mn = s.split()[0]
        st = re.search(r"stamp (\d+)", s) if mn == "s_memtime" else None
        cur["ins"].append(f"s_memtime#{st.group(1)}" if st else mn)
    blocks.append(cur)
    return blocks


def budget(blocks, trips):
    phases, cur = [], None
    for b in blocks:
        for mn in b["ins"]:
            if mn.startswith("s_memtime") or cur is None:
                # a stamp build labels each s_memtime with the phase it opens (kernels.h STAMP)
                cur = {"loops": {}, "straight": {}, "phase": int(mn.split("#")[1]) if "#" in mn else None}
                phases.append(cur)
                if mn.startswith("s_memtime"):
                    mn = "s_memtime"
            key = "straight" if b["depth"] <= 1 else "loops"
            tgt = cur["straight"] if key == "straight" else cur["loops"].setdefault(f"{b['header']}@{b['depth']}", {})
            c = classify(mn)
            tgt[c] = tgt.get(c, 0) + 1
            if mn.startswith("v_rcp_f64"):  # (counted again: the Riccati chain's steps per loop body)
                tgt["_rcp"] = tgt.get("_rcp", 0) + 1
    out = []
    for i, p in enumerate(phases):
        dyn = dict(p["straight"])
        for name, cnt in p["loops"].items():
            t = trips.get(name.split("@")[0], 1)
            for c, n in cnt.items():
                if not c.startswith("_"):
                    dyn[c] = dyn.get(c, 0) + t * n
        out.append({"region": i, "phase": p["phase"], "straight": p["straight"], "loops": p["loops"],
                    "dynamic_estimate": dyn, "valu": dyn.get("valu_f64", 0) + dyn.get("valu_other", 0)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--trips", nargs="*", default=[], help="BBx_y=count: trip count of a loop header")
    a = ap.parse_args()
    trips = {t.split("=")[0]: float(t.split("=")[1]) for t in a.trips}
    res = budget(parse(kernel_lines(a.asm, a.symbol)), trips)
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

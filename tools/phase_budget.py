#!/usr/bin/env python3
"""Per-phase budget of the config-2 solve kernel: instructions issued (static ISA of the stamps
build), cycles (s_memtime stamps, measured) and algorithmic FP64 flops, per IPM iteration.

    hipcc ... --cuda-device-only -S -DMPCX_STAMPS -DMPCX_STAMP_SUB -DMPCX_STAMP_EVAL \
        -o k.s csrc/solve_unicycle_xfree.hip
    python tools/phase_budget.py k.s SYMBOL STAMPS.json [--N 20] > profiles/r04_phase_budget.json

Instructions: every s_memtime of the stamps build carries the phase it opens (kernels.h STAMP,
`; stamp p`), so tools/isa_phase_budget.py attributes each instruction to a phase; the Riccati
chain's loop body counts N times, every other loop once (one inertia-correction attempt, one
line-search trial and one barrier-update pass: the config-2 norm).  Cycles: the
slowest wave's stamps (tools/stamp_profile.py on the same build).  Algorithmic flops: per node,
bench.py's accounting (ipm_vector_flops, the stage evaluation and Riccati step measured by
tools/flop_probe.py), times the nodes that carry them.  Lanes: 64 per wave, all issuing.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_phase_budget as ipb  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASES = ["errors", "barrier_update", "sigma", "riccati", "forward", "fraction", "linesearch", "update", "sweep",
          "trial_eval", "ric_stage", "ric_scan", "ric_chain", "ric_post", "err_sums", "err_tests"]
# phase 9 is the line search's trial evaluation in a -DMPCX_STAMP_EVAL build (the loop-exit slot otherwise)


def algorithmic(N, n=3, m=2, nbs=4):
    """Algorithmic FP64 flops per IPM iteration of one config-2 instance, per phase group."""
    with open(os.path.join(ROOT, "profiles", "r04_flop_probe.json")) as f:
        probe = json.load(f)
    E = probe["eval"]["unicycle_quadrature_M4"]["flops_per_unit"]
    R = probe["riccati"]["unicycle"]["flops_per_unit"]
    nz = n + m
    return {
        "errors": N * (n + 2 * n * n + 2 * n * m + 5 * nz + 3 * n + 2 * nbs + 5),
        "barrier_update": N * 3 * nbs,
        "sigma": N * (6 * nbs + 2 * nz),
        "riccati": N * R,
        "forward": N * (2 * m * n + 2 * n * n + 2 * n * m + n + 2 * n * n + 2 * n),
        "fraction": N * (14 * nbs + 5 * nz),
        "linesearch": N * (2 * nz + 2 * n + 3 * n + 2 * nbs + 4),
        "trial_eval": N * E,
        "update": N * (2 * nz + 2 * n + 8 * nbs),
        "sweep": 0,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("stamps")
    ap.add_argument("--N", type=int, default=20)
    a = ap.parse_args()
    blocks = ipb.parse(ipb.kernel_lines(a.asm, a.symbol))
    regions = ipb.budget(blocks, {})
    # the chain loop: the Riccati sub-phases' loop whose body holds the steps' reciprocals (two
    # v_rcp_f64 per step: the sequential chain one step per trip, the row chains two) runs N steps
    per = {}
    for i, r in enumerate(regions):
        ph = r["phase"]
        if ph is None:
            continue
        # phase 9 opens twice: the trial evaluation (closed by stamp 6) and the loop exit, after
        # which the cold blocks (soft restoration, parking, restoration calls) are laid out
        if ph == 9 and not (i + 1 < len(regions) and regions[i + 1]["phase"] == 6):
            continue
        name = PHASES[ph]
        acc = per.setdefault(name, {"valu": 0, "valu_f64": 0, "lds": 0, "vmem": 0, "salu": 0})
        parts = [(r["straight"], 1)]
        if r["loops"]:
            for k, cnt in r["loops"].items():
                # (depth 3: inside the solve loop and the inertia-correction attempts)
                steps = cnt.get("_rcp", 0) // 2 if int(k.split("@")[1]) >= 3 else 0
                t = a.N / steps if (name in ("ric_scan", "ric_chain") and steps) else 1
                parts.append((cnt, t))
        for cnt, t in parts:
            for c, v in cnt.items():
                if c == "valu_f64":
                    acc["valu_f64"] += t * v
                    acc["valu"] += t * v
                elif c == "valu_other":
                    acc["valu"] += t * v
                elif c in acc:
                    acc[c] += t * v
    with open(a.stamps) as f:
        st = json.load(f)
    cyc = st["cycles_per_iter"]
    cycles = {PHASES[i] if i < len(PHASES) else k: round(v * cyc) for i, (k, v) in enumerate(st["share"].items())}
    alg = algorithmic(a.N)
    groups = {  # stamp phases -> algorithmic accounting groups
        "errors": ["errors", "err_sums", "err_tests"], "barrier_update": ["barrier_update"], "sigma": ["sigma"],
        "riccati": ["riccati", "ric_stage", "ric_scan", "ric_chain", "ric_post"], "forward": ["forward"],
        "fraction": ["fraction"], "linesearch": ["linesearch"], "trial_eval": ["trial_eval"], "update": ["update"],
        # the loop-top evaluation: skipped when the line search's first trial (which evaluated
        # derivatives) was accepted, so its static code is large and its cycles small
        "sweep": ["sweep"],
    }
    out = {"_meta": {"kernel": a.symbol, "N": a.N, "source": "static ISA of the stamps build (instructions per IPM "
                     "iteration: chain loop x N steps, other loops x 1) + s_memtime stamps of the slowest wave (cycles)",
                     "cycles_per_iteration": round(cyc), "iters_slowest_wave": st.get("iters_slowest_wave")},
           "phases": {}}
    for g, members in groups.items():
        ins = {"valu": 0, "valu_f64": 0, "lds": 0, "vmem": 0, "salu": 0}
        cy = 0
        for mname in members:
            for c in ins:
                ins[c] += per.get(mname, {}).get(c, 0)
            cy += cycles.get(mname, 0)
        issued_lane_flops = 64 * 2 * ins["valu_f64"]  # upper bound: every f64 VALU an FMA on 64 lanes
        out["phases"][g] = {"valu_instructions": ins["valu"], "valu_f64_instructions": ins["valu_f64"],
                            "lds_instructions": ins["lds"], "salu_instructions": ins["salu"], "cycles": cy,
                            "algorithmic_flops": alg[g],
                            "algorithmic_over_issued_lane_flops": round(alg[g] / issued_lane_flops, 4)
                            if issued_lane_flops else None}
    tot = {k: sum(p[k] for p in out["phases"].values()) for k in ("valu_instructions", "valu_f64_instructions",
                                                                   "cycles", "algorithmic_flops")}
    out["total"] = tot
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

"""Summarise tools/solve_pmc.sh: per-dispatch averages over the solve_kernel dispatches.

    python tools/solve_pmc_summary.py gpurun_out/solve_pmc/c2 [more run dirs ...] > profiles/r03_solve_kernel_pmc.json

Several run directories (one per workload, tools/solve_pmc_all.sh) merge into one record per
kernel.  "_meta.mpcx_source_hash" is the source hash of the library the runs measured (from
the bench lines of the pass logs; all runs must agree): bench.py uses a record only while the
tree's sources still hash to it.

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over waves
(MI355X_MICROARCH.md, PMC units); WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.
FP64 lane-operations = 64 x (ADD + MUL + TRANS + 2 FMA) wave-instructions (inactive lanes
included: an upper bound on useful flops).  Peak FP64 vector: 78.6 TFLOP/s (MI355X spec).
f64_lane_flops_per_group_iteration = the kernel's lane-flops summed over its dispatches / the
IPM iterations of all lane groups in the run (bench.py's `iters_sum_all_steps`, read from the
pass-B log): bench.py scales it by the fraction of lanes holding a node and by a launch's
group-iterations for its live roofline entry.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PEAK_FP64_TFLOPS = 78.6


def counters(d):
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "solve_kernel" not in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} | {"dispatches": len(disp[k]), "_total": dict(cs)}
            for k, cs in agg.items()}


def bench_line(log):
    """The bench JSON line of a pass log (or {})."""
    try:
        for line in open(log):
            if line.startswith("{") and "iters_sum_all_steps" in line:
                return json.loads(line)
    except OSError:
        pass
    return {}


def bench_iters(log):
    """iters_sum_all_steps of the bench JSON line in a pass log."""
    return bench_line(log).get("iters_sum_all_steps")


def durations(d):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "solve_kernel" in r["Kernel_Name"]:
                out[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return out


def summarise(root):
    a, b, tr = counters(os.path.join(root, "a")), counters(os.path.join(root, "b")), durations(os.path.join(root, "trace"))
    res = {}
    for k in a:
        ca, cb = a[k], b.get(k, {})
        ts = sorted(tr.get(k, []))
        t = ts[len(ts) // 2] if ts else None
        wc = ca["SQ_WAVE_CYCLES"]
        f64 = {n: cb.get(f"SQ_INSTS_VALU_{n}_F64", 0.0) for n in ("ADD", "MUL", "FMA", "TRANS")}
        flops = 64 * (f64["ADD"] + f64["MUL"] + f64["TRANS"] + 2 * f64["FMA"])
        tot = cb.get("_total", {})
        flops_total = 64 * sum((2 if n == "FMA" else 1) * tot.get(f"SQ_INSTS_VALU_{n}_F64", 0.0)
                               for n in ("ADD", "MUL", "FMA", "TRANS"))
        its = bench_iters(os.path.join(root, "b.log"))
        r = {"dispatches": ca["dispatches"], "duration_ms_median": None if t is None else round(t * 1e3, 4),
             "wave_cycles_share": {"issuing": round(ca["SQ_ACTIVE_INST_ANY"] / wc, 4),
                                   "dependency_or_pipe_stall": round(ca["SQ_WAIT_INST_ANY"] / wc, 4),
                                   "waitcnt_or_barrier": round(ca["SQ_WAIT_ANY"] / wc, 4)},
             "valu_active_share": round(ca["SQ_ACTIVE_INST_VALU"] / wc, 4),
             "insts_per_dispatch": {"valu": ca["SQ_INSTS_VALU"], "salu": ca["SQ_INSTS_SALU"], "lds": ca["SQ_INSTS_LDS"]},
             "f64_insts_per_dispatch": f64, "f64_lane_flops_per_dispatch": flops,
             "valu_f64_share_of_valu": round(sum(f64.values()) / max(ca["SQ_INSTS_VALU"], 1.0), 4),
             "group_iterations_in_run": its,
             "f64_lane_flops_per_group_iteration": (flops_total / its) if its and ", true," not in k else None,
             # wave-level VALU instructions per IPM iteration of one instance (one wave per instance
             # for groups of 64 lanes or replicated 32-lane groups; G < 64 groups share a wave)
             "valu_insts_per_group_iteration": (ca["_total"]["SQ_INSTS_VALU"] / its) if its and ", true," not in k
             else None}
        if t:
            r["fp64_tflops"] = round(flops / t / 1e12, 3)
            r["fp64_frac_of_peak"] = round(flops / t / 1e12 / PEAK_FP64_TFLOPS, 4)
        r["workload"] = bench_line(os.path.join(root, "b.log")).get("config", {}).get("workload")
        res[k] = r
    return res


def main():
    res, hashes = {}, set()
    for root in sys.argv[1:]:
        res.update(summarise(root))
        for p in ("a", "b", "trace"):
            h = bench_line(os.path.join(root, f"{p}.log")).get("mpcx_source_hash")
            if h:
                hashes.add(h)
    if len(hashes) != 1:
        raise SystemExit(f"runs disagree on (or lack) the library source hash: {sorted(hashes)}")
    root = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
    out = {"_meta": {"mpcx_source_hash": hashes.pop(), "runs": [os.path.relpath(r, root) for r in sys.argv[1:]]}}
    out.update(res)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""HBM bytes of the bench's timed K-step solve launch from two rocprofv3 PMC passes
(profiles/r06_solve_traffic.json; bench.py reads it into roofline.traffic while the tree's
sources still hash to the ones measured).

    python tools/solve_traffic.py FETCH_DIR WRITE_DIR [OUT]

FETCH_DIR / WRITE_DIR hold the *_counter_collection.csv of separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes over
`bench.py --profile-solve-only` (warm-up steps, then the timed launch, then exit).  The timed
launch is the last solve dispatch that is not a resume launch (`solve_kernel<..., false, R>`)
plus any resume dispatch after it.  Corrections as tools/pmc_summary.py (MI355X_MICROARCH.md
§HBM and profiles/r01_pmc_calibration.json): FETCH_SIZE x2 on gfx950, WRITE_SIZE x1, both KiB.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))


def dispatches(d, counter):
    """[(dispatch id, kernel name, counter value)] of the solve kernels, in dispatch order."""
    f = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
    acc = {}
    for r in csv.DictReader(open(f)):
        if "solve_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            k = int(r["Dispatch_Id"])
            name, v = acc.get(k, (r["Kernel_Name"], 0.0))
            acc[k] = (name, v + float(r["Counter_Value"]))
    return [(k, n, v) for k, (n, v) in sorted(acc.items())]


def timed_launch(rows):
    last = max(i for i, (_, n, _) in enumerate(rows) if ", false, " in n)
    return rows[last][1], sum(v for _, _, v in rows[last:]), len(rows) - last


def profiled_hash(d):
    """mpcx_source_hash the profiled bench process printed (its stdout, D + '.log', as
    tools/round_profile.sh writes it): the library that ran under the counters, not the one this
    script would load."""
    log = d.rstrip("/") + ".log"
    for ln in open(log):
        if ln.startswith("{") and "profile_solve_only" in ln:
            return json.loads(ln)["mpcx_source_hash"]
    raise SystemExit(f"{log}: no profile_solve_only line with the source hash")


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "r06_solve_traffic.json")
    kf, fk, nf = timed_launch(dispatches(fdir, "FETCH_SIZE"))
    kw, wk, nw = timed_launch(dispatches(wdir, "WRITE_SIZE"))
    if kf != kw:
        raise SystemExit(f"passes disagree on the timed kernel: {kf} / {kw}")
    hf, hw = profiled_hash(fdir), profiled_hash(wdir)
    if hf != hw:
        raise SystemExit(f"passes profiled different libraries: {hf} / {hw}")
    rd, wr = 2.0 * fk * 1024, wk * 1024
    d = {"kernel": kf, "dispatches_in_timed_launch": [nf, nw], "fetch_size_kib_raw": fk, "write_size_kib_raw": wk,
         "read_bytes_corrected": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
         "command": "bench.py --profile-solve-only (default config 2 workload: warm-up steps, then the timed "
                    "20-step launch)",
         "correction": "FETCH_SIZE x2 (gfx950 counts half of the read bytes; calibrated for 8-B and 16-B per-lane "
                       "loads), WRITE_SIZE x1",
         "mpcx_source_hash": hf}
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()

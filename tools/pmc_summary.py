#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the rk4_sens sweep into profiles/rk4_sens_pmc.json.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR B N [OUT]

FETCH_DIR / WRITE_DIR hold the *_counter_collection.csv of two separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE --kernel-trace` passes over
`bench.py --profile-sweep-only`.  Corrections (MI355X_MICROARCH.md §HBM, and our
own calibration in profiles/r01_pmc_calibration.json with tools/pmc_calib.hip):
FETCH_SIZE counts exactly half of the streamed read bytes for 8-B and 16-B
per-lane loads on gfx950 -> x2; WRITE_SIZE is exact for 8-B per-lane stores.
Both counters are in KiB.
"""
import csv
import glob
import json
import os
import statistics
import sys


def values(d, counter):
    f = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if "rk4_sens" in r["Kernel_Name"] and r["Counter_Name"] == counter]


def main():
    fdir, wdir, B, N = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "rk4_sens_pmc.json")
    fk = statistics.median(values(fdir, "FETCH_SIZE"))
    wk = statistics.median(values(wdir, "WRITE_SIZE"))
    rd = 2.0 * fk * 1024
    wr = wk * 1024
    comp_rd = 8 * B * ((N + 1) * 3 + 2 * N + 3)
    comp_wr = 8 * B * 24 * N
    d = {"kernel": "rk4_sens_kernel", "B": B, "N": N, "fetch_size_kib_raw": fk, "write_size_kib_raw": wk,
         "read_bytes_corrected": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
         "compulsory_read_bytes": comp_rd, "compulsory_write_bytes": comp_wr,
         "survey_algorithmic_bytes": B * (256 * N + 48),
         "correction": "FETCH_SIZE x2 (gfx950 counts half of streamed read bytes; calibrated for 8-B and 16-B "
                       "per-lane loads), WRITE_SIZE x1"}
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()

"""FP64 flops per unit of the harness kernels from a rocprofv3 --pmc run of tools/flop_probe.py:
    python tools/flop_summary.py gpurun_out/flops [units]"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 64 * 4096
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
out = {}
for k, c in acc.items():
    name = "derivs_moments" if "stage_check" in k else "riccati_step+gains" if "riccati_check" in k else k[:40]
    lane = 64.0 / n  # wave instructions -> per-unit lane operations (one unit per lane)
    per = {t: c.get(f"SQ_INSTS_VALU_{t}_F64", 0.0) * lane for t in ("ADD", "MUL", "FMA", "TRANS")}
    out[name] = {"f64_inst_per_unit": per, "flops_per_unit": per["ADD"] + per["MUL"] + per["TRANS"] + 2 * per["FMA"]}
print(json.dumps(out, indent=1))

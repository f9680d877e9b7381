"""FP64 flops per unit of the probe kernels from a rocprofv3 --pmc run of tools/flop_probe.py:
    python tools/flop_summary.py gpurun_out/flops > profiles/r03_flop_probe.json

Dispatches are matched to tools/flop_probe.py's EVALS / RICCATI lists by launch order (the
kernel names carry only the model type, and the unicycle's two cost variants share one)."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from flop_probe import EVALS, N_UNITS, RICCATI  # noqa: E402

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else N_UNITS
disp = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        i = int(r["Dispatch_Id"])
        disp[i][r["Counter_Name"]] += float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
order = sorted(i for i in disp if "probe_kernel" in names[i])
keys = [("eval", e[0]) for e in EVALS] + [("riccati", r[0]) for r in RICCATI]
if len(order) != len(keys):
    raise SystemExit(f"expected {len(keys)} probe dispatches, found {len(order)}")
out = {"units_per_launch": n, "eval": {}, "riccati": {}}
lane = 64.0 / n  # wave instructions -> per-unit lane operations (one unit per lane)
for (kind, key), i in zip(keys, order):
    want = "eval_probe_kernel" if kind == "eval" else "riccati_probe_kernel"
    if want not in names[i]:
        raise SystemExit(f"dispatch {i} is {names[i]}, expected {want} for {key}")
    c = disp[i]
    per = {t: c.get(f"SQ_INSTS_VALU_{t}_F64", 0.0) * lane for t in ("ADD", "MUL", "FMA", "TRANS")}
    out[kind][key] = {"kernel": names[i], "f64_inst_per_unit": per,
                      "flops_per_unit": per["ADD"] + per["MUL"] + per["TRANS"] + 2 * per["FMA"]}
print(json.dumps(out, indent=1))

"""Generate the committed golden fixtures from the reference's own output files.

Run once in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

The reference ships its closed-loop results as .xlsx files written by pandas.
They are decoded here with the standard library only (zipfile + ElementTree;
openpyxl is not installed) and re-emitted as small JSON data files.  Nothing
from the reference's source code is copied: the fixtures are numbers only.

Fixture semantics (decoded from the export code):

* ``Casadi/1exemplo.xlsx`` is written at ``Casadi/multiple_shooting_casadi.py:316-334``:
  ``q = cat_states[:, 0, :].T`` (85 rows) and ``w = cat_controls.reshape((85,2))[1:]``.
  Row r >= 1 holds the state fed to solve r-1 (P[:3] of that solve); row 0 is the
  initial repmat (also the zero state).  Row r holds u0* of solve r for r = 0..83;
  row 84 repeats row 83's control.  Hence solve j (j = 0..83) maps
  ``P_j = [state row j+1 ; 10, 10, 0] -> u0*_j = control row j``.
* ``Casadi/2exemplo.xlsx`` has the same layout from ``Casadi/single_shooting_v2.py:292-301``.
* ``Casadi/3exemplo.xlsx`` (mpctools variant, ``mpctools/multiple_shooting_mpctools.py:141-150``)
  and ``Inverted_pendulum/invertpend_data_py.xlsx``
  (``Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:80-88``) are kept
  as secondary fixtures for later rows of SURVEY.md §8(f).
"""
import json
import os
import zipfile
import xml.etree.ElementTree as ET

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
NS = "{http://schemas.openxmlformats.org/spreadsheetml/2006/main}"


def read_xlsx(path):
    z = zipfile.ZipFile(path)
    shared = []
    if "xl/sharedStrings.xml" in z.namelist():
        for si in ET.fromstring(z.read("xl/sharedStrings.xml")).iter(NS + "si"):
            shared.append("".join(t.text or "" for t in si.iter(NS + "t")))
    rows = []
    for r in ET.fromstring(z.read("xl/worksheets/sheet1.xml")).iter(NS + "row"):
        row = []
        for c in r.findall(NS + "c"):
            v = c.find(NS + "v")
            if c.get("t") == "inlineStr":
                row.append("".join(t.text or "" for t in c.iter(NS + "t")))
            elif v is None:
                row.append(None)
            elif c.get("t") == "s":
                row.append(shared[int(v.text)])
            else:
                row.append(float(v.text))
        rows.append(row)
    return rows


def table(path, ncols):
    rows = read_xlsx(path)[1:]  # drop the header row (column names)
    return [[float(x) for x in r[1:1 + ncols]] for r in rows]


def main():
    fx = {}
    for name, rel in [("multiple_shooting", "Casadi/1exemplo.xlsx"),
                      ("single_shooting", "Casadi/2exemplo.xlsx"),
                      ("mpctools", "Casadi/3exemplo.xlsx")]:
        t = table(os.path.join(REF, rel), 6)
        fx[name] = {"source": rel, "columns": ["x", "y", "theta", "v", "w", "t"], "rows": t}
    with open(os.path.join(OUT, "unicycle_N10_golden.json"), "w") as f:
        json.dump(fx, f, indent=0)
    t = table(os.path.join(REF, "Inverted_pendulum/invertpend_data_py.xlsx"), 6)
    with open(os.path.join(OUT, "pendulum_N50_golden.json"), "w") as f:
        json.dump({"source": "Inverted_pendulum/invertpend_data_py.xlsx",
                   "columns": ["x1", "x2", "x3", "x4", "u", "t"], "rows": t}, f, indent=0)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()

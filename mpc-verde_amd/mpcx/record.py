"""Closed-loop records in the reference's output formats.

The reference scripts keep their closed loop in three arrays and export one table:

* ``cat_states``  (nx, N+1, iters+1): ``np.dstack`` of every solve's predicted state
  trajectory X (nx x (N+1)), seeded with the initial ``repmat(state_init)``
  (``Casadi/multiple_shooting_casadi.py:211-217,258-261``) -- what
  ``simulation_code.simulate(cat_states, cat_controls, times, T, N, reference)`` animates;
* ``cat_controls`` ((iters+1) nu, 1): ``np.vstack`` of every solve's first control u[:, 0],
  seeded with the zero initial control (``:218,263-266``);
* ``t`` (iters+1, 1): the solve times t0 (``:211,267-270``);
* the exported table (``:316-334``, written to ``1exemplo.xlsx``): x, y, theta = the first
  predicted node of every record (``cat_states[:, 0, :].T``, row 0 = the initial state,
  row r >= 1 = X_0 of solve r-1), v, w = the controls of solves 0.. (the last repeated),
  t = [0, 0, T, 2T, ..., t_last].

:class:`ClosedLoopLog` rebuilds exactly these from ``sol['x']`` vectors (interleaved
layout) so that the reference's plotting and export code runs on mpcx results unchanged.
:func:`write_xlsx` writes the table as the .xlsx pandas would (sheet "Sheet1", index
column first) with the standard library only.
"""
from __future__ import annotations

import io
import zipfile
from xml.sax.saxutils import escape

import numpy as np


def split_solution(w, nx, nu, N):
    """Reference extraction of sol['x'] (``:243-256``): (X (nx, N+1), U (nu, N))."""
    w = np.asarray(w, dtype=np.float64).reshape(-1)
    nz = nx + nu
    X = np.empty((nx, N + 1))
    U = np.empty((nu, N))
    X[:, 0] = w[0:nx]
    for k in range(N):
        U[:, k] = w[nx + nz * k: nx + nz * k + nu]
        X[:, k + 1] = w[nx + nz * k + nu: nx + nz * (k + 1)]
    return X, U


class ClosedLoopLog:
    """The bookkeeping arrays of ``Casadi/multiple_shooting_casadi.py:210-270``."""

    def __init__(self, nx, nu, N, T, x_init, t0=0.0):
        self.nx, self.nu, self.N, self.T = nx, nu, N, float(T)
        x_init = np.asarray(x_init, dtype=np.float64).reshape(nx, 1)
        self.cat_states = np.repeat(x_init, N + 1, axis=1)[:, :, None]  # DM2Arr(repmat(state_init))
        self.cat_controls = np.zeros((nu, 1))  # DM2Arr(u0[:, 0])
        self.t = np.array([[float(t0)]])
        self.times = np.array([[0.0]])

    @classmethod
    def for_ocp(cls, ocp, x_init, t0=0.0):
        return cls(ocp.nx, ocp.nu, ocp.N, ocp.T, x_init, t0)

    def record(self, w, t0, wall_time=0.0):
        """Append one solve (sol['x'] of the solve made at time t0)."""
        X, U = split_solution(w, self.nx, self.nu, self.N)
        self.cat_states = np.dstack((self.cat_states, X))
        self.cat_controls = np.vstack((self.cat_controls, U[:, 0:1]))
        self.t = np.vstack((self.t, [[float(t0)]]))
        self.times = np.vstack((self.times, [[float(wall_time)]]))

    @property
    def n_solves(self):
        return self.cat_states.shape[2] - 1

    def table(self, names=("x", "y", "theta"), unames=("v", "w")):
        """The exported table of ``:316-334`` as {column: array} (pandas-free).  The time
        column is the script's [0, arange(0, round(t_last, 1), T), t_last]; the script
        writes t_last as the literal 16.6 of its own run."""
        n = self.n_solves
        q = self.cat_states[:, 0, :].T  # (n+1, nx)
        wc = self.cat_controls.reshape((n + 1, self.nu))[1:]  # controls of solves 0..n-1
        t_last = round(float(self.t[-1, 0]), 1)
        z = np.append(0.0, np.arange(0.0, t_last, self.T))
        z = np.append(z, t_last)
        if z.shape[0] != n + 1:  # arange's float end point: fall back to the exact grid
            z = np.append(0.0, self.T * np.arange(n))
        out = {name: q[:, i] for i, name in enumerate(names)}
        for i, name in enumerate(unames):
            out[name] = np.append(wc[:, i], wc[-1, i])
        out["t"] = z
        return out

    def frame(self, **kw):
        import pandas as pd

        return pd.DataFrame(self.table(**kw))


def pendulum_table(xcl, ucl, T):
    """``Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:70-88``: xcl
    (4, nsim+1) states, ucl (1, nsim) controls -> x, x_dot, theta, theta_dot, u (0 appended), t."""
    xcl = np.asarray(xcl, float)
    ucl = np.asarray(ucl, float).reshape(-1)
    t = np.arange(xcl.shape[1]) * T
    return {"x": xcl[0], "x_dot": xcl[1], "theta": xcl[2], "theta_dot": xcl[3], "u": np.append(ucl, 0.0), "t": t}


# ---------------------------------------------------------------------------- xlsx
def _col(i):
    s = ""
    i += 1
    while i:
        i, r = divmod(i - 1, 26)
        s = chr(65 + r) + s
    return s


def write_xlsx(path_or_buf, table, sheet="Sheet1", index=True):
    """Write {column: 1-D array} as a one-sheet .xlsx laid out like ``DataFrame.to_excel``
    (header row; with index=True a leading unnamed index column 0..n-1)."""
    cols = list(table.keys())
    data = [np.asarray(table[c], dtype=np.float64) for c in cols]
    n = len(data[0]) if data else 0
    rows = []
    header = ([""] if index else []) + cols
    cells = []
    for j, h in enumerate(header):
        if h == "":
            continue
        cells.append(f'<c r="{_col(j)}1" t="inlineStr"><is><t>{escape(h)}</t></is></c>')
    rows.append(f'<row r="1">{"".join(cells)}</row>')
    for i in range(n):
        vals = ([float(i)] if index else []) + [float(d[i]) for d in data]
        cells = "".join(f'<c r="{_col(j)}{i + 2}"><v>{repr(v)}</v></c>' for j, v in enumerate(vals))
        rows.append(f'<row r="{i + 2}">{cells}</row>')
    sheet_xml = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
                 '<worksheet xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main">'
                 f'<sheetData>{"".join(rows)}</sheetData></worksheet>')
    files = {
        "[Content_Types].xml": (
            '<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
            '<Types xmlns="http://schemas.openxmlformats.org/package/2006/content-types">'
            '<Default Extension="rels" ContentType="application/vnd.openxmlformats-package.relationships+xml"/>'
            '<Default Extension="xml" ContentType="application/xml"/>'
            '<Override PartName="/xl/workbook.xml" '
            'ContentType="application/vnd.openxmlformats-officedocument.spreadsheetml.sheet.main+xml"/>'
            '<Override PartName="/xl/worksheets/sheet1.xml" '
            'ContentType="application/vnd.openxmlformats-officedocument.spreadsheetml.worksheet+xml"/>'
            '</Types>'),
        "_rels/.rels": (
            '<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
            '<Relationships xmlns="http://schemas.openxmlformats.org/package/2006/relationships">'
            '<Relationship Id="rId1" '
            'Type="http://schemas.openxmlformats.org/officeDocument/2006/relationships/officeDocument" '
            'Target="xl/workbook.xml"/></Relationships>'),
        "xl/workbook.xml": (
            '<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
            '<workbook xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main" '
            'xmlns:r="http://schemas.openxmlformats.org/officeDocument/2006/relationships">'
            f'<sheets><sheet name="{escape(sheet)}" sheetId="1" r:id="rId1"/></sheets></workbook>'),
        "xl/_rels/workbook.xml.rels": (
            '<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
            '<Relationships xmlns="http://schemas.openxmlformats.org/package/2006/relationships">'
            '<Relationship Id="rId1" '
            'Type="http://schemas.openxmlformats.org/officeDocument/2006/relationships/worksheet" '
            'Target="worksheets/sheet1.xml"/></Relationships>'),
        "xl/worksheets/sheet1.xml": sheet_xml,
    }
    own = isinstance(path_or_buf, (str, bytes)) or hasattr(path_or_buf, "__fspath__")
    buf = open(path_or_buf, "wb") if own else path_or_buf
    try:
        with zipfile.ZipFile(buf, "w", zipfile.ZIP_DEFLATED) as z:
            for name, text in files.items():
                z.writestr(name, text)
    finally:
        if own:
            buf.close()


def xlsx_bytes(table, **kw):
    b = io.BytesIO()
    write_xlsx(b, table, **kw)
    return b.getvalue()

"""Output and diagnostics around the time step: the reference driver's host code
(SURVEY.md §8f, row f2), restated for the engine's state.

    layer_fields       diagnostics.F90:24-45          h, u, v, dp and interface elevation per layer
    conserved_mass     compute_conserved.F90:7-45     layer mass
    courant            courant.F90:9-127              CFL_B, CFL and the dx/dy minima
    print_diagnostics  print_diagnostics.F90:14-190   stdout report, mass_mlswe.cons line, mlswe_FIN.txt
    write_snapshot     diagnostics.F90:58-92          the `mlswe####` text snapshot
    read_snapshot      mod_restart.F90:260-294        its reader (load_data_mlswe)
    restart_state      mod_restart.F90:15-87          q_df, qb_df, qprime_df from a snapshot
    time_loop          mod_time_loop.F90:61-269       the loop around ti_rk_bcl
    ci_check           CI/bump/check.F90:1-86         the reference CI's acceptance check

All of it is host code on the state copied out of the engine (hnumo_sync); none of it is on
the timed path.  Single rank: the reference's gathers (gather_data) are the identity.
Fortran edit descriptors (Iw, Ew.d, ESw.d, Dw.d) are reproduced so that the files read like
the reference's for the same state (tests/test_diagnostics.py).
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np


# ------------------------------------------------------------------ Fortran edit descriptors
def _special(x: float, w: int) -> str:
    s = "NaN" if math.isnan(x) else ("-Infinity" if x < 0 else "Infinity")
    return s.rjust(w) if len(s) <= w else "*" * w


def _sign(x: float) -> str:
    return "-" if math.copysign(1.0, x) < 0 else ""


def _exponent(e: int, letter: str) -> str:
    s = "+" if e >= 0 else "-"
    return f"{letter}{s}{abs(e):02d}" if abs(e) <= 99 else f"{s}{abs(e):03d}"


def fmt_e(x: float, w: int, d: int, letter: str = "E") -> str:
    """Fortran Ew.d (letter 'D': Dw.d): [-]0.d...dE+xx, right-justified in w columns,
    correctly rounded to d digits."""
    x = float(x)
    if not math.isfinite(x):
        return _special(x, w)
    if x == 0.0:
        digits, e = "0" * d, 0
    else:
        m, ex = f"{abs(x):.{d - 1}e}".split("e")
        digits, e = m.replace(".", ""), int(ex) + 1
    s = _sign(x) + "0." + digits + _exponent(e, letter)
    if len(s) > w:
        s = _sign(x) + "." + digits + _exponent(e, letter)  # the optional leading zero goes first
    return s.rjust(w) if len(s) <= w else "*" * w


def fmt_es(x: float, w: int, d: int) -> str:
    """Fortran ESw.d: [-]d.d...dE+xx."""
    x = float(x)
    if not math.isfinite(x):
        return _special(x, w)
    m, ex = f"{abs(x):.{d}e}".split("e")
    s = _sign(x) + m + _exponent(int(ex), "E")
    return s.rjust(w) if len(s) <= w else "*" * w


def fmt_i(i: int, w: int) -> str:
    s = str(int(i))
    return s.rjust(w) if len(s) <= w else "*" * w


# ------------------------------------------------------------------ fields and diagnostics
def layer_fields(case, q_df):
    """q(5,npoin,nlayers) of diagnostics.F90:24-45: h = (alpha_k/g) dp_k, u_k, v_k, dp_k and
    the elevation of each layer's top interface (zbot plus the thicknesses below, :31-45)."""
    A, S = case.arrays, case.scalars
    L, g, npoin = S["nlayers"], S["gravity"], S["npoin"]
    q = np.zeros((5, npoin, L), order="F")
    for k in range(L):
        q[0, :, k] = (A["alpha"][k] / g) * q_df[0, :, k]
        q[1, :, k] = q_df[1, :, k] / q_df[0, :, k]
        q[2, :, k] = q_df[2, :, k] / q_df[0, :, k]
        q[3, :, k] = q_df[0, :, k]
    elev = np.zeros((npoin, L + 1), order="F")
    elev[:, L] = A["zbot_df"]
    for k in range(L - 1, -1, -1):
        elev[:, k] = elev[:, k + 1] + q[0, :, k]
    q[4] = elev[:, :L]
    return q


def conserved_mass(case, h) -> float:
    """compute_conserved (compute_conserved.F90:7-45): sum over the nodes, in node order, of
    wjac_df*psih_df*h.  psih_df is the identity at the LGL nodes, so node I adds wjac_df(I)*h(I)
    and the other terms add exact zeros; the running sum is sequential (np.add.accumulate)."""
    w = case.arrays.get("wjac_df")
    if w is None:
        w = case.arrays["jac"]
    terms = np.asarray(w, dtype=np.float64).reshape(-1, order="F") * np.asarray(h, dtype=np.float64)
    return float(np.add.accumulate(terms)[-1]) if terms.size else 0.0


def courant(case, qf, qb):
    """courant_cube_mlswe (courant.F90:34-127): velocities averaged over the 4 corners of each
    sub-cell of the LGL grid against the running minimum cell size.  Returns
    (cfl_b, cfl, min_dx, min_dy)."""
    A, S = case.arrays, case.scalars
    ngl, E, L = S["ngl"], S["nelem"], S["nlayers"]
    P, nc = ngl * ngl, max(ngl - 1, 1)
    e = np.arange(E)[:, None, None]
    j = np.arange(nc)[None, :, None]
    i = np.arange(nc)[None, None, :]
    ii, jj = np.minimum(i + 1, ngl - 1), np.minimum(j + 1, ngl - 1)
    corners = [e * P + j * ngl + i, e * P + j * ngl + ii, e * P + jj * ngl + i, e * P + jj * ngl + ii]
    corners = [np.broadcast_to(c, (E, nc, nc)).reshape(-1) for c in corners]
    coord = A["coord"]
    x = np.stack([coord[0, c] for c in corners])
    y = np.stack([coord[1, c] for c in corners])
    min_dx = np.minimum.accumulate(np.concatenate([[1e16], x.max(0) - x.min(0)]))[1:]
    min_dy = np.minimum.accumulate(np.concatenate([[1e16], y.max(0) - y.min(0)]))[1:]

    def avg(f):
        s = np.zeros(corners[0].size)
        for c in corners:
            s = s + f[c] / 4.0
        return s

    cfl_b = max(-1.0e10, float(np.max(np.abs(avg(qb[2])) * S["dt_btp"] / min_dx)),
                float(np.max(np.abs(avg(qb[3])) * S["dt_btp"] / min_dy)))
    cfl = -1.0e10
    for k in range(L):
        cfl = max(cfl, float(np.max(np.abs(avg(qf[1, :, k])) * S["dt"] / min_dx)),
                  float(np.max(np.abs(avg(qf[2, :, k])) * S["dt"] / min_dy)))
    return cfl_b, cfl, float(min_dx[-1]), float(min_dy[-1])


FIELD_NAMES = ("h", "u", "v", "dp", "ssh")
_RULE = " " + "=" * 63
_DASH = " " + "-" * 63


def fin_text(mass_loss, qmax, qmin) -> str:
    """mlswe_FIN.txt (print_diagnostics.F90:167-184) from the per-layer mass loss and the
    max/min of the 5 layer fields (qmax/qmin: (5, nlayers)); dp (field 4) is not written."""
    lines = []
    for k in range(qmax.shape[1]):
        lines.append("Layer = " + fmt_i(k + 1, 8))
        lines.append("Mass Loss  = " + fmt_e(mass_loss[k], 16, 8))
        for i in range(5):
            if i != 3:
                lines.append("Fields:   Max/Min = " + FIELD_NAMES[i].ljust(3) + " " + fmt_e(qmax[i, k], 24, 12) +
                             " " + fmt_e(qmin[i, k], 24, 12))
    return "\n".join(lines) + "\n"


def print_diagnostics(case, qf, qb, time, itime, idone, mass0=None, time_scale=1.0):
    """print_diagnostics_mlswe (print_diagnostics.F90:14-190) for the layer fields `qf`
    (layer_fields) and qb(4,npoin).  Returns (stdout text, mass_mlswe.cons line or None,
    mlswe_FIN.txt text or None).  mass0: the initial layer masses (lcheck_conserved)."""
    S = case.scalars
    L = S["nlayers"]
    mass, xm1 = None, [0.0] * L
    if mass0 is not None:
        mass = [conserved_mass(case, qf[0, :, k]) for k in range(L)]
        xm1 = [abs(mass[k] - mass0[k]) / mass0[k] for k in range(L)]
    qmax, qmin = qf.max(axis=1), qf.min(axis=1)
    qbmax, qbmin = qb.max(axis=1), qb.min(axis=1)
    cfl_b, cfl, dxm, dym = courant(case, qf, qb)
    head = "itime time dt dt_btp = " + fmt_i(itime, 8) + " " + " ".join(
        fmt_es(v, 13, 5) for v in (time / time_scale, S["dt"], S["dt_btp"]))
    cfl_line = "CFL_B = " + fmt_e(cfl_b, 11, 4) + " CFL = " + fmt_e(cfl, 11, 4)
    q_line = lambda tag, i, a, b: f"{tag}: i    Max/Min = " + fmt_i(i + 1, 3) + " " + fmt_e(a, 24, 12) + " " + fmt_e(b, 24, 12)
    cons = fin = None
    if idone == 0:
        if mass is not None:
            cons = fmt_i(itime, 8) + " ".join(fmt_e(m, 16, 8) for m in mass)
        out = [_RULE, head, cfl_line, "dx_min = " + fmt_e(dxm, 11, 4) + " dy_min = " + fmt_e(dym, 11, 4), _DASH]
        for k in range(L):
            out += ["Layer = " + fmt_i(k + 1, 8), "Mass Loss   = " + fmt_e(xm1[k], 22, 8)]
            out += [q_line("Q", i, qmax[i, k], qmin[i, k]) for i in range(5)] + [_DASH]
        out += [_DASH, " Barotropic"] + [q_line("Qb", i, qbmax[i], qbmin[i]) for i in range(4)] + [_RULE]
    else:
        out = [_DASH, " **Simulation Finished**", head, cfl_line, _DASH]
        for k in range(L):
            out += ["Layer = " + fmt_i(k + 1, 8), "Mass Loss  = " + fmt_e(xm1[k], 16, 8)]
            out += [q_line("Q", i, qmax[i, k], qmin[i, k]) for i in range(5)] + [_DASH]
        fin = fin_text(xm1, qmax, qmin)
    return "\n".join(out) + "\n", cons, fin


# ------------------------------------------------------------------ snapshots and restart
def write_snapshot(path, case, q_df, qb):
    """The `mlswe####` text snapshot of diagnostics.F90:58-92, one value per record."""
    S, A = case.scalars, case.arrays
    qf = layer_fields(case, q_df)

    def D(a):
        return [fmt_e(v, 23, 16, "D") for v in np.asarray(a, dtype=np.float64).ravel(order="F")]

    lines = [fmt_i(S["nlayers"], 4), fmt_i(S["npoin"], 10)] + D([S["dt"]]) + D([S["dt_btp"]])
    lines += D(A["coord"][0:2, :])
    lines += D(qb[0]) + D(qb[2]) + D(qb[3])
    for c in (0, 1, 2, 4):
        lines += D(qf[c])
    lines += D(A["zbot_df"])
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def read_snapshot(path) -> dict:
    """load_data_mlswe (mod_restart.F90:260-294): list-directed read of a snapshot."""
    tok = open(path).read().replace("D", "E").replace("d", "e").split()
    nk, npoin = int(tok[0]), int(tok[1])
    v = np.array(tok[2:], dtype=np.float64)
    out = {"nlayers": nk, "npoin": npoin, "dt": v[0], "dt_btp": v[1]}
    o = 2
    out["coord"] = v[o:o + 2 * npoin].reshape(2, npoin, order="F")
    o += 2 * npoin
    out["qb"] = v[o:o + 3 * npoin].reshape(3, npoin)          # rows: qb(1), qb(3), qb(4)
    o += 3 * npoin
    q = np.zeros((3, npoin, nk), order="F")
    for c in range(3):
        q[c] = v[o:o + npoin * nk].reshape(npoin, nk, order="F")
        o += npoin * nk
    out["q"] = q                                              # h, u, v
    out["z"] = v[o:o + npoin * (nk + 1)].reshape(npoin, nk + 1, order="F")
    return out


def restart_state(case, path):
    """restart_mlswe (mod_restart.F90:15-65): (q_df, qb_df, qprime_df) from a snapshot."""
    A, S = case.arrays, case.scalars
    r = read_snapshot(path)
    L, g, npoin = S["nlayers"], S["gravity"], S["npoin"]
    if r["nlayers"] != L or r["npoin"] != npoin:
        raise ValueError(f"{path}: snapshot is {r['nlayers']} layers x {r['npoin']} points")
    pb = A["pbprime_df"]
    qb = np.zeros((4, npoin), order="F")
    qb[0] = r["qb"][0]
    qb[2:4] = r["qb"][1:3]
    qb[1] = qb[0] - pb
    q = np.zeros((3, npoin, L), order="F")
    for k in range(L):
        q[0, :, k] = (g / A["alpha"][k]) * r["q"][0, :, k]
        q[1, :, k] = r["q"][1, :, k] * q[0, :, k]
        q[2, :, k] = r["q"][2, :, k] * q[0, :, k]
    ope = q[0, :, 0].copy()
    for k in range(1, L):
        ope = ope + q[0, :, k]
    ope = ope / pb
    qp = np.zeros((3, npoin, L), order="F")
    for k in range(L):
        qp[0, :, k] = q[0, :, k] / ope
        qp[1, :, k] = q[1, :, k] / q[0, :, k] - qb[2] / qb[0]
        qp[2, :, k] = q[2, :, k] / q[0, :, k] - qb[3] / qb[0]
    return q, qb, qp


# ------------------------------------------------------------------ the time loop
def time_loop(case, stepper, time_final, *, out_dir=".", dump_data=False, time_restart=None,
              lcheck_conserved=True, lprint_diagnostics=True, time_initial=0.0, restart_file_number=0,
              time_scale=1.0, out=None):
    """mod_time_loop.F90:61-269 around stepper.ti_rk_bcl (a hnumo.engine.Engine, resident, or
    in tests the CPU oracle).  Writes the mlswe#### snapshots (dump_data, every
    nint(time_restart/dt) steps), mass_mlswe.cons (lcheck_conserved) and mlswe_FIN.txt into
    out_dir; the stdout report goes to `out` (default sys.stdout).  Returns the final
    (q_df, qb_df, qprime_df)."""
    S = case.scalars
    out = out or sys.stdout
    dt = S["dt"]
    os.makedirs(out_dir, exist_ok=True)
    snap = lambda n: os.path.join(out_dir, f"mlswe{n:04d}")
    q, qb, qp = (np.array(case.arrays[k], order="F") for k in ("q_df", "qb_df", "qprime_df"))
    itime = inorm = 0
    irestart = int(math.floor((time_restart if time_restart is not None else dt) / dt + 0.5)) or 1
    time = time_initial
    qout = None
    if time_initial == 0:
        if dump_data:
            write_snapshot(snap(0), case, q, qb)
            qout = layer_fields(case, q)
    else:
        itime = inorm = restart_file_number
        q, qb, qp = restart_state(case, snap(restart_file_number))
    mass0, cons = None, None
    if lcheck_conserved:
        if qout is None:
            qout = layer_fields(case, q)
        mass0 = [conserved_mass(case, qout[0, :, k]) for k in range(S["nlayers"])]
        cons = open(os.path.join(out_dir, "mass_mlswe.cons"), "w")
    if qout is None:
        qout = layer_fields(case, q)

    def report(idone):
        text, line, fin = print_diagnostics(case, qout, qb, time, itime, idone, mass0, time_scale)
        out.write(text)
        if line is not None and cons is not None:
            cons.write(line + "\n")
        if fin is not None:
            with open(os.path.join(out_dir, "mlswe_FIN.txt"), "w") as fh:
                fh.write(fin)

    if lprint_diagnostics:
        report(0)
    resident = hasattr(stepper, "set_resident")
    if resident:
        stepper.set_resident(True)
    while time < time_final:
        itime += 1
        time = time + dt
        stepper.ti_rk_bcl(q, qb, qp)
        if itime % irestart == 0 and dump_data:
            if resident:
                stepper.sync(q, qb, qp)
            inorm += 1
            write_snapshot(snap(inorm), case, q, qb)
            qout = layer_fields(case, q)
            if lprint_diagnostics:
                report(0)
    if resident:
        stepper.sync(q, qb, qp)
    if cons is not None:
        cons.close()
        cons = None
    if not dump_data:
        qout = layer_fields(case, q)
    report(1)
    return q, qb, qp


# ------------------------------------------------------------------ the reference CI check
def ci_check(fin_text_run: str, fin_text_ref: str, nlayers: int = 2, nfield: int = 4, tol: float = 1e-12):
    """CI/bump/check.F90: per layer the run's mass loss must be <= 1e-12 (:56-62); the relative
    differences of the h/u/v max and min against the reference file are reported (:64-80).
    Returns (ok, {layer: {"mass_loss": x, "h": (err_max, err_min), ...}})."""
    run, ref = fin_text_run.splitlines(), fin_text_ref.splitlines()
    ok, rep = True, {}
    for nl in range(nlayers):
        il = 6 * nl
        ml = float(run[il + 1].split("=")[1])
        ok = ok and ml <= tol
        r = {"mass_loss": ml}
        for ifield in range(2, nfield + 1):
            a, b = run[il + ifield].split(), ref[il + ifield].split()
            r[a[3]] = (abs(float(b[4]) - float(a[4])) / abs(float(b[4])), abs(float(b[5]) - float(a[5])) / abs(float(b[5])))
        rep[nl + 1] = r
    return ok, rep

"""1-D Legendre-Gauss-Lobatto (LGL) bases used by the DG engine.

Host-side setup (not on the hot path).  The arithmetic restates the reference's
basis construction operation for operation so the tables agree bitwise:

* ``lgl``             -> ``legendre_gauss_lobatto`` (mod_legendre.F90:54-111) and
                         ``legendre_poly_loc`` (mod_legendre.F90:188-236)
* ``legendre_basis``  -> ``legendre_basis`` with ``reduce_round_off = .true.``
                         (mod_legendre.F90:246-317)
* ``lagrange_basis``  -> ``lagrange_basis`` (mod_legendre.F90:387-433): the nodal
                         basis on ``ngl`` LGL nodes evaluated at ``nq = 2N+1`` LGL
                         quadrature points (mod_basis.F90:84-87, ``dg_integ_exact``).

Arrays follow the reference's index convention: ``psiq[i, l]`` is node ``i`` at
quadrature point ``l`` (0-based here, 1-based in Fortran).
"""
from __future__ import annotations

import math

import numpy as np

_EPS = np.finfo(np.float64).eps  # thres = epsilon(1.0_rQ), mod_legendre.F90:11


def _legendre_poly(n: int, x: float):
    """Legendre P_n and its first two derivatives at x (mod_legendre.F90:188-236)."""
    p2 = p2_1 = p2_2 = 0.0
    p1 = p1_1 = p1_2 = 0.0
    p0, p0_1, p0_2 = 1.0, 0.0, 0.0
    for j in range(1, n + 1):
        p2, p2_1, p2_2 = p1, p1_1, p1_2
        p1, p1_1, p1_2 = p0, p0_1, p0_2
        a = (2.0 * float(j) - 1.0) / float(j)
        b = (float(j) - 1.0) / float(j)
        p0 = a * x * p1 - b * p2
        p0_1 = a * (p1 + x * p1_1) - b * p2_1
        p0_2 = a * (2.0 * p1_1 + x * p1_2) - b * p2_2
    return p0, p0_1, p0_2


def lgl(ngl: int):
    """LGL nodes and weights (mod_legendre.F90:54-111)."""
    xgl = np.zeros(ngl)
    wgl = np.zeros(ngl)
    if ngl == 1:
        xgl[0] = 0.0
        wgl[0] = 2.0
        return xgl, wgl
    pi = 4.0 * math.atan(1.0)
    n = ngl - 1
    nh = (n + 1) // 2
    p0 = 0.0
    for i in range(1, nh + 1):
        x = math.cos((2.0 * i - 1.0) / (2.0 * n + 1.0) * pi)
        for _ in range(20):
            p0, p0_1, p0_2 = _legendre_poly(n, x)
            dx = -(1.0 - x ** 2) * p0_1 / (-2.0 * x * p0_1 + (1.0 - x ** 2) * p0_2)
            x = x + dx
            if abs(dx) < _EPS:
                break
        xgl[n + 1 - i] = x
        wgl[n + 1 - i] = 2.0 / (float(n * (n + 1)) * p0 ** 2)
    if n + 1 != 2 * nh:
        x = 0.0
        p0, _, _ = _legendre_poly(n, x)
        xgl[nh] = x
        wgl[nh] = 2.0 / (float(n * (n + 1)) * p0 ** 2)
    for i in range(1, nh + 1):
        xgl[i - 1] = -xgl[n + 1 - i]
        wgl[i - 1] = +wgl[n + 1 - i]
    return xgl, wgl


def legendre_basis(ngl: int, xgl: np.ndarray):
    """Nodal cardinal basis and derivative at the LGL nodes (reduce_round_off path).

    Returns ``psi[i, j]`` (identity) and ``dpsi[i, j]`` = d psi_i / dx at node j.
    """
    psi = np.zeros((ngl, ngl))
    dpsi = np.zeros((ngl, ngl))
    bb = np.zeros(ngl)
    cc = np.zeros(ngl)
    for j in range(ngl):
        xj = xgl[j]
        for i in range(ngl):
            ksi = xgl[i]
            if i == j:
                psi[i, j] = 1.0
            else:
                bb[j] = bb[j] + math.log(abs(xj - ksi))
    for j in range(ngl):
        xj = xgl[j]
        for i in range(ngl):
            ksi = xgl[i]
            if i != j:
                # (-1)**(j+i) with Fortran 1-based i, j: parity unchanged by the shift
                sgn = -1.0 if ((i + j) % 2) else 1.0
                dpsi[i, j] = sgn * math.exp(bb[j] - bb[i]) / (xj - ksi)
                cc[j] = cc[j] + dpsi[i, j]
    for j in range(ngl):
        dpsi[j, j] = -cc[j]
    return psi, dpsi


def lagrange_basis(ngl: int, xgl: np.ndarray, nq: int):
    """Nodal basis on ``ngl`` nodes evaluated at ``nq`` LGL points (mod_legendre.F90:387-433)."""
    xnq, wnq = lgl(nq)
    psiq = np.zeros((ngl, nq))
    dpsiq = np.zeros((ngl, nq))
    for l in range(nq):
        xl = xnq[l]
        for i in range(ngl):
            ksi = xgl[i]
            p = 1.0
            d = 0.0
            for j in range(ngl):
                xj = xgl[j]
                if j != i:
                    p = p * (xl - xj) / (ksi - xj)
                ddpsi = 1.0
                if j != i:
                    for k in range(ngl):
                        xk = xgl[k]
                        if k != i and k != j:
                            ddpsi = ddpsi * (xl - xk) / (ksi - xk)
                    d = d + ddpsi / (ksi - xj)
            psiq[i, l] = p
            dpsiq[i, l] = d
    return xnq, wnq, psiq, dpsiq


class Basis:
    """All 1-D tables for polynomial order N (ngl = N+1, nq = 2N+1)."""

    def __init__(self, nop: int):
        self.nop = nop
        self.ngl = nop + 1
        self.nq = 2 * nop + 1
        self.xgl, self.wgl = lgl(self.ngl)
        self.psi, self.dpsi = legendre_basis(self.ngl, self.xgl)
        self.xnq, self.wnq, self.psiq, self.dpsiq = lagrange_basis(self.ngl, self.xgl, self.nq)

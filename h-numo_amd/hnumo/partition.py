"""Element partition of a brick case over ranks with a one-element ghost layer.

Rank r owns a contiguous block of the brick (rank grid px x py).  Its local
mesh is its owned elements (first, in global order) followed by a ghost copy of every
neighbouring element that shares a face with an owned element (in global order).  Local
faces are every global face touching a local element, in global face order, so each
element sees its faces in the same order as on one rank and every face keeps its global
orientation: the arithmetic of an owned element is the single-rank arithmetic, bit for
bit.  Faces between a ghost and a non-local element become inert walls (`-4`) that only
ghost elements touch; ghost results are never used -- the engine refreshes ghost data from
the owning rank at every point where a kernel reads across an element boundary
(csrc/engine.hip, `exchange`).

The halo lists per neighbour rank: `send` = local ids of owned elements the neighbour holds
as ghosts, `recv` = local ids of ghosts that neighbour owns; both in global element order, so
rank a's send list to b and rank b's recv list from a name the same elements in the same order.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .case import Case

# arrays by index kind
_NODE = ["massinv", "pbprime_df", "one_over_pbprime_df", "zbot_df", "fdt2_bcl", "a_bcl", "b_bcl", "wjac_df"]
_NODE_C = ["q_df", "qb_df", "qprime_df", "coord"]              # (ncomp, npoin[, L])
_QUAD = ["pbprime", "one_over_pbprime", "coriolis_quad", "wjac"]
_QUAD_C = ["tau_wind", "grad_zbot_quad"]                        # (2, npoin_q)
_ELEM = ["ksiq_x", "ksiq_y", "etaq_x", "etaq_y", "jacq", "ksi_x", "ksi_y", "eta_x", "eta_y", "jac"]
_FACE_LAST = ["imapl", "imapr", "imapl_q", "imapr_q", "normal_vector", "normal_vector_q", "jac_face", "jac_faceq", "pbprime_face",
              "pbprime_df_face", "one_over_pbprime_edge", "coeff_pbpert_L", "coeff_pbpert_R", "coeff_pbub_LR",
              "coeff_mass_pbub_L", "coeff_mass_pbub_R", "coeff_mass_pbpert_LR", "zbot_face"]
_DENSE_Q = ["psih", "dpsidx", "dpsidy"]                         # (P, npoin_q)
_DENSE_N = ["dpsidx_df", "dpsidy_df"]                           # (P, npoin)
_GLOBAL = ["alpha", "ssprk_a", "ssprk_beta", "psiq", "dpsiq", "psi", "dpsi", "wgl", "wnq"]


@dataclass
class Neighbour:
    rank: int
    send: np.ndarray    # local 0-based owned element ids, global order
    recv: np.ndarray    # local 0-based ghost element ids, global order


@dataclass
class RankCase(Case):
    rank: int = 0
    nranks: int = 1
    nelem_owned: int = 0
    elems: np.ndarray = None          # global 0-based element id of each local element
    faces: np.ndarray = None          # global 0-based face id of each local face
    neighbours: list = field(default_factory=list)

    def owned_nodes(self):
        """Local node slice of the owned elements (they come first)."""
        P = self.scalars["ngl"] ** 2
        return slice(0, self.nelem_owned * P)


def rank_grid(nranks: int):
    """px x py rank grid for a brick: 1x1, 2x1, 2x2, 4x2, ..."""
    px, py = 1, 1
    while px * py < nranks:
        if px <= py:
            px *= 2
        else:
            py *= 2
    if px * py != nranks:
        raise ValueError(f"nranks={nranks} must be a power of two")
    return px, py


def element_owner(nelx: int, nely: int, px: int, py: int) -> np.ndarray:
    if nelx % px or nely % py:
        raise ValueError(f"{nelx}x{nely} elements do not split over a {px}x{py} rank grid")
    bx, by = nelx // px, nely // py
    g = np.arange(nelx * nely)
    return (g % nelx) // bx + ((g // nelx) // by) * px


def _ghosts(owned_mask, el, er):
    inner = er > 0
    a, b = el[inner], er[inner] - 1
    gh = set(b[owned_mask[a] & ~owned_mask[b]].tolist()) | set(a[owned_mask[b] & ~owned_mask[a]].tolist())
    return np.array(sorted(gh), dtype=np.int64)


def partition(case: Case, nranks: int, rank: int) -> RankCase:
    mesh, A, S = case.mesh, case.arrays, case.scalars
    px, py = rank_grid(nranks)
    owner = element_owner(mesh.nelx, mesh.nely, px, py)
    face = np.asarray(A["face"])
    el = face[6].astype(np.int64) - 1
    er = face[7].astype(np.int64)
    owned = np.flatnonzero(owner == rank)
    ghosts = _ghosts(owner == rank, el, er)
    elems = np.concatenate([owned, ghosts])
    g2l = -np.ones(owner.size, dtype=np.int64)
    g2l[elems] = np.arange(elems.size)
    erg = np.where(er > 0, er - 1, -1)
    l_in = g2l[el] >= 0
    r_in = (erg >= 0) & (g2l[np.maximum(erg, 0)] >= 0)
    faces = np.flatnonzero(l_in | r_in)

    ngl, nq = S["ngl"], S["nq"]
    P, Q = ngl * ngl, nq * nq
    nodes = (elems[:, None] * P + np.arange(P)[None, :]).ravel()
    quads = (elems[:, None] * Q + np.arange(Q)[None, :]).ravel()
    B = {}
    for k in _NODE:
        if k in A:
            B[k] = np.asfortranarray(np.asarray(A[k])[nodes])
    for k in _NODE_C:
        if k in A:
            B[k] = np.asfortranarray(np.asarray(A[k])[:, nodes, ...])
    for k in _QUAD:
        if k in A:
            B[k] = np.asfortranarray(np.asarray(A[k])[quads])
    for k in _QUAD_C:
        B[k] = np.asfortranarray(np.asarray(A[k])[:, quads])
    for k in _ELEM:
        B[k] = np.asfortranarray(np.asarray(A[k])[..., elems])
    for k in _FACE_LAST:
        B[k] = np.array(np.asarray(A[k])[..., faces], order="F")
    for k in _GLOBAL:
        B[k] = np.asarray(A[k])
    if "psih" in A:
        for k in _DENSE_Q:
            B[k] = np.asfortranarray(np.asarray(A[k])[:, quads])
        for k in _DENSE_N:
            B[k] = np.asfortranarray(np.asarray(A[k])[:, nodes])
        n = elems.size
        B["indexq"] = np.asfortranarray(np.repeat((np.arange(n)[:, None] * P + np.arange(P)[None, :] + 1).T, Q, axis=1)
                                        .astype(np.int32))
        B["index_df"] = np.asfortranarray(np.repeat((np.arange(n)[:, None] * P + np.arange(P)[None, :] + 1).T, P, axis=1)
                                          .astype(np.int32))

    # local face array: global orientation kept; faces leaving the local mesh become walls
    lf = np.zeros((8, faces.size), dtype=np.int32, order="F")
    lf[4] = face[4, faces]
    lf[5] = face[5, faces]
    fl, fr = el[faces], erg[faces]
    lin, rin = l_in[faces], r_in[faces]
    lf[6] = np.where(lin, g2l[fl] + 1, 0)
    lf[7] = np.where(er[faces] <= 0, er[faces], np.where(rin, g2l[np.maximum(fr, 0)] + 1, -4))
    flip = ~lin                                    # only the (ghost) right element is local
    if flip.any():
        lf[6, flip] = g2l[fr[flip]] + 1
        lf[7, flip] = -4
        lf[4, flip] = face[5, faces[flip]]
        lf[5, flip] = 0
        for a, b in (("imapl", "imapr"), ("imapl_q", "imapr_q")):
            B[a][..., flip] = B[b][..., flip]
            B[b][..., flip] = 0
        for k in ("normal_vector", "normal_vector_q"):
            B[k][..., flip] = -B[k][..., flip]
        for k in ("pbprime_face", "pbprime_df_face", "zbot_face"):
            B[k][:, :, flip] = B[k][::-1][:, :, flip]
        for a, b in (("coeff_pbpert_L", "coeff_pbpert_R"), ("coeff_mass_pbub_L", "coeff_mass_pbub_R")):
            B[a][:, flip], B[b][:, flip] = B[b][:, flip].copy(), B[a][:, flip].copy()
    wall_r = (~rin) & (er[faces] > 0) & lin         # left local, right not local: wall on the ghost
    if wall_r.any():
        lf[5, wall_r] = 0
        B["imapr"][..., wall_r] = 0
        B["imapr_q"][..., wall_r] = 0
    B["face"] = lf

    # halo lists
    neighbours = []
    for r in range(nranks):
        if r == rank:
            continue
        gh_r = set(_ghosts(owner == r, el, er).tolist())
        send = np.array([g2l[g] for g in owned if g in gh_r], dtype=np.int64)
        recv = np.array([g2l[g] for g in ghosts if owner[g] == r], dtype=np.int64)
        if send.size or recv.size:
            neighbours.append(Neighbour(r, send, recv))

    sc = dict(S)
    sc.update(nelem=int(elems.size), npoin=int(elems.size * P), npoin_q=int(elems.size * Q), nface=int(faces.size))
    return RankCase(cfg=case.cfg, basis=case.basis, mesh=None, arrays=B, scalars=sc, rank=rank, nranks=nranks,
                    nelem_owned=int(owned.size), elems=elems, faces=faces, neighbours=neighbours)


def gather_owned(parts, name, global_case):
    """Reassemble a nodal state array (ncomp, npoin[, L]) from the owned parts of each rank."""
    A = np.asarray(global_case.arrays[name])
    out = np.zeros_like(A)
    P = global_case.scalars["ngl"] ** 2
    for pc, arr in parts:
        own = pc.elems[:pc.nelem_owned]
        gn = (own[:, None] * P + np.arange(P)[None, :]).ravel()
        out[:, gn, ...] = np.asarray(arr)[:, :pc.nelem_owned * P, ...]
    return out

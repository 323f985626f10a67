"""Partition of a brick case with the reference's own halo contract: PROCESSOR FACES.

This is how h-NUMO itself partitions (p4est.c:1600-1720 -> mod_p4est / mod_parallel), and
what a multi-rank h-NUMO run hands to ti_rk_bcl:

* a rank holds only its own elements (no ghosts), numbered in its local order;
* a face shared with another rank is a *processor face*: the local element is the left
  element (face(7)), face(8) = 0, face(6) = 0, normals point out of the local element
  (p4est.c:1686-1692, face_type = 2);
* per neighbour rank (mod_parallel num_nbh, nbh_proc 1-based, num_send_recv) the list
  nbh_send_recv of 1-based local face ids shared with it, in an order both ranks agree on
  (p4est sorts the shared faces in a global ordering, p4est.c:1375-1412);
* face traces travel as the sender's side-1 values of each listed face and land in side 2 of
  the receiver's copy, node n to node n (send_receive_bound.F90:272-327 pack,
  create_rhs_dynamics_flux.F90:104-182 unpack), so the two copies of a shared face list its
  nodes in the same physical order.

Element orders: ``order="block"`` gives each rank a px x py block of the brick (local order =
global row-major order); ``order="morton"`` splits the Morton (Z-order) curve of the brick into
nranks contiguous chunks and numbers each rank's elements along the curve, as p4est does.
Shared faces are listed by global face id (a key both sides share).

The arithmetic of a processor face is the reference's multi-rank arithmetic: each rank
evaluates the shared face in its own orientation from its own side and the received side, so
a partitioned run matches the reference Fortran/MPI run on the same partition (pinned by
tests/golden/*_mpi*.npz from oracle/_ref/ref_driver under mpiexec), not the single-rank run
bit for bit (that is the ghost-element partition of hnumo/partition.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .case import Case
from .partition import (_DENSE_N, _DENSE_Q, _ELEM, _FACE_LAST, _GLOBAL, _NODE, _NODE_C, _QUAD, _QUAD_C,
                        element_owner, rank_grid)


@dataclass
class FaceNeighbour:
    rank: int               # 0-based neighbour rank (nbh_proc = rank + 1)
    faces: np.ndarray       # 0-based local face ids shared with it (nbh_send_recv - 1), agreed order


@dataclass
class FaceRankCase(Case):
    rank: int = 0
    nranks: int = 1
    elems: np.ndarray = None          # global 0-based element id of each local element
    faces: np.ndarray = None          # global 0-based face id of each local face
    flipped: np.ndarray = None        # local faces whose orientation was reversed (local = global right)
    fneighbours: list = field(default_factory=list)
    halo_kind: str = "faces"

    @property
    def nelem_owned(self):
        return self.scalars["nelem"]


def morton_owner(nelx: int, nely: int, nranks: int):
    """Owner rank and Morton position of every element: the Z-order curve over (ix, iy) split
    into nranks contiguous chunks of near-equal size (p4est's partition of a uniform forest)."""
    g = np.arange(nelx * nely)
    ix, iy = g % nelx, g // nelx
    key = np.zeros(g.size, dtype=np.int64)
    for b in range(16):
        key |= ((ix >> b) & 1).astype(np.int64) << (2 * b)
        key |= ((iy >> b) & 1).astype(np.int64) << (2 * b + 1)
    order = np.argsort(key, kind="stable")        # curve position -> element
    pos = np.empty_like(order)
    pos[order] = np.arange(g.size)
    n = g.size
    bounds = [(n * r) // nranks for r in range(nranks + 1)]
    owner = np.searchsorted(np.array(bounds[1:]), pos, side="right")
    return owner, pos


def face_partition(case: Case, nranks: int, rank: int, order: str = "block") -> FaceRankCase:
    mesh, A, S = case.mesh, case.arrays, case.scalars
    if order == "block":
        px, py = rank_grid(nranks)
        owner = element_owner(mesh.nelx, mesh.nely, px, py)
        key = np.arange(owner.size)
    elif order == "morton":
        owner, key = morton_owner(mesh.nelx, mesh.nely, nranks)
    else:
        raise ValueError(order)
    face = np.asarray(A["face"])
    el = face[6].astype(np.int64) - 1
    er = face[7].astype(np.int64)
    erg = np.where(er > 0, er - 1, -1)
    mine = np.flatnonzero(owner == rank)
    elems = mine[np.argsort(key[mine], kind="stable")]
    g2l = -np.ones(owner.size, dtype=np.int64)
    g2l[elems] = np.arange(elems.size)
    l_in = owner[el] == rank
    r_in = (erg >= 0) & (owner[np.maximum(erg, 0)] == rank)
    faces = np.flatnonzero(l_in | r_in)               # global order
    proc = (erg >= 0) & (l_in != r_in)                # shared with another rank

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
        B["wjac_df"] = np.asfortranarray(np.asarray(A["wjac_df"])[nodes])

    lf = np.zeros((8, faces.size), dtype=np.int32, order="F")
    fl, fr = el[faces], erg[faces]
    lin, rin, pf = l_in[faces], r_in[faces], proc[faces]
    lf[4] = face[4, faces]
    lf[5] = face[5, faces]
    lf[6] = np.where(lin, g2l[fl] + 1, 0)
    lf[7] = np.where(er[faces] <= 0, er[faces], np.where(rin, g2l[np.maximum(fr, 0)] + 1, 0))
    flip = ~lin                                       # the local element is the global right one
    if flip.any():
        lf[6, flip] = g2l[fr[flip]] + 1
        lf[4, flip] = face[5, faces[flip]]
        for a, b in (("imapl", "imapr"), ("imapl_q", "imapr_q")):
            B[a][..., flip] = B[b][..., flip]
        for k in ("normal_vector", "normal_vector_q"):
            B[k][..., flip] = -B[k][..., flip]
        for k in ("pbprime_face", "pbprime_df_face", "zbot_face"):
            B[k][:, :, flip] = B[k][::-1][:, :, flip]
        # the wave-speed coefficients of compute_reference_edge_variables (mod_initial_mlswe.F90:
        # 379-399) with the sides exchanged: cm <-> cp, i.e. L <-> R (sums and products commute
        # exactly); the edge reciprocal is of the new side 1
        for a, b in (("coeff_pbpert_L", "coeff_pbpert_R"), ("coeff_mass_pbub_L", "coeff_mass_pbub_R")):
            B[a][:, flip], B[b][:, flip] = B[b][:, flip].copy(), B[a][:, flip].copy()
        pb1 = B["pbprime_face"][0][:, flip]
        B["one_over_pbprime_edge"][:, flip] = np.where(pb1 > 0.0, 1.0 / np.where(pb1 > 0.0, pb1, 1.0), 0.0)
    if pf.any():                                       # processor faces: face(6) = 0, face(8) = 0
        lf[5, pf] = 0
        lf[7, pf] = 0
        for k in ("imapr", "imapr_q"):
            B[k][..., pf] = 0
    B["face"] = lf

    fneighbours = []
    gl_face = faces
    for r in range(nranks):
        if r == rank:
            continue
        other = np.where(lin, owner[np.maximum(fr, 0)], owner[fl])
        sel = np.flatnonzero(pf & (other == r))
        if sel.size:
            sel = sel[np.argsort(gl_face[sel], kind="stable")]   # global face order: both sides agree
            fneighbours.append(FaceNeighbour(r, sel.astype(np.int64)))
    sc = dict(S)
    sc.update(nelem=int(elems.size), npoin=int(elems.size * P), npoin_q=int(elems.size * Q), nface=int(faces.size))
    return FaceRankCase(cfg=case.cfg, basis=case.basis, mesh=None, arrays=B, scalars=sc, rank=rank, nranks=nranks,
                        elems=elems, faces=faces, flipped=np.flatnonzero(flip), fneighbours=fneighbours)


def add_dense_tables(pc: FaceRankCase) -> FaceRankCase:
    """The reference's dense per-quad-point tables (psih, dpsidx, ... Tensor_product.F90:50-126)
    for this rank's elements only, built from its own element metrics.  Equal to slicing the
    global tables (face_partition of a dense case): every column depends on its own element
    alone, and the index tables are the same local base + node.  For meshes whose global dense
    tables do not fit (C4: ~6 GB), the reference harness reads these per rank."""
    from types import SimpleNamespace
    from .case import _dense_tables
    _dense_tables(pc.arrays, pc.basis, SimpleNamespace(nelem=int(pc.scalars["nelem"])))
    return pc


def halo_lists(pc: FaceRankCase):
    """mod_parallel's arrays for this rank: num_nbh, nbh_proc (1-based ranks), num_send_recv,
    nbh_send_recv (1-based local face ids), nbh_send_recv_multi (1: conforming)."""
    nb = pc.fneighbours
    nbh_proc = np.array([n.rank + 1 for n in nb], dtype=np.int32)
    num = np.array([n.faces.size for n in nb], dtype=np.int32)
    lst = (np.concatenate([n.faces for n in nb]) + 1).astype(np.int32) if nb else np.zeros(0, np.int32)
    return nbh_proc, num, lst, np.ones(lst.size, dtype=np.int32)


def self_neighbour(pc: FaceRankCase, per_peer: bool = True, mirror_statics: bool = True) -> FaceRankCase:
    """Rank `pc.rank` of a W-rank partition as its own neighbour, in a one-rank communicator (the
    self-neighbour contract of hnumo_engine_create; bench.py --emulate): one GPU runs the rank's
    launches, streams, events and RCCL group calls per stage with every message going to itself.

    per_peer: keep the real per-neighbour lists, each addressed to rank 0 (itself) -- the real
        run's message shape: one ncclSend/ncclRecv pair per neighbour, at its own offset and size
        (send_receive_bound.F90:860-880); False: all processor faces as ONE list.
    mirror_statics: a processor face receives its OWN side-1 traces as side 2, so its side-2
        statics become side 1's too (pbprime_face, pbprime_df_face, zbot_face, and the edge
        wave-speed coefficients of compute_reference_edge_variables, mod_initial_mlswe.F90:355-401,
        with c_- = c_+): the mirror is one consistent neighbour.  For the shipped configurations this
        changes no bit (their bathymetry is continuous, both sides already agree); what keeps an
        emulated lake at rest is the frozen halo (Engine.debug_frozen_halo).  The work
        per face is unchanged.  Modifies and returns pc."""
    pc.nranks, pc.rank = 1, 0
    nb = pc.fneighbours
    if per_peer:
        pc.fneighbours = [FaceNeighbour(0, n.faces) for n in nb]
    else:
        pc.fneighbours = [FaceNeighbour(0, np.concatenate([n.faces for n in nb]))] if nb else []
    if mirror_statics and nb:
        f = np.concatenate([n.faces for n in nb])
        B = pc.arrays
        for k in ("pbprime_face", "pbprime_df_face", "zbot_face"):
            B[k][1][:, f] = B[k][0][:, f]
        alpha = np.asarray(B["alpha"])
        c = np.sqrt(alpha[pc.scalars["nlayers"] - 1] * B["pbprime_face"][0][:, f])
        ok = c > 0.0
        den = np.where(ok, c + c, 1.0)
        z = np.zeros_like(c)
        for k in ("coeff_pbpert_L", "coeff_pbpert_R", "coeff_mass_pbub_L", "coeff_mass_pbub_R"):
            B[k][:, f] = np.where(ok, c / den, z)
        B["coeff_pbub_LR"][:, f] = np.where(ok, 1.0 / den, z)
        B["coeff_mass_pbpert_LR"][:, f] = np.where(ok, c * c / den, z)
    return pc


def gather_faces_state(parts, name, global_case):
    """Reassemble a nodal state array (ncomp, npoin[, L]) from every rank's elements."""
    A = np.asarray(global_case.arrays[name])
    out = np.zeros_like(A)
    P = global_case.scalars["ngl"] ** 2
    for pc, arr in parts:
        gn = (pc.elems[:, None] * P + np.arange(P)[None, :]).ravel()
        out[:, gn, ...] = np.asarray(arr)[:, :, ...]
    return out

"""Correctness check of a multi-GPU run's halo (bench.py at N>1).

After the timed steps every rank advances its partition ONE baroclinic step from the initial
condition over the live transport (RCCL between the GPUs) and compares its state, bit for bit,
with a result computed on its own GPU alone, without RCCL:

  processor-face halo (the reference's contract, hnumo/facepart.py): the same partitions as one
      local exchange group on this GPU (one engine per rank, device copies) -- the transport that
      tests/test_facehalo_gpu.py pins to the reference Fortran under mpiexec.  (A processor-face
      run is not bitwise equal to one rank: each rank evaluates a shared face in its own
      orientation, as the reference does)
  ghost-element halo (hnumo/partition.py): the whole mesh on this GPU as one rank -- the ghost
      layer reproduces single-rank arithmetic on the owned elements bit for bit.

The comparison itself (`compare`) is plain numpy and runs on the CPU in the tests."""
from __future__ import annotations

import numpy as np


def owned(rc, state):
    """The owned part of a rank's nodal state (q, qb, qp): ghost-element ranks keep their owned
    elements first; processor-face ranks own every local element."""
    n = getattr(rc, "nelem_owned", rc.scalars["nelem"]) * rc.scalars["ngl"] ** 2
    return tuple(np.asarray(a)[:, :n, ...] for a in state)


def global_slice(rc, gstate):
    """The owned elements' nodes of a global state (q, qb, qp), in the rank's local order."""
    P = rc.scalars["ngl"] ** 2
    n_own = getattr(rc, "nelem_owned", rc.scalars["nelem"])
    idx = (np.asarray(rc.elems[:n_own])[:, None] * P + np.arange(P)[None, :]).ravel()
    return tuple(np.asarray(a)[:, idx, ...] for a in gstate)


def compare(a, b):
    """(bitwise equal, max relative difference) of two states (q, qb, qp)."""
    same = all(np.array_equal(x, y) for x, y in zip(a, b))
    rel = 0.0
    for x, y in zip(a, b):
        s = float(np.abs(y).max()) or 1.0
        rel = max(rel, float(np.abs(x - y).max()) / s)
    return same, rel


def step_from_ic(eng):
    """One step of a (possibly resident) engine from its case's initial condition; the engine is
    left non-resident."""
    eng.set_resident(False)
    st = eng.state()
    eng.ti_rk_bcl(*st)
    return st


def reference_faces(gcase, nranks, rank, order, device):
    """This rank's state after one step of the processor-face partition run as a local exchange
    group on `device` (every rank's engine in this process)."""
    from .facepart import face_partition
    parts = [face_partition(gcase, nranks, r, order) for r in range(nranks)]
    return reference_faces_cases(parts, rank, device)


def reference_faces_cases(parts, rank, device, frozen=False):
    """reference_faces for given partition cases (ranks 0..n-1 of one partition; a single
    self-neighbour case for bench.py --emulate, frozen: with its frozen halo)."""
    from .engine import Engine, group_ti_rk_bcl, local_group
    engines = [Engine(p, device=device) for p in parts]
    try:
        if frozen:
            for e in engines:
                e.debug_frozen_halo(True)
        local_group(engines)
        states = [e.state() for e in engines]
        group_ti_rk_bcl(engines, states)
        return parts[rank], states[rank]
    finally:
        for e in engines:
            e.close()


def reference_ghost(gcase, rc, device):
    """The owned elements of rank `rc` after one single-rank step of the whole mesh."""
    from .engine import Engine
    e = Engine(gcase, device=device)
    try:
        st = e.state()
        e.ti_rk_bcl(*st)
        return global_slice(rc, st)
    finally:
        e.close()

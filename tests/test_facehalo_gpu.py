"""Multi-rank with the reference's own halo contract (row a9/e): processor-face partitions
(hnumo/facepart.py; block and Morton orders) run as local exchange groups on one GPU -- one
engine per rank, each with the two-stream schedule (boundary elements + trace transport on a
second stream, interior elements beside it) -- against the REFERENCE FORTRAN run under
mpiexec on the same partitions (tests/golden/*_mpi*.npz, tests/golden/make_golden.py mpi):
every rank's state bit for bit after 1-2 baroclinic steps.  The RCCL transport runs the same
exchange points with ncclSend/ncclRecv (one GPU per rank)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.mark.parametrize("name", ["bump10_mpi3m_step2", "lake10_mpi2b_step1", "dg8L3_mpi2b_step2",
                                  "dg8L3_mpi4m_step2", "lake10_mpi4m_step2",
                                  # method_visc == 1: quad-point LDG fluxes across processor faces
                                  "bump10q_mpi2b_step1", "dg8L3q_mpi4m_step2",
                                  # the BASELINE configs at their stated sizes: C5 (lake 200x200,
                                  # 4 Morton ranks) and C4 (316x316 on the 4x2 blocks of the 8-GPU
                                  # metric); strided samples + sha256 of every rank's whole state
                                  "lake200_mpi4m_step1", "dg316L3_mpi8b_step1"])
def test_face_halo_matches_reference_mpi(name):
    _face_halo_run(name)


@pytest.mark.parametrize("nb", ["0", "4"])
def test_face_halo_every_stage_arena_matches_reference_mpi(nb, monkeypatch):
    """The two-stream schedule's hand-offs are the per-stage launches' own stop events
    (Launch::stage; a recorded event for the arena without hipExtLaunchKernelGGL): with each
    other arena forced on a large mesh (HNUMO_STAGE_NB; the default there is the 5-per-CU LEAN
    arena), C5 at its stated size (10,000 elements per rank) still equals the reference under
    mpiexec bit for bit on every rank."""
    monkeypatch.setenv("HNUMO_EXPERIMENTS", "1")
    monkeypatch.setenv("HNUMO_STAGE_NB", nb)
    _face_halo_run("lake200_mpi4m_step1")


def _face_halo_run(name):
    from util import overrides_of, state_sha256
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine, group_ti_rk_bcl, local_group
    from hnumo.facepart import face_partition
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    case = build_case(make_config(str(g["config"]), **overrides_of(g)), dense=False)
    R = int(g["nranks"])
    parts = [face_partition(case, R, r, str(g["order"])) for r in range(R)]
    engines = [Engine(p) for p in parts]
    local_group(engines)
    states = [e.state() for e in engines]
    for _ in range(int(g["nsteps"])):
        group_ti_rk_bcl(engines, states)
    s = int(g.get("stride", 1))
    for r, st in enumerate(states):
        for k, a in zip(("q_df", "qb_df", "qprime_df"), st):
            ref = g[f"{k}_r{r}"]
            a_s = a[:, ::s, ...]
            assert np.array_equal(a_s, ref), (name, r, k, float(np.abs(a_s - ref).max() / np.abs(ref).max()))
            if f"{k}_sha256_r{r}" in g:
                assert state_sha256(a) == str(g[f"{k}_sha256_r{r}"]), (name, r, k)
    for e in engines:
        e.close()


def test_neighbour_listed_twice_is_rejected():
    """mod_parallel lists each neighbour process once (p4est.c:1343-1360) and the transports pair a
    rank's message with the peer's one entry for it: a halo that lists a neighbour rank twice is
    an invalid argument (code 4), not a transfer of mismatched sizes."""
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine, EngineError
    from hnumo.facepart import FaceNeighbour, face_partition
    case = build_case(make_config("bump10"), dense=False)
    pc = face_partition(case, 3, 1, "morton")
    assert len(pc.fneighbours) == 2
    f = pc.fneighbours
    pc.fneighbours = [FaceNeighbour(f[0].rank, f[0].faces[: len(f[0].faces) // 2]),
                      FaceNeighbour(f[0].rank, f[0].faces[len(f[0].faces) // 2:]), f[1]]
    with pytest.raises(EngineError) as ei:
        Engine(pc)
    assert ei.value.code == 4 and "listed twice" in str(ei.value)

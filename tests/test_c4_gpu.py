"""C4 (BASELINE.json configs[3]): the double gyre at ~1e5 elements (316x316, N=4, 3 layers,
dt=40 s, dt_btp=2 s), the size the 8-GPU metric is quoted on.

Parity at full size is pinned against the reference Fortran itself: the fixture
dg316L3_mpi8b_step1 (the reference under mpiexec -n 8 on the 4x2 block partition of the 8-GPU
metric; strided samples + the sha256 of every rank's whole state) runs in
test_facehalo_gpu.py.  This file adds size-independent properties at full size (finite state,
per-layer mass conserved to the reference CI's 1e-12, CI/bump/check.F90:58) and the multi-rank
identity: the 8-way ghost-halo decomposition (4x2 blocks of 79x158 elements, local exchange
group on this one GPU) reproduces the single-rank engine bit for bit."""
import numpy as np
import pytest

from util import layer_mass

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c4():
    from hnumo.case import build_case, make_config
    return build_case(make_config("dg316L3"), dense=False)


@pytest.fixture(scope="module")
def c4_single(c4):
    from hnumo.engine import Engine
    e = Engine(c4)
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    path = e.stage_path
    e.close()
    return q, qb, qp, path


def test_c4_single_rank_step(c4, c4_single):
    q, qb, qp, path = c4_single
    assert c4.scalars["nelem"] == 99856 and c4.scalars["N_btp"] == 20
    assert path == "per-stage"  # 99,856 workgroups cannot all be resident: per-stage launches
    for a in (q, qb, qp):
        assert np.isfinite(a).all()
    m0 = layer_mass(c4, c4.arrays["q_df"])
    loss = np.abs(layer_mass(c4, q) - m0) / m0
    assert (loss <= 1e-12).all(), loss
    # the wind has started the gyres: the state moved
    assert np.abs(qb[2]).max() > 0.0 and not np.array_equal(qb, c4.arrays["qb_df"])


def test_c4_eight_way_partition_bitwise(c4, c4_single):
    from hnumo.engine import Engine, group_ti_rk_bcl, local_group
    from hnumo.partition import gather_owned, partition
    q, qb, qp, _ = c4_single
    parts = [partition(c4, 8, r) for r in range(8)]
    assert [p.nelem_owned for p in parts] == [79 * 158] * 8
    engines = [Engine(p) for p in parts]
    local_group(engines)
    states = [e.state() for e in engines]
    group_ti_rk_bcl(engines, states)
    for j, name in enumerate(("q_df", "qb_df", "qprime_df")):
        got = gather_owned([(p, s[j]) for p, s in zip(parts, states)], name, c4)
        ref = (q, qb, qp)[j]
        assert np.array_equal(got, ref), (name, float(np.abs(got - ref).max()))
    for e in engines:
        e.close()

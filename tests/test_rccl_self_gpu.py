"""The RCCL transport of the processor-face halo on ONE GPU.  RCCL refuses two ranks of one
communicator on one device, so the multi-GPU path (csrc/engine.hip face_tx / trace_exchange,
comm_mode 2: ncclSend/ncclRecv inside ncclGroupStart/End, stage traces on the second stream,
the baroclinic face messages and the quad-point LDG fluxes on the engine stream) is exercised
with a one-rank communicator whose processor faces are listed under the rank itself (the
self-neighbour contract of hnumo_engine_create): every listed face receives its own side 1.
The same partition run through the local exchange group (device copies; the transport that
tests/test_facehalo_gpu.py pins to the reference Fortran under mpiexec) must give the same
bits: the RCCL send/receive order, buffers, offsets and stream ordering are then those of the
validated path.  Reference: send_receive_bound.F90:806-885, create_rhs_dynamics_flux.F90:104-182."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def self_neighbour_case(cfg, **ov):
    from hnumo.case import build_case, make_config
    from hnumo.facepart import face_partition
    pc = face_partition(build_case(make_config(cfg, **ov), dense=False), 2, 0, "block")
    pc.nranks = 1
    for n in pc.fneighbours:
        n.rank = 0
    return pc


# (nodal LDG: the two-stream schedule; method_visc 1: one stream, LDG fluxes exchanged per stage.
# Not bump10q: its viscosity is strong enough on 200-m elements that the mirror halo of the
# self-neighbour contract, with the reference's face flux that is not antisymmetric in the two
# sides' orientation (mod_laplacian_quad.F90:485-486), runs away in the first step on both
# transports alike -- DESIGN.md §8)
@pytest.mark.parametrize("cfg,ov,graph", [("bump10", {}, "0"), ("dg8L3q", dict(method_visc=3), "0"),
                                          ("dg8L3q", dict(method_visc=3), "1"), ("dg8L3q", {}, "0"),
                                          ("dg8L3q", {}, "1")])
def test_rccl_self_exchange_matches_local_group(cfg, ov, graph, monkeypatch):
    from hnumo.engine import Engine, group_ti_rk_bcl, local_group
    pc = self_neighbour_case(cfg, **ov)
    assert sum(n.faces.size for n in pc.fneighbours) > 0
    e_loc = Engine(pc)
    local_group([e_loc])
    monkeypatch.setenv("HNUMO_GRAPH", graph)   # RCCL engines: direct launches (0) or captured step (1)
    e_rccl = Engine(pc, comm_id=Engine.rccl_unique_id())
    monkeypatch.delenv("HNUMO_GRAPH")
    a, b = e_loc.state(), e_rccl.state()
    for _ in range(2):
        group_ti_rk_bcl([e_loc], [a])
        e_rccl.ti_rk_bcl(*b)
    assert all(np.isfinite(x).all() for x in a)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    e_rccl.close()
    e_loc.close()


def test_rccl_self_per_peer_lists_match_local_group_and_one_list():
    """The real multi-peer message shape on one GPU (missing 1): rank 1 of the 4x2
    block partition (C4/8's shape: neighbours 0, 2 and 5, each with its own list) keeps its three
    lists, every one addressed to itself -- three ncclSend/ncclRecv pairs to self inside one group,
    at the real offsets and sizes (send_receive_bound.F90:860-880, create_rhs_communicator.F90:
    193-262).  Over RCCL (direct launches and the captured step) it must equal the same partition
    run through the local exchange group, and the one-list mirror, bit for bit."""
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine, group_ti_rk_bcl, local_group
    from hnumo.facepart import face_partition, self_neighbour
    g = build_case(make_config("dg8L3q"), dense=False)
    pc = self_neighbour(face_partition(g, 8, 1, "block"))
    assert [n.rank for n in pc.fneighbours] == [0, 0, 0] and min(n.faces.size for n in pc.fneighbours) > 0
    one = self_neighbour(face_partition(g, 8, 1, "block"), per_peer=False)
    e_loc, e_one = Engine(pc), Engine(one)
    local_group([e_loc])
    local_group([e_one])
    eng = {}
    for graph in ("0", "1"):
        os.environ["HNUMO_GRAPH"] = graph
        try:
            eng[graph] = Engine(pc, comm_id=Engine.rccl_unique_id())
        finally:
            del os.environ["HNUMO_GRAPH"]
    sts = {k: e.state() for k, e in eng.items()}
    a, c = e_loc.state(), e_one.state()
    for _ in range(2):
        group_ti_rk_bcl([e_loc], [a])
        group_ti_rk_bcl([e_one], [c])
        for k, e in eng.items():
            e.ti_rk_bcl(*sts[k])
    assert all(np.isfinite(x).all() for x in a)
    for b in list(sts.values()) + [c]:
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    for e in list(eng.values()) + [e_loc, e_one]:
        e.close()


def test_frozen_halo_keeps_the_lake_at_rest_on_both_transports():
    """bench.py --emulate of C5 (the lake at rest on a Morton partition, its rank 1 with three
    neighbours): with the frozen halo (hnumo_debug_frozen_halo) each processor face keeps receiving
    the initial message -- the real at-rest neighbour's traces -- so the rank stays at rest like the
    real 4-rank run (the mirror, its own traces, runs away: DESIGN.md §8.1), and RCCL equals the
    local exchange group bit for bit.  The frozen halo is refused on a real multi-rank engine."""
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine, EngineError, group_ti_rk_bcl, local_group
    from hnumo.facepart import face_partition, self_neighbour
    g = build_case(make_config("lake10"), dense=False)
    parts = [face_partition(g, 4, r, "morton") for r in range(4)]
    real = [Engine(p) for p in parts]
    local_group(real)
    with pytest.raises(EngineError):
        real[1].debug_frozen_halo(True)
    rs = [e.state() for e in real]
    pc = self_neighbour(face_partition(g, 4, 1, "morton"))
    assert len(pc.fneighbours) == 3
    e_loc = Engine(pc)
    e_loc.debug_frozen_halo(True)
    local_group([e_loc])
    e_rccl = Engine(pc, comm_id=Engine.rccl_unique_id())
    e_rccl.debug_frozen_halo(True)
    a, b = e_loc.state(), e_rccl.state()
    for _ in range(3):
        group_ti_rk_bcl(real, rs)
        group_ti_rk_bcl([e_loc], [a])
        e_rccl.ti_rk_bcl(*b)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    u_real = np.abs(rs[1][1][2:4]).max()
    u_emu = np.abs(a[1][2:4]).max()
    assert np.isfinite(a[1]).all() and u_emu < 1e-5, (u_emu, u_real)
    for e in real + [e_loc, e_rccl]:
        e.close()

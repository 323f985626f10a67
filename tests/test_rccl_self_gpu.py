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

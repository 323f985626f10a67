"""The persistent sub-cycle launch (btp_subcycle_kernel, one launch per barotropic sub-cycle of
mod_rk_mlswe.F90:82-116) needs every element's workgroup resident at once.  These tests give
the launch more LDS per workgroup than fits (HNUMO_PERSIST_LDS_PAD, dynamic LDS the kernel does
not use) and check each of the three guards (csrc/engine.hip, kernels_btp.hip
residency_rendezvous):
  * the occupancy estimate at create rejects the launch;
  * the stage-less trial launch at create rejects it when the estimate is bypassed;
  * with both bypassed, the launch itself finds its workgroups not co-resident, does no work
    and ends; the engine drops the persistent path and repeats the step on per-stage launches.
Every case must then reproduce the reference Fortran's step bit for bit (golden fixtures)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PAD = 30000  # bytes: ~84 KB of LDS per workgroup, one per CU -- 256 slots for 625 elements


def golden_case(name, case_factory):
    from util import overrides_of
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    return g, case_factory(str(g["config"]), **overrides_of(g))


def assert_golden(g, q, qb, qp):
    s = int(g["stride"])
    assert np.array_equal(q[:, ::s, :], g["q_df"]) and np.array_equal(qb[:, ::s], g["qb_df"])
    assert np.array_equal(qp[:, ::s, :], g["qprime_df"])


def make_engine(case, monkeypatch, guard):
    from hnumo.engine import Engine
    monkeypatch.setenv("HNUMO_EXPERIMENTS", "1")
    monkeypatch.setenv("HNUMO_PERSIST_LDS_PAD", str(PAD))
    monkeypatch.setenv("HNUMO_PERSIST_GUARD", guard)
    try:
        return Engine(case)
    finally:
        monkeypatch.delenv("HNUMO_PERSIST_LDS_PAD")
        monkeypatch.delenv("HNUMO_PERSIST_GUARD")
        monkeypatch.delenv("HNUMO_EXPERIMENTS")


def test_default_engine_is_persistent_and_resident(case_factory):
    """dg25L3 (625 elements, 3 workgroups per CU): all three checks pass."""
    from hnumo.engine import Engine
    g, case = golden_case("dg25L3_step1", case_factory)
    e = Engine(case)
    info = e.persistent_info
    assert e.stage_path == "persistent", info
    assert info["trial_launch"][0] == 1 and info["occupancy_blocks_per_cu"][0] * info["cus"] >= 625, info
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    assert_golden(g, q, qb, qp)
    assert e.persistent_info["fallbacks"] == 0
    e.close()


def test_estimate_rejects_oversized_arena(case_factory, monkeypatch):
    g, case = golden_case("dg25L3_step1", case_factory)
    e = make_engine(case, monkeypatch, "estimate")
    info = e.persistent_info
    assert e.stage_path == "per-stage", info
    assert info["occupancy_blocks_per_cu"][0] * info["cus"] < 625, info
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    assert_golden(g, q, qb, qp)
    e.close()


def test_trial_launch_rejects_oversized_arena(case_factory, monkeypatch):
    g, case = golden_case("dg25L3_step1", case_factory)
    e = make_engine(case, monkeypatch, "trial")
    info = e.persistent_info
    assert e.stage_path == "per-stage", info
    assert info["trial_launch"][0] == 0, info
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    assert_golden(g, q, qb, qp)
    e.close()


def test_launch_falls_back_when_not_coresident(case_factory, monkeypatch):
    """No estimate, no trial: the first step's persistent launch is not co-resident.  It must
    end (rendezvous abort, not a hang), leave the state untouched, and the engine must redo
    the step on per-stage launches -- the reference's bits."""
    g, case = golden_case("dg25L3_step1", case_factory)
    e = make_engine(case, monkeypatch, "0")
    assert e.stage_path == "persistent"
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    assert_golden(g, q, qb, qp)
    info = e.persistent_info
    assert e.stage_path == "per-stage" and info["fallbacks"] == 1, info
    e.close()


def test_resident_run_falls_back(case_factory, monkeypatch):
    """Resident mode (state kept on the device), 3 steps in one run: the aborted first step
    leaves the device state as it was and the retried steps continue from it -- the same bits
    as an engine on per-stage launches from the start (HNUMO_PERSISTENT=0)."""
    from hnumo.engine import Engine
    _, case = golden_case("dg25L3_step1", case_factory)
    e = make_engine(case, monkeypatch, "0")
    monkeypatch.setenv("HNUMO_PERSISTENT", "0")
    e0 = Engine(case)
    monkeypatch.delenv("HNUMO_PERSISTENT")
    a, b = e.state(), e0.state()
    e.set_resident(True)
    for _ in range(3):
        e.ti_rk_bcl(*a)
        e0.ti_rk_bcl(*b)
    e.sync(*a)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert e.persistent_info["fallbacks"] == 1
    e.close()
    e0.close()


def test_corrector_abort_is_redone_and_path_recovers(case_factory, monkeypatch):
    """The corrector's persistent launch gives up after the predictor's sub-cycle and its
    baroclinic kernels ran (hnumo_debug_force_abort: launch 0 of the step is the predictor's
    sub-cycle, launch 1 the corrector's).  The step is redone on per-stage launches with the
    reference's bits; the next step runs on per-stage launches too (the back-off of one run after
    a first abort, include/hnumo_engine.h), the one after re-probes residency with a trial launch,
    finds the grid resident and runs persistent again -- the same bits as an engine on per-stage
    launches from the start."""
    from hnumo.engine import Engine
    g, case = golden_case("dg25L3_step1", case_factory)
    e = Engine(case)
    assert e.stage_path == "persistent"
    e.debug_force_abort(1)
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    assert_golden(g, q, qb, qp)
    st = e.persistent_stats
    assert st["aborts"] == 1 and st["reprobes"] == 0 and e.stage_path == "per-stage", st
    monkeypatch.setenv("HNUMO_PERSISTENT", "0")
    e0 = Engine(case)
    monkeypatch.delenv("HNUMO_PERSISTENT")
    a = [x.copy(order="F") for x in (q, qb, qp)]
    for k in range(3):
        e.ti_rk_bcl(q, qb, qp)
        e0.ti_rk_bcl(*a)
        assert e.stage_path == ("per-stage" if k == 0 else "persistent"), (k, e.persistent_stats)
    for x, y in zip((q, qb, qp), a):
        assert np.array_equal(x, y)
    st = e.persistent_stats
    assert st == {"aborts": 1, "reprobes": 1, "recovered": 1, "wait": -1}, st
    e.close()
    e0.close()


def test_predict_on_resident_engine_reuploads(case_factory):
    """hnumo_predict replaces the device state with the caller's input (ABI v7): a resident
    engine's next step then starts from the caller's arrays, not from its old device state."""
    from hnumo.engine import Engine
    _, case = golden_case("dg25L3_step1", case_factory)
    e = Engine(case)
    e.set_resident(True)
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)                        # device state: step 1
    p = [x.copy(order="F") for x in e.state()]
    e.predict(*p)                                 # device state: the IC's predictor input
    r = e.state()
    e.ti_rk_bcl(*r)                               # must start from r (the IC), not from step 1
    e.sync(*r)
    e1 = Engine(case)
    s = e1.state()
    e1.ti_rk_bcl(*s)
    for x, y in zip(r, s):
        assert np.array_equal(x, y)
    e.close()
    e1.close()


def test_step_breakdown_abort_advances_exactly_nsteps(case_factory, monkeypatch):
    """hnumo_step_breakdown whose second step's corrector launch gives up (launch 3 from now):
    the first step stands, only the second is redone on per-stage launches, so the state advances
    by exactly the 2 steps asked -- the same bits as 3 steps of an engine on per-stage launches
    (1 ti_rk_bcl + the breakdown's 2), and the retry does not spend the back-off wait."""
    from hnumo.engine import Engine
    _, case = golden_case("dg25L3_step1", case_factory)
    e = Engine(case)
    assert e.stage_path == "persistent"
    e.set_resident(True)
    a = e.state()
    e.ti_rk_bcl(*a)
    e.debug_force_abort(3)
    bd = e.step_breakdown(2)
    assert bd and all(v >= 0 for v in bd.values()), bd
    st = e.persistent_stats
    assert st["aborts"] == 1 and st["reprobes"] == 0 and st["wait"] == 1, st
    e.sync(*a)
    monkeypatch.setenv("HNUMO_PERSISTENT", "0")
    e0 = Engine(case)
    monkeypatch.delenv("HNUMO_PERSISTENT")
    b = e0.state()
    for _ in range(3):
        e0.ti_rk_bcl(*b)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    e.close()
    e0.close()

"""GPU parity tests: the HIP engine (through the C ABI) against the CPU oracle on the same
inputs, and against the reference's golden vectors.

Bar: normwise relative difference <= 1e-10 (BASELINE.json north_star), for both summation
modes of the barotropic stage (hnumo_set_summation):
  reference -- the default: the reference's summation order (kernels_btp.hip header); on the
               shipped configurations the engine is bit-identical to the oracle -- and the
               oracle to the reference Fortran (tests/test_oracle.py) -- which test_bitwise_*
               assert;
  factored  -- opt-in sum factorisation: thicknesses within 1e-10, momenta within rounding of
               the cancelling pressure terms (test_factored_summation_parity)."""
import os

import numpy as np
import pytest

from util import layer_mass, rel, state_sha256

pytestmark = pytest.mark.gpu
TOL = 1e-10
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def engines():
    made = {}
    yield made
    for e in made.values():
        e.close()


def get_engine(engines, case, summation="reference"):
    from hnumo.engine import Engine
    key = (id(case), summation)
    if key not in engines:
        engines[key] = Engine(case, summation=summation)
    return engines[key]


@pytest.mark.parametrize("cfg", ["bump10", "dg25", "dg25L3", "bump10q", "dg8L3q"])
def test_rhs_stage_parity(cfg, case_factory, engines):
    import oracle as O
    case = case_factory(cfg)
    o = O.Oracle(case)
    e = get_engine(engines, case)
    q, qb, qp = o.state()
    # give the state some velocity so every term of the stage is active
    o.btp_bcl_coeffs(qp)
    o.ti_barotropic_ssprk(qb, qp)
    o.btp_bcl_coeffs(qp)
    r_o = o.create_rhs_btp(qb, qp)
    e.btp_bcl_coeffs(qp)
    r_e = e.create_rhs_btp(qb, qp)
    for v in range(3):
        assert rel(r_e[v], r_o[v]) < 1e-12, (v, rel(r_e[v], r_o[v]))
    for f in ["Q_uu_dp", "H_bcl", "Q_uv_dp_edge", "H_bcl_edge", "btp_dpp_graduv", "pbprime_visc",
              "btp_graduv_dpp_face", "H_ave", "Qu_ave", "ope_face_ave", "graduvb_ave", "graduvb_face_ave",
              "btp_mass_flux_face_ave", "uvb_face_ave"]:
        assert rel(e.field(f), o.field(f)) < 1e-12, f


@pytest.mark.parametrize("cfg", ["bump10", "dg25L3"])
def test_barotropic_subcycle_parity(cfg, case_factory, engines):
    import oracle as O
    from hnumo import bundle as B
    case = case_factory(cfg)
    o = O.Oracle(case)
    e = get_engine(engines, case)
    q, qb, qp = o.state()
    qb_e = qb.copy(order="F")
    o.btp_bcl_coeffs(qp)
    o.ti_barotropic_ssprk(qb, qp)
    e.btp_bcl_coeffs(qp)
    e.ti_barotropic_ssprk(qb_e, qp)
    for v in range(4):
        assert rel(qb_e[v], qb[v]) < 1e-11, (v, rel(qb_e[v], qb[v]))
    for f, _ in B.FIELDS:
        if f.startswith("sum_layer"):
            continue
        assert rel(e.field(f), o.field(f)) < 1e-10, (f, rel(e.field(f), o.field(f)))


@pytest.mark.parametrize("cfg,nsteps", [("bump10", 2), ("lake10", 1), ("dg25", 2), ("dg25L3", 2)])
def test_baroclinic_step_parity(cfg, nsteps, case_factory, engines):
    import oracle as O
    case = case_factory(cfg)
    o = O.Oracle(case)
    e = get_engine(engines, case)
    q, qb, qp = o.state()
    qe, qbe, qpe = e.state()
    for _ in range(nsteps):
        o.ti_rk_bcl(q, qb, qp)
        e.ti_rk_bcl(qe, qbe, qpe)
    L = case.scalars["nlayers"]
    for k in range(L):
        for v in range(3):
            assert rel(qe[v, :, k], q[v, :, k]) < TOL, ("q", v, k, rel(qe[v, :, k], q[v, :, k]))
            assert rel(qpe[v, :, k], qp[v, :, k]) < TOL, ("qprime", v, k, rel(qpe[v, :, k], qp[v, :, k]))
    for v in range(4):
        assert rel(qbe[v], qb[v]) < TOL, ("qb", v, rel(qbe[v], qb[v]))


@pytest.mark.parametrize("cfg", ["bump10", "dg25L3", "bump10q", "dg8L3q"])
def test_bitwise_step(cfg, case_factory, engines):
    """The engine reproduces the reference arithmetic bit for bit (2 baroclinic steps)."""
    import oracle as O
    case = case_factory(cfg)
    o = O.Oracle(case)
    e = get_engine(engines, case, "reference")
    q, qb, qp = o.state()
    qe, qbe, qpe = e.state()
    for _ in range(2):
        o.ti_rk_bcl(q, qb, qp)
        e.ti_rk_bcl(qe, qbe, qpe)
    assert np.array_equal(qe, q) and np.array_equal(qbe, qb) and np.array_equal(qpe, qp)
    from hnumo import bundle as B
    for f, _ in B.FIELDS:
        assert np.array_equal(e.field(f), o.field(f)), f


@pytest.mark.parametrize("cfg", ["bump10s", "dg8L3s"])
def test_shear_stress_bitwise(cfg, case_factory):
    """ad_mlswe > 0 (implicit vertical shear stress, mod_create_rhs_mlswe.F90:146-279, fused into
    mom_elem_kernel) with the corrector reading the predicted momenta
    (HNUMO_SHEAR_CORRECTOR_PREDICTED): engine == oracle bit for bit over 2 steps."""
    import oracle as O
    from hnumo.engine import Engine
    case = case_factory(cfg, shear_corrector=1)
    o = O.Oracle(case)
    e = Engine(case)
    q, qb, qp = o.state()
    qe, qbe, qpe = e.state()
    for _ in range(2):
        o.ti_rk_bcl(q, qb, qp)
        e.ti_rk_bcl(qe, qbe, qpe)
    assert np.isfinite(q).all()
    assert np.array_equal(qe, q) and np.array_equal(qbe, qb) and np.array_equal(qpe, qp)
    e.close()


def test_shear_stress_reference_corrector_is_nonfinite(case_factory):
    """ad_mlswe > 0 with the default HNUMO_SHEAR_CORRECTOR_REFERENCE: momentum() hands
    rhs_layer_shear_stress its never-assigned `uv` (mod_splitting.F90:119,158), zeros under
    the reference build's -finit-real=zero, so the solve divides 0/0 and the corrector's layer
    momenta are NaN in the oracle; the engine reports it as HNUMO_ERR_NONFINITE."""
    import oracle as O
    from hnumo.engine import Engine, EngineError
    case = case_factory("bump10s")
    o = O.Oracle(case)
    q, qb, qp = o.state()
    o.ti_rk_bcl(q, qb, qp)
    assert np.isnan(q[1:]).any() and np.isfinite(qb).all()
    e = Engine(case)
    with pytest.raises(EngineError) as ei:
        e.ti_rk_bcl(*e.state())
    assert ei.value.code == 2
    e.close()


GOLDEN_STEPS = ["bump10_step2", "lake10_step1", "dg25_step1", "dg25L3_step1", "bump10q_step1", "dg8L3q_step1",
                "dg8N7L3_step1", "bump10_b2ns_step1", "bump10_mixed_step1", "lake10L3_step1", "bump10q_ns_step1",
                "dg8L3q_mixed_step1", "qmbump8_step2", "qmdg8L3_step1", "bump16_step1",
                # C3 at its stated size (25x25, N=7): strided sample + sha256 of the whole state
                "dg25N7L3_step1"]


@pytest.mark.parametrize("name", GOLDEN_STEPS)
def test_engine_matches_reference_golden(name, case_factory, engines):
    """The engine against the reference Fortran's own outputs (tests/golden, made by
    tests/golden/make_golden.py), incl. N=7 and the branches the shipped namelists do not run:
    quadratic drag (botfr=2), no-slip (2) and mixed walls, the 3-layer lake."""
    from util import overrides_of
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    case = case_factory(str(g["config"]), **overrides_of(g))
    e = get_engine(engines, case)
    q, qb, qp = e.state()
    for _ in range(int(g["nsteps"])):
        e.ti_rk_bcl(q, qb, qp)
    s = int(g["stride"])
    for k, a in [("q_df", q[:, ::s, :]), ("qprime_df", qp[:, ::s, :]), ("qb_df", qb[:, ::s])]:
        for v in range(a.shape[0]):
            assert rel(a[v], g[k][v]) < TOL, (k, v, rel(a[v], g[k][v]))
    # the engine reproduces the reference arithmetic: the state is bit-identical
    assert np.array_equal(q[:, ::s, :], g["q_df"]) and np.array_equal(qb[:, ::s], g["qb_df"])
    assert np.array_equal(qp[:, ::s, :], g["qprime_df"])
    for k, a in (("q_df", q), ("qb_df", qb), ("qprime_df", qp)):
        if k + "_sha256" in g:        # strided fixtures: the whole state, bit for bit
            assert state_sha256(a) == str(g[k + "_sha256"]), k


@pytest.mark.parametrize("name", ["bump10s_predict", "dg8L3s_predict"])
def test_predictor_matches_reference_golden(name, case_factory):
    """ad_mlswe > 0 (implicit vertical shear stress, mod_create_rhs_mlswe.F90:146-279): the
    prediction half of ti_rk_bcl through hnumo_predict against the reference Fortran's own
    predictor (ref_driver mode 4, its never-assigned tau_u(nlayers+1) zero as under the
    reference's -finit-real=zero build; oracle/zero_init_wrap.c) -- bit for bit."""
    from util import overrides_of
    from hnumo.engine import Engine
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    case = case_factory(str(g["config"]), **overrides_of(g))
    e = Engine(case)
    q, qb, qp = e.state()
    e.predict(q, qb, qp)
    assert np.array_equal(qb, g["qb_df"]) and np.array_equal(q, g["q_df"]) and np.array_equal(qp, g["qprime_df"])
    e.close()


BRANCH_VARIANTS = {
    "botfr2_noslip": ("bump10", dict(botfr=2, cd=1e-3, visc=25.0, method_visc=3, y_boundary=(2, 2))),
    "beta_mixed": ("bump10", dict(botfr=1, cd=1e-7, f0=1e-4, beta=1e-11, x_boundary=(2, 4))),
    "lake_L3": ("lake10", dict(nlayers=3)),
    "quadldg_noslip_botfr2": ("bump10q", dict(y_boundary=(2, 2), botfr=2, cd=1e-3)),
    "dg_L3_mixed": ("dg8L3q", dict(x_boundary=(2, 4))),
    "dg_L3_noslip_botfr2": ("dg8L3q", dict(method_visc=3, botfr=2, cd=1e-3, x_boundary=(2, 2), y_boundary=(2, 2))),
}


@pytest.mark.parametrize("variant", sorted(BRANCH_VARIANTS))
def test_branch_variants_bitwise(variant, case_factory):
    """Shipped-code branches no shipped namelist runs (mod_rhs_btp.F90:163-168 quadratic drag;
    mod_barotropic_terms.F90:89-90 / mod_laplacian_quad.F90 no-slip walls; mixed walls; a
    3-layer lake): engine == oracle bit for bit over 2 baroclinic steps, every time average
    included (the oracle is pinned to the reference on these, tests/test_oracle.py)."""
    import oracle as O
    from hnumo import bundle as B
    from hnumo.engine import Engine
    name, ov = BRANCH_VARIANTS[variant]
    case = case_factory(name, **ov)
    o = O.Oracle(case)
    e = Engine(case)
    q, qb, qp = o.state()
    qe, qbe, qpe = e.state()
    for _ in range(2):
        o.ti_rk_bcl(q, qb, qp)
        e.ti_rk_bcl(qe, qbe, qpe)
    assert np.isfinite(q).all() and np.isfinite(qb).all()
    assert np.array_equal(qe, q) and np.array_equal(qbe, qb) and np.array_equal(qpe, qp)
    for f, _ in B.FIELDS:
        assert np.array_equal(e.field(f), o.field(f)), f
    e.close()


def test_n7_step_parity(case_factory):
    """C3 configuration (N=7, 3 layers, LDS-tiled 8x8 nodes / 15x15 quad points)."""
    import oracle as O
    from hnumo.engine import Engine
    case = case_factory("dg25N7L3", nelx=8, nely=8)
    o = O.Oracle(case)
    e = Engine(case)
    q, qb, qp = o.state()
    qe, qbe, qpe = e.state()
    o.ti_rk_bcl(q, qb, qp)
    e.ti_rk_bcl(qe, qbe, qpe)
    for v in range(4):
        assert rel(qbe[v], qb[v]) < TOL, (v, rel(qbe[v], qb[v]))
    assert rel(qe, q) < TOL and rel(qpe, qp) < TOL, (rel(qe, q), rel(qpe, qp))
    e.close()


def test_mass_conservation_and_resident_mode(case_factory):
    from hnumo.engine import Engine
    case = case_factory("bump10")
    e = Engine(case)
    q, qb, qp = e.state()
    m0 = layer_mass(case, q)
    e.set_resident(True)
    for _ in range(5):
        e.ti_rk_bcl(q, qb, qp)
    e.sync(q, qb, qp)
    loss = np.abs(layer_mass(case, q) - m0) / m0
    assert (loss <= 1e-12).all(), loss
    e.close()


def test_negative_thickness_is_reported(case_factory):
    from hnumo.engine import Engine, EngineError
    case = case_factory("bump10", dt=5.0e4, dt_btp=1.0e4)
    e = Engine(case)
    q, qb, qp = e.state()
    with pytest.raises(EngineError) as ei:
        for _ in range(3):
            e.ti_rk_bcl(q, qb, qp)
    assert ei.value.code in (1, 2)
    e.close()


def test_default_summation_is_reference(case_factory):
    from hnumo.engine import Engine
    e = Engine(case_factory("bump10"))
    assert e.summation == "reference"
    e.set_summation("factored")
    assert e.summation == "factored"
    e.close()


@pytest.mark.parametrize("cfg", ["bump10", "lake10", "dg25L3"])
def test_factored_summation_parity(cfg, case_factory, engines):
    """Opt-in sum-factorised stage (HNUMO_SUM_FACTORED) after 2 baroclinic steps.  Layer
    thicknesses and pb' meet the 1e-10 bar.  The momentum RHS is a difference of pressure
    terms ~1e7 times larger, so reordering its sums moves the momenta by rounding of those
    terms: bounded against the momentum scale dp*sqrt(g*dp) of a gravity wave (1e-6), not
    against the momenta themselves (~0 in the lake at rest)."""
    import oracle as O
    case = case_factory(cfg)
    o = O.Oracle(case)
    e = get_engine(engines, case, "factored")
    q, qb, qp = o.state()
    qe, qbe, qpe = e.state()
    for _ in range(2):
        o.ti_rk_bcl(q, qb, qp)
        e.ti_rk_bcl(qe, qbe, qpe)
    g = case.scalars["gravity"]
    for k in range(case.scalars["nlayers"]):
        assert rel(qe[0, :, k], q[0, :, k]) < TOL and rel(qpe[0, :, k], qp[0, :, k]) < TOL, k
        dp = np.abs(q[0, :, k]).max()
        scale = dp * np.sqrt(g * dp)
        for v in (1, 2):
            assert np.abs(qe[v, :, k] - q[v, :, k]).max() / scale < 1e-6, (k, v)
    pb = np.abs(qb[0]).max()
    assert rel(qbe[0], qb[0]) < TOL and np.abs(qbe[1] - qb[1]).max() / pb < TOL
    for v in (2, 3):
        assert np.abs(qbe[v] - qb[v]).max() / (pb * np.sqrt(g * pb)) < 1e-6, v


@pytest.mark.parametrize("cfg", ["bump10", "dg25L3", "dg25N7L3"])
def test_persistent_subcycle_matches_stage_launches(cfg, case_factory, monkeypatch):
    """The persistent sub-cycle kernel (one launch per sub-cycle, neighbour hand-offs in the
    launch) gives the same bits as one launch per stage (HNUMO_PERSISTENT=0).  dg25N7L3 (C3,
    625 elements at N=7): the slim LDS arena fits 3 workgroups per CU, so all are resident."""
    from hnumo.engine import Engine
    case = case_factory(cfg)
    e1 = Engine(case)
    assert e1.stage_path == "persistent", e1.stage_path
    monkeypatch.setenv("HNUMO_PERSISTENT", "0")
    e0 = Engine(case)
    monkeypatch.delenv("HNUMO_PERSISTENT")
    a, b = e1.state(), e0.state()
    for _ in range(2):
        e1.ti_rk_bcl(*a)
        e0.ti_rk_bcl(*b)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    from hnumo import bundle as B
    for f, _ in B.FIELDS:
        assert np.array_equal(e1.field(f), e0.field(f)), f
    e1.close()
    e0.close()


@pytest.mark.parametrize("nb", ["0", "4", "5"])
def test_stage_arenas_match_reference_golden(nb, case_factory, monkeypatch):
    """The per-stage kernel in each of its LDS arenas (StageCfg NBK: 0 = the 3-per-CU arena of
    small meshes, 4 and 5 = the LEAN arenas of large meshes, e.g. C4) on dg25L3 -- one launch per
    stage, HNUMO_STAGE_NB forcing the arena -- equals the reference Fortran's step bit for bit."""
    from util import overrides_of
    from hnumo.engine import Engine
    g = dict(np.load(os.path.join(GOLD, "dg25L3_step1.npz"), allow_pickle=False))
    case = case_factory(str(g["config"]), **overrides_of(g))
    monkeypatch.setenv("HNUMO_PERSISTENT", "0")
    monkeypatch.setenv("HNUMO_STAGE_NB", nb)
    monkeypatch.setenv("HNUMO_EXPERIMENTS", "1")
    e = Engine(case)
    monkeypatch.delenv("HNUMO_PERSISTENT")
    monkeypatch.delenv("HNUMO_STAGE_NB")
    monkeypatch.delenv("HNUMO_EXPERIMENTS")
    assert e.overrides == ["HNUMO_STAGE_NB=" + nb, "HNUMO_PERSISTENT=0"]
    assert e.stage_path == "per-stage"
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    s = int(g["stride"])
    assert np.array_equal(q[:, ::s, :], g["q_df"]) and np.array_equal(qb[:, ::s], g["qb_df"])
    assert np.array_equal(qp[:, ::s, :], g["qprime_df"])
    e.close()

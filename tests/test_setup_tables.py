"""Row a18: the set-up tables hnumo/case.py builds for the engine and the oracle are the
reference's own, bit for bit.  tests/golden/setup_*.npz hold the outputs of the REFERENCE's
set-up routines (oracle/_ref/ref_driver mode 6, tests/golden/make_golden.py setup), run in
mod_initial_create's order (mod_initial.F90:159-183) on the same mesh:

  initial_conditions               initial_conditions.F90:1-416 (bump, lakeAtrest, double-gyre:
                                   q_df, qb_df, qprime_df; pbprime at nodes / quad points /
                                   faces, the reciprocals, alpha, zbot_df, tau_wind_df)
  compute_reference_edge_variables mod_initial_mlswe.F90:355-401 (coeff_*)
  bot_topo_derivatives             :29-120 (zbot_face)
  compute_gradient_quad            mod_Tensorproduct.F90:57-110 (grad_zbot_quad)
  wind_stress_coriolis             mod_initial_mlswe.F90:280-352 (tau_wind, coriolis_quad,
                                   fdt2_bcl, a_bcl, b_bcl; gravity = 9.806)
  ssprk_coefficients               :582-681 (ssprk_a, ssprk_beta); N_btp, dt_btp
                                   (mod_initial.F90:176-177)

The harness zero-fills what the reference build's -finit-real=zero zero-fills (the unzeroed
one_plus_eta_temp and zbot accumulations)."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
SETUP = ["setup_bump10", "setup_lake10L3", "setup_dg25", "setup_dg8N7", "setup_qmbump8"]


def _mine(case, k, shape):
    if k in ("N_btp", "dt_btp", "gravity"):
        return np.array([case.scalars[k]], dtype=np.float64)
    return np.asarray(case.arrays[k], dtype=np.float64).reshape(shape, order="F")


@pytest.mark.parametrize("name", SETUP)
def test_setup_tables_match_reference_routines(name, case_factory):
    from hnumo import bundle as B
    from util import overrides_of
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    case = case_factory(str(g["config"]), **overrides_of(g))
    d = B.dims(case)
    s = int(g["stride"])
    for k, shp in B.SETUP_OUT:
        mine = _mine(case, k, B.shape_of(shp, d)).reshape(-1, order="F")[::s]
        assert np.array_equal(mine, g["ref_" + k]), k


@pytest.mark.ref
@pytest.mark.parametrize("name,kw", [("bump10", {}), ("lake10", dict(nlayers=3)), ("dg25", dict(nelx=8, nely=8)),
                                     ("bump10", dict(x_boundary=(2, 4), f0=1e-4, beta=1e-11))])
def test_setup_tables_vs_reference_fortran(name, kw, case_factory):
    """Full arrays (no stride), straight from the reference harness."""
    import oracle as O
    from hnumo import bundle as B
    case = case_factory(name, **kw)
    ref = O.run_reference(case, "setup", 1)
    d = B.dims(case)
    for k, shp in B.SETUP_OUT:
        assert np.array_equal(_mine(case, k, B.shape_of(shp, d)), ref[k]), k

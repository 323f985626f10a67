"""The drop-in, end to end: the reference's own Fortran harness (oracle/_ref/ref_driver)
against the same harness with ti_rk_bcl replaced by the HIP engine through the Fortran
ISO_C_BINDING bridge (oracle/_ref/dropin_driver; include/hnumo_engine.f90 +
h-numo_amd/fortran/hnumo_bridge.F90).  Both binaries are built in the build container from
/root/reference sources (oracle/build_ref.sh) and travel to the GPU box with the repo.

Parity bar: bit-identical state and time averages (same as test_engine_gpu.test_bitwise_step;
default summation order).
"""
import os

import numpy as np
import pytest

from hnumo import bundle as B

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref", "ref_driver")
DROPIN = os.path.join(REPO, "oracle", "_ref", "dropin_driver")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (os.path.exists(REF) and os.path.exists(DROPIN)),
                                 reason="oracle/_ref drivers not built (build container builds them)")]


@pytest.mark.parametrize("name,nsteps", [("bump10", 2), ("dg25L3", 1)])
def test_dropin_matches_reference_bitwise(case_factory, name, nsteps):
    import oracle as O
    case = case_factory(name)
    ref = O.run_reference(case, "step", nsteps)
    got = O.run_reference(case, "step", nsteps, dropin=True)
    for k in ("q_df", "qb_df", "qprime_df"):
        assert np.array_equal(got[k], ref[k]), k
    for k, _ in B.FIELDS:
        assert np.array_equal(got[k], ref[k]), k

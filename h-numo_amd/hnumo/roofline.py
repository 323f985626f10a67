"""Algorithmic-byte model of the hot path.

Counting rule: each distinct array element the stage's math must read or write counts
once at 8 bytes; accumulators count read + write; intermediates that never leave the
stage are free; the 1-D basis is free; the reference's dense psih/dpsidx tables are an
implementation choice and are NOT counted.  Face terms are weighted by F/E.

Per element and barotropic stage (P = n^2 nodes, Q = m^2 quad points, n = N+1, m = 2N+1):
  volume  44*P + 39*Q doubles
     nodal: qb in 4P, qb0/qb2 6P, qprime(layer L) 3P, statics 13P (pbprime_df,
            1/pbprime_df, massinv, pbprime_visc, btp_dpp_graduv(4), metrics(4), wjac_df),
            accumulators RMW 14P (ope2_ave_df, uvb_ave_df(2), graduvb_ave(4)), qb out 4P
     quad:  statics 15Q (wjac, coriolis, tau_wind(2), grad_zbot(2), 1/pbprime, H_bcl,
            Q_uu/uv/vv_dp, metrics(4)), accumulators RMW 24Q (12 fields)
  face    47*n + 46*m doubles per face
     traces 18n (qb both sides 8n, pbprime_df_face 2n, grad both sides 8n),
     statics 13n + 14m, accumulators RMW 16n + 32m
"""
from __future__ import annotations

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
HBM_MEASURED_GBS = 6290.0    # float4 copy measured on MI355X (same table)


def kernel_src_sha16() -> str:
    """sha256[:16] of the stage kernels' sources (csrc/kernels_btp.hip, csrc/engine_internal.h): the
    key that ties a committed PMC summary (profiles/roofline_pmc.json) to the kernels it measured."""
    import hashlib
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
    h = hashlib.sha256()
    for f in ("kernels_btp.hip", "engine_internal.h"):
        with open(os.path.join(d, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def stage_bytes_per_element(nop: int, faces_per_element: float) -> float:
    n, m = nop + 1, 2 * nop + 1
    P, Q = n * n, m * m
    return 8.0 * (44 * P + 39 * Q + faces_per_element * (47 * n + 46 * m))


def bcl_bytes_per_element(nop: int, nlayers: int, faces_per_element: float) -> float:
    """Algorithmic bytes of the baroclinic part of ONE step per element (same counting rule,
    per kernel family, predictor + corrector; P, Q, n, m as above, L layers):
      btp_bcl_coeffs_qdf  elem: qprime in 3PL, dpp_graduv out 4PL, dpprime_visc out PL,
                          Q_*/H_bcl out 4Q, btp_dpp_graduv + pbprime_visc out 5P
                          face: qprime faces 6nL, graduv_dpp_face out 10nL, edge coeffs 4m,
                          btp_graduv_dpp_face 10n
      layer mass          elem: qprime 3PL, dp in/out 2PL, dp' out PL, ope/uvb averages 3Q,
                          sum_layer_mass_flux 2Q;  face: qprime faces 6nL, face averages 6m,
                          flux mL, sums 2m
      consistency         elem: dp' PL, q 2PL, averages + sums 4Q;  face: dp' traces 2nL,
                          averages + sums 4m, flux mL
      layer momentum      elem: qprime 3PL, q in/out 6PL, qprime out 3PL, dpp_graduv 4PL,
                          dpprime_visc PL, qb 4P, 10 quad averages 10Q, 7 nodal averages 7P;
                          face: qprime faces 6nL, graduv_dpp_face 10nL, graduvb_face_ave 8n,
                          12 face averages 12m, fluxes 4mL, LDG 2nL
    i.e. per half-step 34PL + 23Q + 16P + F/E*(40nL + 6mL + 28m + 18n); twice per step.
    About 1 % of the sub-cycle's 2*N_btp*kstages stages."""
    n, m = nop + 1, 2 * nop + 1
    P, Q, L = n * n, m * m, nlayers
    half = 34 * P * L + 23 * Q + 16 * P + faces_per_element * (40 * n * L + 6 * m * L + 28 * m + 18 * n)
    return 8.0 * 2 * half


def owned_elements(case) -> int:
    """Elements this engine advances (a RankCase's ghosts are excluded)."""
    return int(getattr(case, "nelem_owned", 0) or case.scalars["nelem"])


def stage_bytes(case) -> float:
    """Algorithmic bytes of ONE btp_stage_kernel launch (all owned elements)."""
    S = case.scalars
    E, F = S["nelem"], S["nface"]
    return owned_elements(case) * stage_bytes_per_element(S["ngl"] - 1, F / E)


def step_bytes(case) -> float:
    """Algorithmic bytes of ONE baroclinic step: E*(2*N_btp*kstages*B_stage + B_bcl_step)."""
    S = case.scalars
    E, F = S["nelem"], S["nface"]
    return stage_bytes(case) * 2 * S["N_btp"] * S["kstages"] + \
        owned_elements(case) * bcl_bytes_per_element(S["ngl"] - 1, S["nlayers"], F / E)


def element_updates_per_step(case) -> int:
    S = case.scalars
    return owned_elements(case) * 2 * S["N_btp"] * S["kstages"]


def stage_bytes_cfg(cfg: dict) -> float:
    """stage_bytes of a brick configuration (hnumo.case.make_config) without building it:
    E = nelx*nely elements, F = (nelx+1)*nely + nelx*(nely+1) faces."""
    ex, ey = int(cfg["nelx"]), int(cfg["nely"])
    E, F = ex * ey, (ex + 1) * ey + ex * (ey + 1)
    return E * stage_bytes_per_element(int(cfg["nop"]), F / E)

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


def stage_bytes_per_element(nop: int, faces_per_element: float) -> float:
    n, m = nop + 1, 2 * nop + 1
    P, Q = n * n, m * m
    return 8.0 * (44 * P + 39 * Q + faces_per_element * (47 * n + 46 * m))


def stage_bytes(case) -> float:
    """Algorithmic bytes of ONE btp_stage_kernel launch (all elements)."""
    S = case.scalars
    E, F = S["nelem"], S["nface"]
    return E * stage_bytes_per_element(S["ngl"] - 1, F / E)


def element_updates_per_step(case) -> int:
    S = case.scalars
    return S["nelem"] * 2 * S["N_btp"] * S["kstages"]

"""Flat binary 'bundle' of every ti_rk_bcl input, readable from Fortran stream I/O.

Used to hand one Case to the reference harness (oracle/ref_driver.F90) and back.  The
layout is: int32[16] header, float64[8] header, then every array of BUNDLE_ARRAYS in
order, raw little-endian, Fortran (column-major) element order.
"""
from __future__ import annotations

import numpy as np

# (name, dtype, shape in terms of the header dims)
BUNDLE_ARRAYS = [
    ("face", "i4", "8,nface"), ("imapl", "i4", "3,ngl,nface"), ("imapr", "i4", "3,ngl,nface"),
    ("imapl_q", "i4", "3,nq,nface"), ("imapr_q", "i4", "3,nq,nface"),
    ("indexq", "i4", "npts,npoin_q"), ("index_df", "i4", "npts,npoin"),
    ("normal_vector", "f8", "3,ngl,nface"), ("normal_vector_q", "f8", "3,nq,nface"),
    ("jac_face", "f8", "ngl,nface"), ("jac_faceq", "f8", "nq,nface"), ("massinv", "f8", "npoin"),
    ("psiq", "f8", "ngl,nq"), ("dpsiq", "f8", "ngl,nq"), ("psi", "f8", "ngl,ngl"), ("dpsi", "f8", "ngl,ngl"),
    ("psih", "f8", "npts,npoin_q"), ("dpsidx", "f8", "npts,npoin_q"), ("dpsidy", "f8", "npts,npoin_q"),
    ("wjac", "f8", "npoin_q"), ("dpsidx_df", "f8", "npts,npoin"), ("dpsidy_df", "f8", "npts,npoin"),
    ("wjac_df", "f8", "npoin"),
    ("pbprime", "f8", "npoin_q"), ("pbprime_df", "f8", "npoin"), ("one_over_pbprime", "f8", "npoin_q"),
    ("one_over_pbprime_df", "f8", "npoin"), ("pbprime_face", "f8", "2,nq,nface"),
    ("pbprime_df_face", "f8", "2,ngl,nface"), ("one_over_pbprime_edge", "f8", "nq,nface"),
    ("coeff_pbpert_L", "f8", "nq,nface"), ("coeff_pbpert_R", "f8", "nq,nface"),
    ("coeff_pbub_LR", "f8", "nq,nface"), ("coeff_mass_pbub_L", "f8", "nq,nface"),
    ("coeff_mass_pbub_R", "f8", "nq,nface"), ("coeff_mass_pbpert_LR", "f8", "nq,nface"),
    ("alpha", "f8", "nlayers"), ("tau_wind", "f8", "2,npoin_q"), ("coriolis_quad", "f8", "npoin_q"),
    ("grad_zbot_quad", "f8", "2,npoin_q"), ("zbot_df", "f8", "npoin"), ("zbot_face", "f8", "2,nq,nface"),
    ("fdt2_bcl", "f8", "npoin"), ("a_bcl", "f8", "npoin"), ("b_bcl", "f8", "npoin"),
    ("ssprk_a", "f8", "kstages,3"), ("ssprk_beta", "f8", "kstages"),
    ("q_df", "f8", "3,npoin,nlayers"), ("qb_df", "f8", "4,npoin"), ("qprime_df", "f8", "3,npoin,nlayers"),
]

# optional trailer (dropin_driver): the per-point metrics of mod_metrics the bridge reads
METRIC_ARRAYS = [
    ("ksiq_x", "f8", "nq,nq,nelem"), ("ksiq_y", "f8", "nq,nq,nelem"), ("etaq_x", "f8", "nq,nq,nelem"),
    ("etaq_y", "f8", "nq,nq,nelem"), ("jacq", "f8", "nq,nq,nelem"),
    ("ksi_x", "f8", "ngl,ngl,nelem"), ("ksi_y", "f8", "ngl,ngl,nelem"), ("eta_x", "f8", "ngl,ngl,nelem"),
    ("eta_y", "f8", "ngl,ngl,nelem"), ("jac", "f8", "ngl,ngl,nelem"),
]

# engine / oracle fields copied out for parity (mod_variables), with shapes
FIELDS = [
    ("ope_ave", "npoin_q"), ("H_ave", "npoin_q"), ("Qu_ave", "npoin_q"), ("Qv_ave", "npoin_q"),
    ("Quv_ave", "npoin_q"), ("ope2_ave", "npoin_q"), ("btp_mass_flux_ave", "2,npoin_q"),
    ("uvb_ave", "2,npoin_q"), ("tau_bot_ave", "2,npoin_q"), ("tau_wind_ave", "2,npoin_q"),
    ("ope2_ave_df", "npoin"), ("uvb_ave_df", "2,npoin"), ("uvb_face_ave", "2,2,nq,nface"),
    ("btp_mass_flux_face_ave", "2,nq,nface"), ("ope_face_ave", "2,nq,nface"),
    ("ope2_face_ave", "2,nq,nface"), ("Qu_face_ave", "2,nq,nface"), ("Qv_face_ave", "2,nq,nface"),
    ("Quv_face_ave", "2,nq,nface"), ("H_face_ave", "nq,nface"), ("one_plus_eta_edge_2_ave", "nq,nface"),
    ("graduvb_ave", "4,npoin"), ("graduvb_face_ave", "4,2,ngl,nface"),
    ("Q_uu_dp", "npoin_q"), ("Q_uv_dp", "npoin_q"), ("Q_vv_dp", "npoin_q"), ("H_bcl", "npoin_q"),
    ("Q_uu_dp_edge", "nq,nface"), ("Q_uv_dp_edge", "nq,nface"), ("Q_vv_dp_edge", "nq,nface"),
    ("H_bcl_edge", "nq,nface"), ("btp_dpp_graduv", "4,npoin"), ("pbprime_visc", "npoin"),
    ("btp_graduv_dpp_face", "5,2,ngl,nface"), ("sum_layer_mass_flux", "2,npoin_q"),
    ("sum_layer_mass_flux_face", "2,nq,nface"),
]

MODES = {"rhs": 1, "btp": 2, "step": 3, "predict": 4, "diag": 5, "setup": 6, "geom": 7}
TEST_CASE_ID = {"bump": 1, "lakeAtrest": 2, "double-gyre": 3}

# outputs of mode "setup" (oracle/ref_driver.F90 mode 6: the reference's own start-up routines)
SETUP_OUT = [
    ("q_df", "3,npoin,nlayers"), ("qb_df", "4,npoin"), ("qprime_df", "3,npoin,nlayers"), ("pbprime", "npoin_q"),
    ("pbprime_df", "npoin"), ("pbprime_face", "2,nq,nface"), ("pbprime_df_face", "2,ngl,nface"),
    ("one_over_pbprime", "npoin_q"), ("one_over_pbprime_df", "npoin"), ("one_over_pbprime_edge", "nq,nface"),
    ("coeff_pbpert_L", "nq,nface"), ("coeff_pbpert_R", "nq,nface"), ("coeff_pbub_LR", "nq,nface"),
    ("coeff_mass_pbub_L", "nq,nface"), ("coeff_mass_pbub_R", "nq,nface"), ("coeff_mass_pbpert_LR", "nq,nface"),
    ("alpha", "nlayers"), ("zbot_df", "npoin"), ("zbot_face", "2,nq,nface"), ("grad_zbot_quad", "2,npoin_q"),
    ("tau_wind", "2,npoin_q"), ("coriolis_quad", "npoin_q"), ("fdt2_bcl", "npoin"), ("a_bcl", "npoin"),
    ("b_bcl", "npoin"), ("ssprk_a", "kstages,3"), ("ssprk_beta", "kstages"), ("N_btp", "1"), ("dt_btp", "1"),
    ("gravity", "1"),
]


def dims(case) -> dict:
    S = case.scalars
    return dict(nelem=S["nelem"], npoin=S["npoin"], npoin_q=S["npoin_q"], nface=S["nface"],
                ngl=S["ngl"], nq=S["nq"], nlayers=S["nlayers"], npts=S["ngl"] ** 2,
                kstages=S["kstages"])


def shape_of(expr: str, d: dict):
    return tuple(int(eval(t, {}, d)) for t in expr.split(","))


def write_bundle(path: str, case, mode: str, nsteps: int = 1, metrics: bool = False):
    """metrics=True appends METRIC_ARRAYS (read only by oracle/_ref/dropin_driver)."""
    S = case.scalars
    d = dims(case)
    hi = np.zeros(16, dtype="<i4")
    hi[:14] = [S["nelem"], S["npoin"], S["npoin_q"], S["nface"], S["ngl"], S["nq"], S["nlayers"],
               S["ngl"] - 1, S["kstages"], S["N_btp"], S["method_visc"], S["botfr"], nsteps, MODES[mode]]
    hi[14] = 1 if getattr(case, "halo_kind", None) == "faces" else 0      # halo trailer present
    if mode == "setup":
        hi[15] = TEST_CASE_ID[case.cfg["test_case"]]
    hd = np.zeros(8, dtype="<f8")
    hd[:7] = [S["dt"], S["dt_btp"], S["visc"], S["cd"], S["ad"], S["gravity"], S["max_shear_dz"]]
    with open(path, "wb") as fh:
        fh.write(hi.tobytes())
        fh.write(hd.tobytes())
        trailer = (METRIC_ARRAYS if metrics else []) + ([("coord", "f8", "3,npoin")] if mode in ("diag", "geom") else [])
        if mode == "setup":
            trailer = METRIC_ARRAYS[:5] + [("coord", "f8", "3,npoin")]
        for name, dt, shp in BUNDLE_ARRAYS + trailer:
            a = np.asarray(case.arrays[name])
            want = shape_of(shp, d)
            assert a.size == int(np.prod(want)), (name, a.shape, want)
            fh.write(np.asarray(a, dtype="<" + dt).ravel(order="F").tobytes())
        if mode == "setup":
            c = case.cfg
            sp = [c["xdims"][0], c["xdims"][1], c["ydims"][0], c["ydims"][1], c["f0"], c["beta"]]
            fh.write(np.asarray(sp, dtype="<f8").tobytes())
        if hi[14]:
            # processor-face halo (mod_parallel): num_nbh, nbh_proc, num_send_recv, nbh_send_recv
            from .facepart import halo_lists
            nbh_proc, num, lst, _ = halo_lists(case)
            fh.write(np.array([nbh_proc.size, lst.size], dtype="<i4").tobytes())
            for a in (nbh_proc, num, lst):
                fh.write(np.asarray(a, dtype="<i4").tobytes())


def read_outputs(path: str, case, mode: str) -> dict:
    """Outputs of the reference harness: state (+ rhs for mode 'rhs'), FIELDS, reference basis."""
    d = dims(case)
    raw = np.fromfile(path, dtype="<f8")
    off = 0
    out = {}

    def take(name, shp):
        nonlocal off
        n = int(np.prod(shp))
        out[name] = raw[off:off + n].reshape(shp, order="F").copy()
        off += n

    take("q_df", shape_of("3,npoin,nlayers", d))
    take("qb_df", shape_of("4,npoin", d))
    take("qprime_df", shape_of("3,npoin,nlayers", d))
    take("rhs", shape_of("3,npoin", d))
    for name, shp in FIELDS:
        take(name, shape_of(shp, d))
    ngl, nq = d["ngl"], d["nq"]
    take("ref_xgl", (ngl,))
    take("ref_wgl", (ngl,))
    take("ref_xnq", (nq,))
    take("ref_wnq", (nq,))
    take("ref_psiq", (ngl, nq))
    take("ref_dpsiq", (ngl, nq))
    take("ref_psi", (ngl, ngl))
    take("ref_dpsi", (ngl, ngl))
    assert off == raw.size, (off, raw.size)
    return out


# outputs of mode "geom" (oracle/ref_driver.F90 mode 7: the reference's metrics, metrics_quad,
# create_normals and create_normals_quad on the bundle's node coordinates and faces)
GEOM_OUT = [
    ("ksi_x", "ngl,ngl,nelem"), ("ksi_y", "ngl,ngl,nelem"), ("eta_x", "ngl,ngl,nelem"), ("eta_y", "ngl,ngl,nelem"),
    ("jac", "ngl,ngl,nelem"), ("ksiq_x", "nq,nq,nelem"), ("ksiq_y", "nq,nq,nelem"), ("etaq_x", "nq,nq,nelem"),
    ("etaq_y", "nq,nq,nelem"), ("jacq", "nq,nq,nelem"), ("normal_vector", "3,ngl,nface"), ("jac_face", "ngl,nface"),
    ("normal_vector_q", "3,nq,nface"), ("jac_faceq", "nq,nface"),
]


def read_geom_outputs(path: str, case) -> dict:
    """Outputs of the reference harness in mode "geom" (GEOM_OUT order)."""
    d = dims(case)
    raw = np.fromfile(path, dtype="<f8")
    off, out = 0, {}
    for name, shp in GEOM_OUT:
        s = shape_of(shp, d)
        n = int(np.prod(s))
        out[name] = raw[off:off + n].reshape(s, order="F").copy()
        off += n
    assert off == raw.size, (off, raw.size)
    return out


def read_setup_outputs(path: str, case) -> dict:
    """Outputs of the reference harness in mode "setup" (SETUP_OUT order)."""
    d = dims(case)
    raw = np.fromfile(path, dtype="<f8")
    off, out = 0, {}
    for name, shp in SETUP_OUT:
        s = shape_of(shp, d)
        n = int(np.prod(s))
        out[name] = raw[off:off + n].reshape(s, order="F").copy()
        off += n
    assert off == raw.size, (off, raw.size)
    return out

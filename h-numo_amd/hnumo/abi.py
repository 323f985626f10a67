"""ctypes mirror of include/hnumo_engine.h (descriptor structs) and helpers that fill
them from a Case.  No torch types cross the boundary: plain pointers and sizes."""
from __future__ import annotations

import ctypes as C

import numpy as np

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class MeshDesc(C.Structure):
    _fields_ = [
        ("nelem", C.c_int32), ("npoin", C.c_int32), ("npoin_q", C.c_int32), ("nface", C.c_int32),
        ("ngl", C.c_int32), ("nq", C.c_int32), ("nlayers", C.c_int32),
        ("face", _ip), ("imapl", _ip), ("imapr", _ip),
        ("normal_vector", _dp), ("normal_vector_q", _dp), ("jac_face", _dp), ("jac_faceq", _dp),
        ("massinv", _dp), ("psiq", _dp), ("dpsiq", _dp), ("psi", _dp), ("dpsi", _dp),
        ("ksiq_x", _dp), ("ksiq_y", _dp), ("etaq_x", _dp), ("etaq_y", _dp), ("jacq", _dp),
        ("ksi_x", _dp), ("ksi_y", _dp), ("eta_x", _dp), ("eta_y", _dp), ("jac", _dp),
        ("psih", _dp), ("dpsidx", _dp), ("dpsidy", _dp), ("wjac", _dp), ("indexq", _ip),
        ("dpsidx_df", _dp), ("dpsidy_df", _dp), ("wjac_df", _dp), ("index_df", _ip),
        ("imapl_q", _ip), ("imapr_q", _ip),
    ]


class StaticDesc(C.Structure):
    _fields_ = [(n, _dp) for n in (
        "pbprime", "pbprime_df", "one_over_pbprime", "one_over_pbprime_df", "pbprime_face",
        "pbprime_df_face", "one_over_pbprime_edge", "coeff_pbpert_L", "coeff_pbpert_R",
        "coeff_pbub_LR", "coeff_mass_pbub_L", "coeff_mass_pbub_R", "coeff_mass_pbpert_LR",
        "alpha", "tau_wind", "coriolis_quad", "grad_zbot_quad", "zbot_df", "zbot_face",
        "fdt2_bcl", "a_bcl", "b_bcl", "ssprk_a", "ssprk_beta")]


class Params(C.Structure):
    _fields_ = [
        ("dt", C.c_double), ("dt_btp", C.c_double), ("visc_mlswe", C.c_double),
        ("cd_mlswe", C.c_double), ("ad_mlswe", C.c_double), ("gravity", C.c_double),
        ("N_btp", C.c_int32), ("kstages", C.c_int32), ("method_visc", C.c_int32), ("botfr", C.c_int32),
        ("max_shear_dz", C.c_double), ("shear_corrector", C.c_int32), ("reserved", C.c_int32),
    ]


class HaloDesc(C.Structure):
    _fields_ = [
        ("rank", C.c_int32), ("nranks", C.c_int32), ("num_nbh", C.c_int32),
        ("nbh_proc", _ip), ("num_send_recv", _ip), ("nbh_send_recv", _ip),
        ("comm_id", C.POINTER(C.c_ubyte)),
        ("nelem_owned", C.c_int32), ("num_ghost_send", _ip), ("ghost_send", _ip),
        ("num_ghost_recv", _ip), ("ghost_recv", _ip),
    ]


class Halo:
    """HaloDesc for a multi-rank case (keeps the index arrays alive): a hnumo.facepart.FaceRankCase
    (the reference's processor-face lists, mod_parallel) or a hnumo.partition.RankCase (ghost
    elements)."""

    def __init__(self, rc, comm_id: bytes | None = None):
        if getattr(rc, "halo_kind", None) == "faces":
            self._faces(rc, comm_id)
            return
        nb = rc.neighbours
        self.keep = {
            "nbh_proc": np.array([n.rank for n in nb], dtype=np.int32),
            "num_send_recv": np.zeros(len(nb), dtype=np.int32),
            "num_ghost_send": np.array([len(n.send) for n in nb], dtype=np.int32),
            "ghost_send": np.concatenate([np.asarray(n.send, dtype=np.int32) + 1 for n in nb]
                                         or [np.zeros(0, np.int32)]).astype(np.int32),
            "num_ghost_recv": np.array([len(n.recv) for n in nb], dtype=np.int32),
            "ghost_recv": np.concatenate([np.asarray(n.recv, dtype=np.int32) + 1 for n in nb]
                                         or [np.zeros(0, np.int32)]).astype(np.int32),
        }
        h = HaloDesc()
        h.rank, h.nranks, h.num_nbh, h.nelem_owned = rc.rank, rc.nranks, len(nb), rc.nelem_owned
        for k, v in self.keep.items():
            setattr(h, k, v.ctypes.data_as(_ip) if v.size else None)
        self._comm(h, comm_id)
        self.desc = h

    def _comm(self, h, comm_id):
        if comm_id is not None:
            self.keep["comm_id"] = np.frombuffer(bytearray(comm_id), dtype=np.uint8).copy()
            h.comm_id = self.keep["comm_id"].ctypes.data_as(C.POINTER(C.c_ubyte))

    def _faces(self, rc, comm_id):
        from .facepart import halo_lists
        nbh_proc, num, lst, _ = halo_lists(rc)
        self.keep = {"nbh_proc": nbh_proc, "num_send_recv": num, "nbh_send_recv": lst}
        h = HaloDesc()
        h.rank, h.nranks, h.num_nbh, h.nelem_owned = rc.rank, rc.nranks, nbh_proc.size, rc.scalars["nelem"]
        for k, v in self.keep.items():
            setattr(h, k, v.ctypes.data_as(_ip) if v.size else None)
        self._comm(h, comm_id)
        self.desc = h


def ptr(a: np.ndarray | None):
    """Pointer to a contiguous Fortran-order array (keeps no reference: caller owns it)."""
    if a is None:
        return None
    if a.dtype == np.int32:
        return a.ctypes.data_as(_ip)
    assert a.dtype == np.float64, a.dtype
    return a.ctypes.data_as(_dp)


def _f(a: np.ndarray, dtype):
    """Flat contiguous copy in Fortran element order."""
    return np.ascontiguousarray(np.asarray(a, dtype=dtype).ravel(order="F"))


class Descriptors:
    """Builds and owns (keeps alive) the flat arrays behind the three descriptors."""

    MESH_F8 = ["normal_vector", "normal_vector_q", "jac_face", "jac_faceq", "massinv", "psiq", "dpsiq",
               "psi", "dpsi", "ksiq_x", "ksiq_y", "etaq_x", "etaq_y", "jacq", "ksi_x", "ksi_y", "eta_x",
               "eta_y", "jac"]
    DENSE_F8 = ["psih", "dpsidx", "dpsidy", "wjac", "dpsidx_df", "dpsidy_df", "wjac_df"]
    DENSE_I4 = ["indexq", "index_df"]

    def __init__(self, case, dense: bool = False):
        A, S = case.arrays, case.scalars
        self.keep = {}
        for k in ("face", "imapl", "imapr", "imapl_q", "imapr_q"):
            self.keep[k] = _f(A[k], np.int32)
        for k in self.MESH_F8:
            self.keep[k] = _f(A[k], np.float64)
        if dense:
            for k in self.DENSE_F8:
                self.keep[k] = _f(A[k], np.float64)
            for k in self.DENSE_I4:
                self.keep[k] = _f(A[k], np.int32)
        for name, _ in StaticDesc._fields_:
            self.keep["s_" + name] = _f(A[name], np.float64)
        m = MeshDesc()
        for k in ("nelem", "npoin", "npoin_q", "nface", "ngl", "nq", "nlayers"):
            setattr(m, k, S[k])
        for k in ["face", "imapl", "imapr", "imapl_q", "imapr_q"] + self.MESH_F8:
            setattr(m, k, ptr(self.keep[k]))
        if dense:
            for k in self.DENSE_F8 + self.DENSE_I4:
                setattr(m, k, ptr(self.keep[k]))
        s = StaticDesc()
        for name, _ in StaticDesc._fields_:
            setattr(s, name, ptr(self.keep["s_" + name]))
        p = Params(dt=S["dt"], dt_btp=S["dt_btp"], visc_mlswe=S["visc"], cd_mlswe=S["cd"],
                   ad_mlswe=S["ad"], gravity=S["gravity"], N_btp=S["N_btp"], kstages=S["kstages"],
                   method_visc=S["method_visc"], botfr=S["botfr"],
                   max_shear_dz=S["max_shear_dz"], shear_corrector=S["shear_corrector"])
        self.mesh, self.statics, self.params = m, s, p

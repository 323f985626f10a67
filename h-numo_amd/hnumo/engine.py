"""Python host mirror of the reference's engine boundary (ti_rk_bcl and its parity hooks)
over the C ABI of libhnumo_engine.so (include/hnumo_engine.h).

The product path is the HIP library; there is no CPU fallback.  Loading fails loudly if
the library is missing or no GPU is visible.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import bundle as _bundle
from .abi import Descriptors, Halo, HaloDesc

LIB_PATH = os.environ.get("HNUMO_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "libhnumo_engine.so")  # HNUMO_LIB: A/B experiments only
_lib = None

ERRORS = {1: "negative layer thickness", 2: "non-finite value", 3: "HIP/RCCL error", 4: "invalid argument"}


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"hnumo engine error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


def lib():
    """Load libhnumo_engine.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        vp, dp = C.c_void_p, C.POINTER(C.c_double)
        L.hnumo_engine_create.argtypes = [vp, vp, vp, vp, C.c_int, C.POINTER(vp)]
        L.hnumo_engine_destroy.argtypes = [vp]
        L.hnumo_last_error.argtypes = [vp]
        L.hnumo_last_error.restype = C.c_char_p
        L.hnumo_ti_rk_bcl.argtypes = [vp, dp, dp, dp]
        L.hnumo_ti_barotropic_ssprk.argtypes = [vp, dp, dp]
        L.hnumo_predict.argtypes = [vp, dp, dp, dp]
        L.hnumo_btp_bcl_coeffs.argtypes = [vp, dp]
        L.hnumo_create_rhs_btp.argtypes = [vp, dp, dp, dp]
        L.hnumo_get_field.argtypes = [vp, C.c_char_p, dp, C.c_int64]
        L.hnumo_set_resident.argtypes = [vp, C.c_int]
        L.hnumo_sync.argtypes = [vp, dp, dp, dp]
        L.hnumo_bench_steps.argtypes = [vp, C.c_int, dp, dp, C.POINTER(C.c_int64)]
        L.hnumo_abi_version.restype = C.c_int
        L.hnumo_time_stage_kernel.argtypes = [vp, C.c_int, dp]
        L.hnumo_rccl_unique_id.argtypes = [C.POINTER(C.c_ubyte)]
        L.hnumo_local_group.argtypes = [C.POINTER(vp), C.c_int]
        L.hnumo_group_ti_rk_bcl.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(dp), C.POINTER(dp), C.POINTER(dp)]
        L.hnumo_debug_stage_profile.argtypes = [vp, C.POINTER(C.c_uint64), C.c_int64]
        L.hnumo_set_summation.argtypes = [vp, C.c_int]
        L.hnumo_get_summation.argtypes = [vp]
        L.hnumo_get_summation.restype = C.c_int
        L.hnumo_stage_path.argtypes = [vp]
        L.hnumo_stage_path.restype = C.c_int
        L.hnumo_persistent_info.argtypes = [vp, C.POINTER(C.c_int32)]
        L.hnumo_persistent_stats.argtypes = [vp, C.POINTER(C.c_int32)]
        L.hnumo_debug_force_abort.argtypes = [vp, C.c_int]
        L.hnumo_debug_frozen_halo.argtypes = [vp, C.c_int]
        L.hnumo_step_breakdown.argtypes = [vp, C.c_int, C.c_char_p, C.c_int64, dp, C.c_int, C.POINTER(C.c_int)]
        L.hnumo_stream_copy_bw.argtypes = [C.c_int, C.c_int64, C.c_int, dp]
        L.hnumo_overrides.argtypes = [vp, C.c_char_p, C.c_int64]
        _lib = L
    return _lib


def _dp(a, size=None, name="array"):
    """Pointer to a float64 Fortran-contiguous array of exactly `size` elements (the C side
    reads and writes fixed-size blocks, so a wrong shape must never reach it)."""
    if not isinstance(a, np.ndarray) or a.dtype != np.float64 or not a.flags["F_CONTIGUOUS"]:
        raise ValueError(f"{name}: need a Fortran-contiguous float64 numpy array")
    if not a.flags["WRITEABLE"]:
        raise ValueError(f"{name}: array is read-only")
    if size is not None and a.size != size:
        raise ValueError(f"{name}: {a.size} elements, expected {size}")
    return a.ctypes.data_as(C.POINTER(C.c_double))


SUMMATION = {"reference": 0, "factored": 1}   # HNUMO_SUM_REFERENCE / HNUMO_SUM_FACTORED


class Engine:
    """One engine per GPU: device-resident ti_rk_bcl for one Case."""

    def __init__(self, case, device: int = 0, halo: HaloDesc | None = None, comm_id: bytes | None = None,
                 summation: str | None = None):
        """case: a hnumo.case.Case, or a hnumo.partition.RankCase (multi-rank; its ghost-layer
        halo is passed to the engine, with RCCL when comm_id is given).  summation:
        "reference" (the default: bit-identical to the reference order) or "factored"
        (sum-factorised, faster, ~1e-7 relative from the reference; see hnumo_set_summation)."""
        self.case = case
        self.desc = Descriptors(case, dense=False)
        self.dims = _bundle.dims(case)
        self.h = C.c_void_p()
        if halo is None and (getattr(case, "nranks", 1) > 1 or getattr(case, "fneighbours", None)):
            self._halo = Halo(case, comm_id)
            halo = self._halo.desc
        self.halo = halo
        L = lib()
        rc = L.hnumo_engine_create(C.byref(self.desc.mesh), C.byref(self.desc.statics), C.byref(self.desc.params),
                                   C.byref(halo) if halo is not None else None, device, C.byref(self.h))
        if rc:
            msg = L.hnumo_last_error(self.h).decode()
            self._destroy()
            raise EngineError(rc, msg)
        if summation is not None:
            self.set_summation(summation)

    def _check(self, rc):
        if rc:
            raise EngineError(rc, lib().hnumo_last_error(self.h).decode())

    def state(self):
        A = self.case.arrays
        return (np.array(A["q_df"], order="F"), np.array(A["qb_df"], order="F"),
                np.array(A["qprime_df"], order="F"))

    # sizes of q_df(3,npoin,L), qb_df(4,npoin), qprime_df(3,npoin,L)
    def _sizes(self):
        d = self.dims
        return 3 * d["npoin"] * d["nlayers"], 4 * d["npoin"], 3 * d["npoin"] * d["nlayers"]

    def _state_ptrs(self, q, qb, qp):
        nq, nb, np_ = self._sizes()
        return _dp(q, nq, "q_df"), _dp(qb, nb, "qb_df"), _dp(qp, np_, "qprime_df")

    # = ti_rk_bcl (ti_rk_bcl.F90:9)
    def ti_rk_bcl(self, q, qb, qp):
        self._check(lib().hnumo_ti_rk_bcl(self.h, *self._state_ptrs(q, qb, qp)))

    # = the prediction half of ti_rk_bcl (ti_rk_bcl.F90:43-57): q, qb, qp become q_df2, the
    # sub-cycled qb_df and qprime_df2
    def predict(self, q, qb, qp):
        self._check(lib().hnumo_predict(self.h, *self._state_ptrs(q, qb, qp)))

    def btp_bcl_coeffs(self, qp):
        self._check(lib().hnumo_btp_bcl_coeffs(self.h, _dp(qp, self._sizes()[2], "qprime_df")))

    # = ti_barotropic_ssprk_mlswe (mod_rk_mlswe.F90:19)
    def ti_barotropic_ssprk(self, qb, qp):
        _, nb, np_ = self._sizes()
        self._check(lib().hnumo_ti_barotropic_ssprk(self.h, _dp(qb, nb, "qb_df"), _dp(qp, np_, "qprime_df")))

    # = create_rhs_btp (mod_rhs_btp.F90:28)
    def create_rhs_btp(self, qb, qp):
        _, nb, np_ = self._sizes()
        rhs = np.zeros((3, self.dims["npoin"]), order="F")
        self._check(lib().hnumo_create_rhs_btp(self.h, _dp(rhs), _dp(qb, nb, "qb_df"), _dp(qp, np_, "qprime_df")))
        return rhs

    def field(self, name):
        shp = dict(_bundle.FIELDS)[name]
        out = np.zeros(_bundle.shape_of(shp, self.dims), order="F")
        self._check(lib().hnumo_get_field(self.h, name.encode(), _dp(out), out.size))
        return out

    def set_summation(self, mode: str):
        self._check(lib().hnumo_set_summation(self.h, SUMMATION[mode]))

    @property
    def summation(self) -> str:
        return {v: k for k, v in SUMMATION.items()}[lib().hnumo_get_summation(self.h)]

    @property
    def stage_path(self) -> str:
        """'persistent' (one launch per sub-cycle) or 'per-stage' (one launch per stage)."""
        return "persistent" if lib().hnumo_stage_path(self.h) == 1 else "per-stage"

    @property
    def persistent_info(self) -> dict:
        """Residency of the persistent sub-cycle launch (hnumo_persistent_info)."""
        out = (C.c_int32 * 8)()
        self._check(lib().hnumo_persistent_info(self.h, out))
        v = list(out)
        return {"persistent": v[0] == 1, "occupancy_blocks_per_cu": (v[1], v[2]), "cus": v[3],
                "trial_launch": (v[4], v[5]), "fallbacks": v[6], "lds_bytes_per_workgroup": v[7]}

    @property
    def persistent_stats(self) -> dict:
        """The persistent path's in-launch residency check over the engine's life
        (hnumo_persistent_stats): launches that gave up, trial re-probes, re-probes that found the
        grid resident again, and the runs left before the next re-probe (-1: not suspended)."""
        out = (C.c_int32 * 4)()
        self._check(lib().hnumo_persistent_stats(self.h, out))
        v = list(out)
        return {"aborts": v[0], "reprobes": v[1], "recovered": v[2], "wait": v[3]}

    @property
    def overrides(self) -> list:
        """The HNUMO_* environment settings this engine read at create (hnumo_overrides):
        "NAME=value", with " (ignored: HNUMO_EXPERIMENTS!=1)" for experiment knobs not honoured."""
        buf = C.create_string_buffer(4096)
        self._check(lib().hnumo_overrides(self.h, buf, len(buf)))
        return [x for x in buf.value.decode().split(";") if x]

    def debug_force_abort(self, k: int):
        """Test hook: the k-th persistent sub-cycle launch from now (0 = the next) gives up as a
        launch whose workgroups are not co-resident does (hnumo_debug_force_abort)."""
        self._check(lib().hnumo_debug_force_abort(self.h, int(k)))

    def debug_frozen_halo(self, on: bool = True):
        """Emulation hook (self-neighbour engines only, bench.py --emulate): every halo exchange
        site sends its first message again and again -- an at-rest neighbour for an at-rest case
        (hnumo_debug_frozen_halo).  Set before the first step."""
        self._check(lib().hnumo_debug_frozen_halo(self.h, int(on)))

    def set_resident(self, on: bool):
        self._check(lib().hnumo_set_resident(self.h, int(on)))

    def sync(self, q, qb, qp):
        self._check(lib().hnumo_sync(self.h, *self._state_ptrs(q, qb, qp)))

    def bench_steps(self, nsteps: int):
        t = C.c_double()
        k = C.c_double()
        n = C.c_int64()
        self._check(lib().hnumo_bench_steps(self.h, nsteps, C.byref(t), C.byref(k), C.byref(n)))
        return t.value, k.value, n.value

    def time_stage_kernel(self, nsubcycles: int = 2) -> float:
        """Average btp_stage_kernel duration (ms), HIP events on the engine stream."""
        k = C.c_double()
        self._check(lib().hnumo_time_stage_kernel(self.h, nsubcycles, C.byref(k)))
        return k.value

    def stage_profile(self):
        n = self.dims["nelem"] * 32
        out = np.zeros(n, dtype=np.uint64)
        self._check(lib().hnumo_debug_stage_profile(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), n))
        return out.reshape(-1, 32)

    def step_breakdown(self, nsteps: int = 2) -> dict:
        """Microseconds per step of every kernel family of the step, in launch order
        (hnumo_step_breakdown: direct launches with an event after each; the state advances)."""
        names = C.create_string_buffer(4096)
        us = (C.c_double * 64)()
        n = C.c_int()
        self._check(lib().hnumo_step_breakdown(self.h, nsteps, names, len(names), us, 64, C.byref(n)))
        keys = names.value.decode().split("\n") if n.value else []
        return {k: us[i] for i, k in enumerate(keys)}

    @staticmethod
    def stream_copy_bw(device: int = 0, nbytes: int = 1 << 30, reps: int = 10) -> tuple:
        """(GB/s, variant) of the fastest 16-byte stream copy between two buffers of nbytes, reps
        launches back to back (read + write counted; hnumo_stream_copy_bw)."""
        out = (C.c_double * 2)()
        rc = lib().hnumo_stream_copy_bw(device, nbytes, reps, out)
        if rc:
            raise EngineError(rc, "stream copy measurement failed")
        return out[0], out[1]

    @staticmethod
    def rccl_unique_id() -> bytes:
        buf = (C.c_ubyte * 128)()
        rc = lib().hnumo_rccl_unique_id(buf)
        if rc:
            raise EngineError(rc, "ncclGetUniqueId failed")
        return bytes(buf)

    def _destroy(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().hnumo_engine_destroy(self.h)
            self.h = C.c_void_p()

    def close(self):
        self._destroy()

    def __del__(self):
        try:
            self._destroy()
        except Exception:
            pass


def local_group(engines):
    """Join the engines of one process (ranks 0..n-1, same device) into a local exchange group."""
    arr = (C.c_void_p * len(engines))(*[e.h.value for e in engines])
    rc = lib().hnumo_local_group(arr, len(engines))
    if rc:
        raise EngineError(rc, "hnumo_local_group failed (ranks must be 0..n-1 on one device)")
    for e in engines:
        e._group = arr


def group_ti_rk_bcl(engines, states):
    """One baroclinic step of every engine of a local group; states[i] = (q, qb, qp) arrays."""
    n = len(engines)
    if len(states) != n:
        raise ValueError("one (q, qb, qp) state per engine")
    arr = engines[0]._group
    ptrs = [e._state_ptrs(*states[i]) for i, e in enumerate(engines)]
    mk = lambda j: (C.POINTER(C.c_double) * n)(*[ptrs[i][j] for i in range(n)])
    rc = lib().hnumo_group_ti_rk_bcl(arr, n, mk(0), mk(1), mk(2))
    if rc:
        msgs = [lib().hnumo_last_error(e.h).decode() for e in engines]
        raise EngineError(rc, "; ".join(m for m in msgs if m))

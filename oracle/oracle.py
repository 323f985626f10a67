"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU oracle (oracle/hnumo_oracle.c)
and a runner for the reference harness (oracle/_ref/ref_driver).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "h-numo_amd"))
from hnumo.abi import Descriptors  # noqa: E402
from hnumo import bundle as _bundle  # noqa: E402

LIB_PATH = os.path.join(HERE, "libhnumo_oracle.so")
REF_DRIVER = os.path.join(HERE, "_ref", "ref_driver")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "libhnumo_oracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, dp = C.c_void_p, C.POINTER(C.c_double)
        L.oracle_create.argtypes = [vp, vp, vp, C.POINTER(vp)]
        L.oracle_ti_rk_bcl.argtypes = [vp, dp, dp, dp]
        L.oracle_predict.argtypes = [vp, dp, dp, dp]
        L.oracle_ti_barotropic_ssprk.argtypes = [vp, dp, dp]
        L.oracle_btp_bcl_coeffs.argtypes = [vp, dp]
        L.oracle_create_rhs_btp.argtypes = [vp, dp, dp, dp]
        L.oracle_get_field.argtypes = [vp, C.c_char_p, dp, C.c_int64]
        L.oracle_zero_accumulators.argtypes = [vp]
        L.oracle_destroy.argtypes = [vp]
        L.oracle_last_error.argtypes = [vp]
        L.oracle_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Oracle:
    """CPU restatement of ti_rk_bcl on one Case (state arrays in Fortran layout)."""

    def __init__(self, case):
        self.case = case
        self.desc = Descriptors(case, dense=True)
        self.h = C.c_void_p()
        L = lib()
        rc = L.oracle_create(C.byref(self.desc.mesh), C.byref(self.desc.statics),
                             C.byref(self.desc.params), C.byref(self.h))
        if rc:
            raise RuntimeError(L.oracle_last_error(self.h).decode())
        d = _bundle.dims(case)
        self.dims = d

    def _check(self, rc):
        if rc:
            raise RuntimeError(f"oracle rc={rc}: {lib().oracle_last_error(self.h).decode()}")

    def state(self):
        A = self.case.arrays
        return (np.array(A["q_df"], order="F"), np.array(A["qb_df"], order="F"),
                np.array(A["qprime_df"], order="F"))

    def ti_rk_bcl(self, q, qb, qp):
        self._check(lib().oracle_ti_rk_bcl(self.h, _dp(q), _dp(qb), _dp(qp)))

    def predict(self, q, qb, qp):
        """The prediction half of ti_rk_bcl (ti_rk_bcl.F90:43-57) in place (momentum_mass hook)."""
        self._check(lib().oracle_predict(self.h, _dp(q), _dp(qb), _dp(qp)))

    def btp_bcl_coeffs(self, qp):
        self._check(lib().oracle_btp_bcl_coeffs(self.h, _dp(qp)))

    def ti_barotropic_ssprk(self, qb, qp):
        self._check(lib().oracle_ti_barotropic_ssprk(self.h, _dp(qb), _dp(qp)))

    def create_rhs_btp(self, qb, qp):
        rhs = np.zeros((3, self.dims["npoin"]), order="F")
        lib().oracle_zero_accumulators(self.h)
        self._check(lib().oracle_create_rhs_btp(self.h, _dp(rhs), _dp(qb), _dp(qp)))
        return rhs

    def field(self, name):
        shp = dict(_bundle.FIELDS)[name]
        shape = _bundle.shape_of(shp, self.dims)
        out = np.zeros(shape, order="F")
        self._check(lib().oracle_get_field(self.h, name.encode(), _dp(out), out.size))
        return out

    def __del__(self):
        if getattr(self, "h", None) and self.h.value:
            lib().oracle_destroy(self.h)
            self.h = C.c_void_p()


DROPIN_DRIVER = os.path.join(os.path.dirname(REF_DRIVER), "dropin_driver")


def run_reference(case, mode: str, nsteps: int = 1, workdir: str | None = None, dropin: bool = False) -> dict:
    """Run the reference Fortran (oracle/_ref/ref_driver) on `case`; returns its outputs.

    dropin=True runs oracle/_ref/dropin_driver instead: the same Fortran harness with
    ti_rk_bcl replaced by the HIP engine through the Fortran bridge (mode "step" only; GPU)."""
    driver = DROPIN_DRIVER if dropin else REF_DRIVER
    if not os.path.exists(driver):
        raise FileNotFoundError(driver)
    tmp = workdir or tempfile.mkdtemp(prefix="hnumo_ref_")
    fin = os.path.join(tmp, "bundle.bin")
    fout = os.path.join(tmp, "out.bin")
    _bundle.write_bundle(fin, case, mode, nsteps, metrics=dropin)
    env = dict(os.environ)
    def _stack():
        # the reference keeps npoin-sized automatic arrays on the stack (e.g. ti_rk_bcl.F90:35-38)
        import resource
        resource.setrlimit(resource.RLIMIT_STACK, (resource.RLIM_INFINITY, resource.RLIM_INFINITY))

    r = subprocess.run([driver, fin, fout], env=env, cwd=tmp, preexec_fn=_stack,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{os.path.basename(driver)} failed ({r.returncode}): {r.stdout[-2000:]} {r.stderr[-2000:]}")
    if mode == "setup":
        out = _bundle.read_setup_outputs(fout, case)
    elif mode == "geom":
        out = _bundle.read_geom_outputs(fout, case)
    else:
        out = _bundle.read_outputs(fout, case, mode)
    out["stdout"] = r.stdout
    if workdir is None:
        for f in (fin, fout):
            os.remove(f)
        os.rmdir(tmp)
    return out


MPIEXEC = os.environ.get("HNUMO_MPIEXEC", "/opt/conda/bin/mpiexec")


def run_reference_mpi(parts, mode: str, nsteps: int = 1) -> list:
    """Run the reference Fortran under `mpiexec -n len(parts)` on a processor-face partition
    (hnumo.facepart.face_partition, one FaceRankCase per rank): every rank reads its own bundle
    and the reference's own MPI halo exchange runs.  Returns the outputs of every rank."""
    if not os.path.exists(REF_DRIVER):
        raise FileNotFoundError(REF_DRIVER)
    tmp = tempfile.mkdtemp(prefix="hnumo_refmpi_")
    fin, fout = os.path.join(tmp, "bundle.bin"), os.path.join(tmp, "out.bin")
    for r, pc in enumerate(parts):
        _bundle.write_bundle(f"{fin}.{r}", pc, mode, nsteps)

    def _stack():
        import resource
        resource.setrlimit(resource.RLIMIT_STACK, (resource.RLIM_INFINITY, resource.RLIM_INFINITY))

    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [MPIEXEC, "-launcher", "fork", "-n", str(len(parts)), REF_DRIVER, fin, fout]
    r = subprocess.run(cmd, env=env, cwd=tmp, preexec_fn=_stack, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=3600)
    if r.returncode != 0:
        raise RuntimeError(f"mpiexec ref_driver failed ({r.returncode}): {r.stdout[-2000:]} {r.stderr[-2000:]}")
    outs = []
    for k, pc in enumerate(parts):
        o = _bundle.read_outputs(f"{fout}.{k}", pc, mode)
        o["stdout"] = r.stdout
        outs.append(o)
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)
    return outs

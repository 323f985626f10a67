"""The Fortran side of the boundary (include/hnumo_engine.f90): it compiles, and its bind(C)
descriptor types have exactly the sizes of the C structs (checked against the ctypes mirror
of include/hnumo_engine.h that test_abi.py pins field by field)."""
import ctypes as C
import os
import shutil
import subprocess
import tempfile

import pytest

from hnumo import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FC = shutil.which("amdflang") or "/opt/rocm/lib/llvm/bin/amdflang"

PROG = """
program sizes
    use iso_c_binding, only: c_sizeof
    use hnumo_engine_c
    type(hnumo_mesh_desc) :: m
    type(hnumo_static_desc) :: s
    type(hnumo_params) :: p
    type(hnumo_halo_desc) :: h
    print '(4I8)', c_sizeof(m), c_sizeof(s), c_sizeof(p), c_sizeof(h)
end program sizes
"""


@pytest.mark.skipif(not os.path.exists(FC) or not os.path.exists(os.path.join(REPO, "h-numo_amd", "libhnumo_engine.so")),
                    reason="no Fortran compiler or engine library")
def test_fortran_interface_struct_sizes():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "sizes.f90")
        open(src, "w").write(PROG)
        subprocess.run([FC, "-c", os.path.join(REPO, "include", "hnumo_engine.f90")], cwd=d, check=True,
                       capture_output=True)
        # linking against the real library also proves every bound symbol resolves
        lib = os.path.join(REPO, "h-numo_amd")
        subprocess.run([FC, src, "hnumo_engine.o", "-o", "sizes", "-L" + lib, "-lhnumo_engine",
                        "-Wl,-rpath," + lib], cwd=d, check=True, capture_output=True)
        out = subprocess.run([os.path.join(d, "sizes")], check=True, capture_output=True, text=True).stdout
    got = [int(x) for x in out.split()]
    want = [C.sizeof(abi.MeshDesc), C.sizeof(abi.StaticDesc), C.sizeof(abi.Params), C.sizeof(abi.HaloDesc)]
    assert got == want


@pytest.mark.skipif(not os.path.exists(FC), reason="no Fortran compiler")
def test_fortran_interface_binds_every_abi_function():
    """Every compute entry point of the C header has a bind(C) interface in the module."""
    src = open(os.path.join(REPO, "include", "hnumo_engine.f90")).read()
    for fn in ("hnumo_engine_create", "hnumo_engine_destroy", "hnumo_abi_version", "hnumo_last_error",
               "hnumo_ti_rk_bcl", "hnumo_ti_barotropic_ssprk", "hnumo_btp_bcl_coeffs", "hnumo_create_rhs_btp",
               "hnumo_get_field", "hnumo_set_resident", "hnumo_sync"):
        assert f"name='{fn}'" in src, fn

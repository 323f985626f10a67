"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/hnumo_engine.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(REPO, "include", "hnumo_engine.h")).read()
    return sorted(set(re.findall(r"\b(hnumo_[a-z_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("hnumo_engine_create", "hnumo_ti_rk_bcl", "hnumo_ti_barotropic_ssprk", "hnumo_create_rhs_btp",
                 "hnumo_get_field", "hnumo_engine_destroy", "hnumo_last_error"):
        assert must in names


def test_library_exports_all_symbols():
    from hnumo import engine
    path = engine.LIB_PATH
    if not os.path.exists(path):
        pytest.skip("libhnumo_engine.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    for name in declared():
        assert hasattr(lib, name), name
    lib.hnumo_abi_version.restype = ctypes.c_int
    assert lib.hnumo_abi_version() == 10


def test_descriptor_struct_matches_header():
    """ctypes mirror field order == header field order (hnumo_mesh_desc etc.)."""
    from hnumo import abi
    src = open(os.path.join(REPO, "include", "hnumo_engine.h")).read()
    for cname, pyst in [("hnumo_mesh_desc", abi.MeshDesc), ("hnumo_static_desc", abi.StaticDesc),
                        ("hnumo_params", abi.Params), ("hnumo_halo_desc", abi.HaloDesc)]:
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            decl = re.sub(r"^(const\s+)?(unsigned\s+)?\w+\s*", "", decl)
            names += [n.strip().lstrip("*").strip() for n in decl.split(",")]
        assert names == [f[0] for f in pyst._fields_], cname

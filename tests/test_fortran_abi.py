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


@pytest.mark.ref
def test_bridge_multirank_branch_compiles_links_and_runs_to_the_device():
    """The Fortran bridge's multi-rank branch (hnumo_bridge.F90: mod_parallel's processor-face
    lists, the RCCL id from rank 0 broadcast with MPI_Bcast) is compiled and linked into
    oracle/_ref/dropin_driver with the reference and libhnumo_engine (oracle/build_ref.sh).
    On this GPU-less host a 2-rank mpiexec run must get through the reference's start-up into
    that branch and stop at its first device call -- rank 0's hnumo_rccl_unique_id -- with the
    bridge's own message (on a GPU box the same run is tests/test_dropin_gpu.py's territory)."""
    import subprocess
    import tempfile
    import oracle as O
    from hnumo import bundle as B
    from hnumo.case import build_case, make_config
    from hnumo.facepart import face_partition
    if not os.path.exists(O.DROPIN_DRIVER):
        pytest.skip("dropin_driver not built")
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present: the run would not stop at the device boundary")
    except ImportError:
        pass
    nm = subprocess.run(["nm", "-u", O.DROPIN_DRIVER], capture_output=True, text=True).stdout
    assert "hnumo_rccl_unique_id" in nm and "hnumo_engine_create" in nm
    case = build_case(make_config("bump10"))
    parts = [face_partition(case, 2, r, "block") for r in range(2)]
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "bundle.bin"), os.path.join(d, "out.bin")
        for r, pc in enumerate(parts):
            B.write_bundle(f"{fin}.{r}", pc, "step", 1, metrics=True)
        r = subprocess.run([O.MPIEXEC, "-launcher", "fork", "-n", "2", O.DROPIN_DRIVER, fin, fout], cwd=d,
                           capture_output=True, text=True, timeout=300)
    assert "hnumo_bridge: hnumo_rccl_unique_id failed" in r.stdout + r.stderr, (r.stdout[-1000:], r.stderr[-1000:])


def _bridge_halo_dump(parts, d):
    """Run oracle/_ref/dropin_driver under mpiexec on `parts` with HNUMO_BRIDGE_HALO_DUMP set: each
    rank's bridge writes the hnumo_halo_desc it built from mod_parallel, then (no GPU here) stops at
    its first device call.  Returns the per-rank dumps."""
    import numpy as np
    import oracle as O
    from hnumo import bundle as B
    fin, fout, dump = os.path.join(d, "bundle.bin"), os.path.join(d, "out.bin"), os.path.join(d, "halo")
    for r, pc in enumerate(parts):
        B.write_bundle(f"{fin}.{r}", pc, "step", 1, metrics=True)
    env = dict(os.environ, HNUMO_BRIDGE_HALO_DUMP=dump)
    p = subprocess.run([O.MPIEXEC, "-launcher", "fork", "-n", str(len(parts)), O.DROPIN_DRIVER, fin, fout], cwd=d,
                       capture_output=True, text=True, timeout=300, env=env)
    out = []
    for r in range(len(parts)):
        assert os.path.exists(f"{dump}.{r}"), ("no halo dump from rank", r, p.stdout[-1000:], p.stderr[-1000:])
        a = np.fromfile(f"{dump}.{r}", dtype="<i4")
        rank, nranks, nn, nown, n = (int(x) for x in a[:5])
        rest = a[5:]
        assert rest.size == 2 * nn + n
        out.append({"rank": rank, "nranks": nranks, "num_nbh": nn, "nelem_owned": nown,
                    "nbh_proc": rest[:nn], "num_send_recv": rest[nn:2 * nn], "nbh_send_recv": rest[2 * nn:]})
    return out


@pytest.mark.ref
@pytest.mark.parametrize("cfg,kw,nranks,order", [("lake10", {}, 4, "morton"),
                                                  ("dg25L3", {"nelx": 8, "nely": 8}, 8, "block")])
def test_bridge_multirank_descriptor_equals_engine_lists(cfg, kw, nranks, order):
    """The Fortran bridge's multi-rank branch (hnumo_bridge.F90) builds hnumo_halo_desc from
    mod_parallel (num_nbh, nbh_proc 1-based, num_send_recv, nbh_send_recv; mod_parallel.F90:106-171
    as p4est.c:1343-1412 fills them).  Run under mpiexec on a Morton lake (4 ranks) and a 4x2-block
    double gyre (8 ranks), every rank's descriptor, read back through its own pointers, equals
    hnumo.facepart.halo_lists and the Python host's HaloDesc -- the lists the engine is tested with
    (tests/test_facehalo_gpu.py) -- field by field, including the 1-based nbh_proc."""
    import numpy as np
    import oracle as O
    from hnumo.abi import Halo
    from hnumo.case import build_case, make_config
    from hnumo.facepart import face_partition, halo_lists
    if not os.path.exists(O.DROPIN_DRIVER):
        pytest.skip("dropin_driver not built")
    case = build_case(make_config(cfg, **kw))
    parts = [face_partition(case, nranks, r, order) for r in range(nranks)]
    with tempfile.TemporaryDirectory() as d:
        dumps = _bridge_halo_dump(parts, d)
    for r, (pc, got) in enumerate(zip(parts, dumps)):
        proc, num, lst, _ = halo_lists(pc)
        assert (got["rank"], got["nranks"], got["nelem_owned"]) == (r, nranks, pc.scalars["nelem"])
        assert got["num_nbh"] == proc.size and got["num_nbh"] > 0
        assert np.array_equal(got["nbh_proc"], proc) and np.array_equal(got["num_send_recv"], num)
        assert np.array_equal(got["nbh_send_recv"], lst)
        assert set(got["nbh_proc"]) <= set(range(1, nranks + 1)) and r + 1 not in set(got["nbh_proc"])
        h = Halo(pc)
        assert (h.desc.rank, h.desc.nranks, h.desc.num_nbh, h.desc.nelem_owned) == \
            (got["rank"], got["nranks"], got["num_nbh"], got["nelem_owned"])
        for k in ("nbh_proc", "num_send_recv", "nbh_send_recv"):
            assert np.array_equal(h.keep[k], got[k]), (r, k)
    # every shared face is listed by both of its ranks, the same number of times
    pairs = {}
    for r, got in enumerate(dumps):
        for p, n in zip(got["nbh_proc"], got["num_send_recv"]):
            pairs[(r, int(p) - 1)] = int(n)
    assert all(pairs[(b, a)] == n for (a, b), n in pairs.items())

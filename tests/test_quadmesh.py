"""Row f3 (meshes beyond the brick): general conforming quadrilateral grids, hnumo/quadmesh.py.

* the geometry -- metric terms at the nodes and quadrature points, normals and face Jacobians
  at the face nodes and face quadrature points -- equals the reference's own metrics,
  metrics_quad, create_normals and create_normals_quad (oracle/_ref/ref_driver mode 7, fixture
  tests/golden/geom_qmbump8.npz) bit for bit, on a grid of general bilinear quadrilaterals
  whose neighbours run along shared edges in both directions;
* the face maps list both sides' face points in one physical order (the engine writes a face
  trace of node n into the neighbour's node-n slot);
* an Abaqus .inp grid (the format p4est reads for lread_external_grid) round-trips.
The reference step on these grids is pinned by tests/golden/qm*_step*.npz (tests/test_oracle.py
on the CPU oracle, tests/test_engine_gpu.py on the engine) and the set-up tables by
setup_qmbump8 (tests/test_setup_tables.py)."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def test_geometry_matches_reference_routines(case_factory):
    from hnumo import bundle as B
    g = dict(np.load(os.path.join(GOLD, "geom_qmbump8.npz"), allow_pickle=False))
    case = case_factory(str(g["config"]))
    d = B.dims(case)
    for k, shp in B.GEOM_OUT:
        mine = np.asarray(case.arrays[k], dtype=np.float64).reshape(B.shape_of(shp, d), order="F")
        assert np.array_equal(mine, g["ref_" + k]), k


def test_face_points_agree_physically(case_factory):
    case = case_factory("qmdg8L3")
    m, A = case.mesh, case.arrays
    P, Q, ngl, nq = m.npts, m.nqq, m.ngl, m.nq
    coord = A["coord"]
    assert m._rev.any() and not m._rev.all()        # both directions occur
    for f in range(m.nface):
        el, er = m.face[6, f] - 1, m.face[7, f]
        if er <= 0:
            continue
        for n in range(ngl):
            il, jl = m.imapl[0, n, f] - 1, m.imapl[1, n, f] - 1
            ir, jr = m.imapr[0, n, f] - 1, m.imapr[1, n, f] - 1
            assert np.allclose(coord[:2, el * P + jl * ngl + il], coord[:2, (er - 1) * P + jr * ngl + ir], atol=1e-6)
        # quad points: mirrored through the face centre when the sides run opposite ways
        il = m.imapl_q[0, :, f] - 1 + (m.imapl_q[1, :, f] - 1) * nq
        ir = m.imapr_q[0, :, f] - 1 + (m.imapr_q[1, :, f] - 1) * nq
        assert len(set(il.tolist())) == nq and len(set(ir.tolist())) == nq
    # outward unit normals of the left element
    nv = m.normal_vector
    assert np.allclose(nv[0] ** 2 + nv[1] ** 2, 1.0)
    for f in range(m.nface):
        el = m.face[6, f] - 1
        cen = coord[:2, el * P:(el + 1) * P].mean(axis=1)
        n = ngl // 2
        p = coord[:2, el * P + (m.imapl[1, n, f] - 1) * ngl + m.imapl[0, n, f] - 1]
        assert nv[0, n, f] * (p[0] - cen[0]) + nv[1, n, f] * (p[1] - cen[1]) > 0


def test_flat_grid_reproduces_brick_metrics(case_factory):
    flat = case_factory("qmbump8", mesh=("warp", 0.0, False))
    brick = case_factory("qmbump8", mesh=None)
    for k in ("ksi_x", "eta_y", "jac", "ksiq_x", "etaq_y", "jacq"):
        assert np.allclose(flat.arrays[k], brick.arrays[k], rtol=1e-13, atol=1e-15), k
    assert np.isclose(flat.arrays["jac"].sum(), 2000.0 * 2000.0, rtol=1e-14)


def test_inp_round_trip(tmp_path, case_factory):
    from hnumo.quadmesh import read_inp, warped_brick, write_inp
    V, Qd, bc = warped_brick(6, 5, (0.0, 2000.0), (0.0, 1500.0), 0.2, True, 4)
    bc[next(iter(bc))] = 2                      # one no-slip wall edge
    path = str(tmp_path / "EXTERNAL_MESH.inp")
    write_inp(path, V, Qd, bc)
    V2, Q2, bc2 = read_inp(path)
    assert np.array_equal(V2, V) and np.array_equal(Q2, Qd) and bc2 == bc
    a = case_factory("qmbump8", mesh=("inp", path), nelx=6, nely=5, ydims=(0.0, 1500.0))
    b = case_factory("qmbump8", mesh=("warp", 0.2, True), nelx=6, nely=5, ydims=(0.0, 1500.0))
    for k in ("face", "imapl", "imapr", "ksiq_x", "jac_faceq"):
        if k == "face":
            # (the one no-slip edge)
            assert sorted((-b.arrays[k][7])[b.arrays[k][7] < 0].tolist()) != sorted((-a.arrays[k][7])[a.arrays[k][7] < 0].tolist())
            continue
        assert np.array_equal(a.arrays[k], b.arrays[k]), k


def test_clockwise_element_is_rejected():
    from hnumo.quadmesh import QuadMesh
    V = np.array([[0.0, 0.0], [1.0, 0.0], [1.0, 1.0], [0.0, 1.0]])
    with pytest.raises(ValueError):
        QuadMesh(V, np.array([[0, 3, 2, 1]]), {}, 5, 9)


def test_inconsistent_boundary_tags_are_rejected():
    """A :BC_ line element must lie on a boundary edge (p4est_bc_read_inp attaches it to the one
    element side there): one on an interior edge, or on an edge no element has, is an error."""
    from hnumo.quadmesh import QuadMesh
    V = np.array([[0.0, 0.0], [1.0, 0.0], [2.0, 0.0], [0.0, 1.0], [1.0, 1.0], [2.0, 1.0]])
    Qd = np.array([[0, 1, 4, 3], [1, 2, 5, 4]])
    QuadMesh(V, Qd, {frozenset((0, 1)): 2}, 5, 9)                  # a boundary edge: fine
    with pytest.raises(ValueError, match="interior"):
        QuadMesh(V, Qd, {frozenset((1, 4)): 2}, 5, 9)              # the shared edge
    with pytest.raises(ValueError, match="no element"):
        QuadMesh(V, Qd, {frozenset((0, 5)): 2}, 5, 9)              # not an edge

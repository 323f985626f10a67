"""The reference's own partition contract -- processor faces (hnumo/facepart.py) -- on CPU.

* every element is owned by exactly one rank; every local element has its 4 faces; a shared
  face appears on both ranks with the local element on the left, face(8) = 0, face(6) = 0
  (p4est.c:1686-1692), listed once in nbh_send_recv;
* across ranks (torch.distributed, gloo, world size 2 and 4): rank a's list of faces shared
  with b and rank b's list shared with a name the same global faces in the same order, their
  face nodes are the same physical points node by node (the receiver puts node n of the
  message into node n of side 2, create_rhs_dynamics_flux.F90:165-171) and the two copies'
  normals are opposite;
* the multi-rank golden fixtures (the reference under mpiexec, tests/golden/make_golden.py
  mpi) were made from the setup code as it is now (bundle hashes), and, where the reference
  harness exists, the reference reproduces them (-m ref)."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from hnumo.case import build_case, make_config
from hnumo.facepart import face_partition, halo_lists

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MPI_FIXTURES = ["bump10_mpi3m_step2", "lake10_mpi2b_step1", "dg8L3_mpi2b_step2", "dg8L3_mpi4m_step2",
                "lake10_mpi4m_step2", "bump10q_mpi2b_step1", "dg8L3q_mpi4m_step2"]


@pytest.mark.parametrize("nranks,order", [(2, "block"), (4, "block"), (3, "morton"), (5, "morton")])
def test_face_partition_covers_mesh(nranks, order):
    case = build_case(make_config("bump16"), dense=False)
    seen = np.zeros(case.scalars["nelem"], int)
    P = case.scalars["ngl"] ** 2
    for r in range(nranks):
        pc = face_partition(case, nranks, r, order)
        seen[pc.elems] += 1
        f = pc.arrays["face"]
        cnt = np.zeros(pc.scalars["nelem"], int)
        for k in (6, 7):
            v = f[k]
            np.add.at(cnt, v[v > 0] - 1, 1)
        assert (cnt == 4).all()
        proc = np.flatnonzero(f[7] == 0)
        assert (f[5, proc] == 0).all() and (f[6, proc] > 0).all()
        _, num, lst, multi = halo_lists(pc)
        assert sorted((lst - 1).tolist()) == proc.tolist() and (multi == 1).all()
        gn = (pc.elems[:, None] * P + np.arange(P)[None, :]).ravel()
        for k in ("qb_df", "q_df", "qprime_df"):
            assert np.array_equal(pc.arrays[k], np.asarray(case.arrays[k])[:, gn, ...])
    assert (seen == 1).all()


def _face_points(case, pc, faces):
    """Physical (x, y) of the face nodes of local faces, in the order of imapl."""
    from hnumo.basis import Basis
    b = Basis(case.scalars["ngl"] - 1)
    P, ngl = b.ngl ** 2, b.ngl
    coord = case.mesh.node_coords(b.xgl)
    out = []
    for f in faces:
        e = pc.arrays["face"][6, f] - 1
        ge = pc.elems[e]
        i, j = pc.arrays["imapl"][0, :, f] - 1, pc.arrays["imapl"][1, :, f] - 1
        I = ge * P + j * ngl + i
        out.append(np.stack([coord[0, I], coord[1, I]], 1).tolist())
    return out


def _worker(rank, world, port, order, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = build_case(make_config("bump16"), dense=False)
        pc = face_partition(case, world, rank, order)
        mine = {}
        for n in pc.fneighbours:
            nv = pc.arrays["normal_vector"][:2, :, n.faces].T.tolist()
            mine[n.rank] = (pc.faces[n.faces].tolist(), _face_points(case, pc, n.faces), nv)
        allv = [None] * world
        dist.all_gather_object(allv, mine)
        ok = True
        for n in pc.fneighbours:
            gf, pts, nv = mine[n.rank]
            pgf, ppts, pnv = allv[n.rank][rank]
            ok &= pgf == gf                    # same faces, same order (nbh_send_recv)
            ok &= ppts == pts                  # node n of the message is node n of my face
            ok &= bool(np.array_equal(np.asarray(pnv), -np.asarray(nv)))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,order", [(2, "block"), (4, "morton")])
def test_processor_face_lists_agree_across_ranks_gloo(world, order):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + world * 11 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, order, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


def _mpi_parts(g):
    from util import overrides_of
    case = build_case(make_config(str(g["config"]), **overrides_of(g)))
    R = int(g["nranks"])
    return case, [face_partition(case, R, r, str(g["order"])) for r in range(R)]


# the BASELINE configs at their stated sizes (C5 lake 200x200 on 4 ranks, C4 316x316 on 8): the
# reference bundles (dense tables included) are GBs, so the fixtures carry a hash of every rank's
# non-dense inputs and halo lists instead (tests/util.py partition_inputs_sha256)
MPI_FIXTURES_FULLSIZE = ["lake200_mpi4m_step1", "dg316L3_mpi8b_step1"]


@pytest.mark.parametrize("name", MPI_FIXTURES_FULLSIZE)
def test_fullsize_mpi_fixture_inputs_current(name):
    from util import overrides_of, partition_inputs_sha256
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    case = build_case(make_config(str(g["config"]), **overrides_of(g)), dense=False)
    R = int(g["nranks"])
    for r in range(R):
        pc = face_partition(case, R, r, str(g["order"]))
        assert pc.scalars["nelem"] == int(g[f"nelem_r{r}"])
        assert partition_inputs_sha256(pc) == str(g[f"inputs_sha256_r{r}"]), (name, r)


@pytest.mark.parametrize("name", MPI_FIXTURES)
def test_mpi_fixture_inputs_current(name):
    import tempfile, hashlib
    from hnumo import bundle as B
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    _, parts = _mpi_parts(g)
    for r, pc in enumerate(parts):
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "b.bin")
            B.write_bundle(p, pc, "step", int(g["nsteps"]))
            h = hashlib.sha256(open(p, "rb").read()).hexdigest()
        assert h == str(g[f"bundle_sha256_r{r}"]), (name, r)


@pytest.mark.ref
@pytest.mark.parametrize("name", MPI_FIXTURES[:2])
def test_reference_mpi_reproduces_fixture(name):
    import oracle as O
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    _, parts = _mpi_parts(g)
    outs = O.run_reference_mpi(parts, "step", int(g["nsteps"]))
    for r, o in enumerate(outs):
        for k in ("q_df", "qb_df", "qprime_df"):
            assert np.array_equal(o[k], g[f"{k}_r{r}"]), (r, k)

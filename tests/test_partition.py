"""Partition / halo contract of the multi-rank path, on CPU.

* every element is owned by exactly one rank; each local element has its 4 faces;
* a ghost carries exactly its owner's data (statics and state), so refreshing it from the
  owner makes it indistinguishable from the owner's element;
* across ranks (torch.distributed, gloo, world size 2 and 4): rank a's send list to b and
  rank b's receive list from a name the same global elements in the same order.
"""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from hnumo.case import build_case, make_config
from hnumo.partition import element_owner, partition, rank_grid


def _check_local(case, pc):
    P = case.scalars["ngl"] ** 2
    f = pc.arrays["face"]
    cnt = np.zeros(pc.scalars["nelem"], int)
    for k in (6, 7):
        v = f[k]
        np.add.at(cnt, v[v > 0] - 1, 1)
    assert (cnt == 4).all()
    assert (f[7] != 0).all()                     # no processor faces in the ghost-layer scheme
    gn = (pc.elems[:, None] * P + np.arange(P)[None, :]).ravel()
    for k in ("qb_df", "q_df", "qprime_df"):
        assert np.array_equal(pc.arrays[k], np.asarray(case.arrays[k])[:, gn, ...])
    for k in ("massinv", "pbprime_df", "one_over_pbprime_df"):
        assert np.array_equal(pc.arrays[k], np.asarray(case.arrays[k])[gn])


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_partition_covers_mesh(nranks):
    case = build_case(make_config("bump16"), dense=False)
    px, py = rank_grid(nranks)
    owner = element_owner(case.mesh.nelx, case.mesh.nely, px, py)
    seen = np.zeros(case.scalars["nelem"], int)
    for r in range(nranks):
        pc = partition(case, nranks, r)
        assert (owner[pc.elems[:pc.nelem_owned]] == r).all()
        assert (owner[pc.elems[pc.nelem_owned:]] != r).all()
        seen[pc.elems[:pc.nelem_owned]] += 1
        _check_local(case, pc)
    assert (seen == 1).all()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = build_case(make_config("bump16"), dense=False)
        pc = partition(case, world, rank)
        mine = {n.rank: (pc.elems[n.send].tolist(), pc.elems[n.recv].tolist()) for n in pc.neighbours}
        allv = [None] * world
        dist.all_gather_object(allv, mine)
        ok = True
        for n in pc.neighbours:
            peer_send, peer_recv = allv[n.rank][rank]
            ok &= peer_send == pc.elems[n.recv].tolist()   # what they send is what I hold as ghosts
            ok &= peer_recv == pc.elems[n.send].tolist()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_halo_lists_agree_across_ranks_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world * 7 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res

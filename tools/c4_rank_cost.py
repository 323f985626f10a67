"""Per-GPU cost of the 8-GPU C4 configuration, measured on ONE GPU (VERDICT r03 "next" 5).

One rank of the 8-GPU run holds a 79x158 block (12,482 elements) of the 316x316 double gyre
(face_partition, 4x2 blocks, the reference's processor-face contract) and, per barotropic stage,
runs its boundary elements on a second stream, ships their traces over RCCL and runs its
interior elements beside it (csrc/engine.hip launch_subcycle).  RCCL refuses two ranks on one
device, so the rank is run here as a self-neighbour engine (tests/test_rccl_self_gpu.py): a
one-rank communicator whose per-neighbour processor-face lists are addressed to itself -- the same
streams, events, element split, launches and RCCL group calls (one send/recv pair per neighbour)
per stage as the real rank, with each message going to itself instead of over xGMI.  Compared with:
  block     the same 79x158 elements as a single-rank engine (walls instead of processor faces,
            one stream, graph-captured step): the per-GPU work without any halo machinery;
  local     the self-neighbour partition through the local exchange group (device copies);
  rccl      the self-neighbour RCCL engine, direct launches (the default of RCCL engines);
  rccl_g    the same with the step captured into a hipGraph (HNUMO_GRAPH=1).
Prints one JSON line per variant (ms per step, stage kernel time, state hash: rccl == local
bitwise) and a projection of the C4/8 step time.

    python tools/c4_rank_cost.py [--steps 3] [--rank 1]
"""
import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))


def state_hash(e, st=None):
    q, qb, qp = st if st is not None else e.state()
    if st is None:
        e.sync(q, qb, qp)
    return hashlib.sha256(q.tobytes() + qb.tobytes() + qp.tobytes()).hexdigest()[:16]


def timed(e, steps, group=False):
    from hnumo.engine import group_ti_rk_bcl
    # (no torch here: the engine calls synchronise their streams before returning)
    if group:
        e.set_resident(True)
        st = [e.state()]
        for _ in range(2):              # warm-up (uploads), as many steps as the resident variants
            group_ti_rk_bcl([e], st)
        t0 = time.perf_counter()
        for _ in range(steps):
            group_ti_rk_bcl([e], st)
        t = (time.perf_counter() - t0) / steps
        return t, None
    e.set_resident(True)
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)              # uploads, captures (or not) the step
    e.bench_steps(1)
    t0 = time.perf_counter()
    _, k_ms, _ = e.bench_steps(steps)
    return (time.perf_counter() - t0) / steps, k_ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rank", type=int, default=1, help="rank of the 4x2 partition (1: three neighbours)")
    ap.add_argument("--variants", default="block,local,rccl,rccl_g")
    ap.add_argument("--no-projection", action="store_true")
    ap.add_argument("--one-list", action="store_true")
    args = ap.parse_args()
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine, local_group
    from hnumo.facepart import face_partition
    g = build_case(make_config("dg316L3"), dense=False)
    pc = face_partition(g, 8, args.rank, "block")
    nbrs = [(n.rank, int(n.faces.size)) for n in pc.fneighbours]
    # the self-neighbour contract: the rank's per-neighbour processor-face lists, each addressed to
    # the rank itself (facepart.self_neighbour; --one-list: all faces as one list, rounds 3-5)
    from hnumo.facepart import self_neighbour
    pc = self_neighbour(pc, per_peer=not args.one_list)
    E = pc.scalars["nelem"]
    S = g.scalars
    stages = 2 * S["N_btp"] * S["kstages"]
    res = {}
    for v in args.variants.split(","):
        if v == "block":
            c = make_config("dg316L3", nelx=79, nely=158, xdims=(0.0, 2.0e6 / 4), ydims=(0.0, 2.0e6 / 2))
            e = Engine(build_case(c, dense=False))
            t, k = timed(e, args.steps)
        elif v == "local":
            e = Engine(pc)
            local_group([e])
            t, k = timed(e, args.steps, group=True)
        else:
            os.environ["HNUMO_GRAPH"] = "1" if v == "rccl_g" else "0"
            e = Engine(pc, comm_id=Engine.rccl_unique_id())
            os.environ.pop("HNUMO_GRAPH")
            t, k = timed(e, args.steps)
        h = state_hash(e) if v != "block" else None
        e.close()
        res[v] = {"variant": v, "elements": E, "ms_per_step": round(t * 1e3, 3),
                  "us_per_stage": round(t * 1e6 / stages, 2),
                  "stage_kernel_us": round(k * 1e3, 2) if k and k > 0 else None, "state": h}
        print(json.dumps(res[v]), flush=True)
    if "block" in res:
        for v in ("rccl", "rccl_g", "local"):
            if v in res:
                d = res[v]["ms_per_step"] - res["block"]["ms_per_step"]
                res[v]["overhead_ms_per_step"] = round(d, 3)
                res[v]["overhead_us_per_stage"] = round(d * 1e3 / stages, 2)
    best = min((res[v]["ms_per_step"], v) for v in ("rccl", "rccl_g") if v in res) if ("rccl" in res or "rccl_g" in res) else None
    out = {"config": "dg316L3 rank %d of 4x2 blocks (%d elements, neighbours %s)" % (args.rank, E, nbrs),
           "stages_per_step": stages, "variants": res}
    if best:
        t = best[0] * 1e-3
        out["projection_c4_8gpu"] = {
            "mode": best[1], "ms_per_step": best[0],
            "EU_per_s": round(S["nelem"] * stages / t, 1),
            "note": "each of the 8 GPUs runs its block as measured here; xGMI transfer time of the real "
                    "messages (<= 3 x 50 KB per stage) not included"}
        if "rccl" in res and "rccl_g" in res:
            out["bitwise_rccl_vs_local"] = res["rccl"]["state"] == res.get("local", {}).get("state") == res["rccl_g"]["state"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()

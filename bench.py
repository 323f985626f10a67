"""Benchmark of the MI355X MLSWE time-step engine (h-NUMO ti_rk_bcl hot path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config dg25L3]

One "step" is one baroclinic time step ti_rk_bcl (ti_rk_bcl.F90:9-87): two barotropic
SSP(5,3) sub-cycles of N_btp*kstages stages each plus the layer predictor-corrector,
on device-resident state (hipGraph replay).  Metric (BASELINE.json): DG element-updates
per second, one element-update = one element advanced by one barotropic stage with all
layers, EU/s = E * 2*N_btp*kstages / T_step.  Inputs are the analytic double-gyre initial
condition (data: synthetic IC, no files).

Multi-GPU (torch.distributed.run, one rank per GPU; weak scaling): the double gyre is
enlarged to px*py blocks of 25x25 elements (same element size, rank grid 2x1, 2x2, 4x2)
and each rank owns one block plus a one-element ghost layer (hnumo/partition.py); the
engine refreshes ghost data from the owners over RCCL point-to-point (xGMI) at every
exchange point of the step (csrc/engine.hip `exchange`).  value = element-updates of all
ranks / max time over ranks.  If the RCCL halo cannot be set up on every rank, the ranks
fall back to independent replicas and say so in config.parallelism.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "h-numo_amd"))


def cpu_baseline(case, steps: int):
    """Time the reference Fortran itself (oracle/_ref/ref_driver, built from the
    reference sources in the build container) on this host, 1 rank/1 core; fall back to
    the C restatement (oracle) if the binary cannot run here."""
    from hnumo import bundle as B
    from hnumo.roofline import element_updates_per_step
    eus = element_updates_per_step(case) * steps
    ref = os.path.join(REPO, "oracle", "_ref", "ref_driver")
    sample = f"{case.cfg['name']} ({case.scalars['nelem']} elements, N={case.scalars['ngl'] - 1}, " \
             f"L={case.scalars['nlayers']}), {steps} baroclinic steps"
    if os.path.exists(ref):
        try:
            with tempfile.TemporaryDirectory() as d:
                fin, fout = os.path.join(d, "b.bin"), os.path.join(d, "o.bin")
                B.write_bundle(fin, case, "step", steps)

                def _stack():
                    import resource
                    resource.setrlimit(resource.RLIMIT_STACK, (resource.RLIM_INFINITY, resource.RLIM_INFINITY))

                env = dict(os.environ, OMP_NUM_THREADS="1")
                r = subprocess.run(["taskset", "-c", "0", ref, fin, fout], cwd=d, env=env, preexec_fn=_stack,
                                   capture_output=True, text=True, timeout=600)
                if r.returncode == 0:
                    t = [float(line.split()[1]) for line in r.stdout.splitlines() if line.startswith("REF_TIME")][0]
                    return {"value": eus / t, "unit": "element-updates/s", "cores": 1, "kind": "reference",
                            "sample": sample + f" of the reference Fortran (amdflang -O2), {t:.2f} s"}
        except Exception as exc:  # pragma: no cover - diagnostic only
            print(f"[bench] reference baseline failed: {exc}", file=sys.stderr)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    o = O.Oracle(case)
    q, qb, qp = o.state()
    t0 = time.perf_counter()
    for _ in range(steps):
        o.ti_rk_bcl(q, qb, qp)
    t = time.perf_counter() - t0
    return {"value": eus / t, "unit": "element-updates/s", "cores": 1, "kind": "port",
            "sample": sample + f" of the C restatement (oracle/hnumo_oracle.c, -O2), {t:.2f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="dg25L3")
    ap.add_argument("--cpu-steps", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--summation", default="reference", choices=["reference", "factored"],
                    help="stage summation order (hnumo_set_summation); only 'reference' meets the 1e-10 bar")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine
    from hnumo.roofline import HBM_PEAK_GBS, element_updates_per_step, stage_bytes

    base_cfg = make_config(args.config)
    case = build_case(base_cfg, dense=False)         # the per-GPU block (roofline, workload name)
    eng, parallelism = None, "single"
    if world > 1:
        from hnumo.partition import partition, rank_grid
        px, py = rank_grid(world)
        x0, x1 = base_cfg["xdims"]
        y0, y1 = base_cfg["ydims"]
        gcfg = make_config(args.config, nelx=base_cfg["nelx"] * px, nely=base_cfg["nely"] * py,
                           xdims=(x0, x0 + (x1 - x0) * px), ydims=(y0, y0 + (y1 - y0) * py))
        gcase = build_case(gcfg, dense=False)
        obj = [Engine.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        err = None
        try:
            eng = Engine(partition(gcase, world, rank), device=local_rank, comm_id=obj[0], summation=args.summation)
        except Exception as exc:  # pragma: no cover - depends on the node
            err = f"{type(exc).__name__}: {exc}"
        bad = torch.tensor([1 if err else 0], device="cuda")
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if bad.item():
            if eng is not None:
                eng.close()
            eng = None
            parallelism = f"replicas{world} (RCCL halo unavailable: {err or 'on another rank'})"
        else:
            parallelism = f"domain decomposition {px}x{py} x ({base_cfg['nelx']}x{base_cfg['nely']}), ghost halo over RCCL"
    if eng is None:
        eng = Engine(case, device=local_rank, summation=args.summation)
    eng.set_resident(True)
    q, qb, qp = eng.state()
    eng.ti_rk_bcl(q, qb, qp)                       # uploads the state, builds the graph
    if args.warmup > 1:
        eng.bench_steps(args.warmup - 1)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    _, k_ms, _ = eng.bench_steps(args.steps)         # synchronises the engine stream
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    path = eng.stage_path
    kname = "btp_subcycle_kernel" if path == "persistent" else "btp_stage_kernel"
    k_src = "graph event nodes around the corrector sub-cycle"
    if not (k_ms and k_ms > 0):
        k_ms = eng.time_stage_kernel(2)
        k_src = "events around 2 direct corrector sub-cycles" + (" (incl. halo exchanges)" if world > 1 else "")
    if path == "persistent":
        k_src += "; one launch per sub-cycle, time per stage = launch time / (N_btp*kstages)"
    eng.sync(q, qb, qp)
    if not (abs(qb).max() < 1e30):
        raise RuntimeError("non-finite state after benchmark")

    eu = element_updates_per_step(case) * args.steps * world   # every rank owns one block of E elements
    value = eu / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    sb = stage_bytes(case)
    roof = None
    if k_ms and k_ms > 0:
        achieved = sb / (k_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": kname, "kernel_avg_us": round(k_ms * 1e3, 3),
                "algorithmic_bytes_per_launch": int(sb), "timing": k_src}
        pmc = os.path.join(REPO, "profiles", "pmc_btp_stage.json")
        if os.path.exists(pmc):
            try:
                d = json.load(open(pmc))
                if d.get("config") == args.config and d.get("kernel", "btp_stage_kernel") == kname:
                    roof["traffic"] = d["hbm_bytes_per_launch"]
            except Exception:
                pass
    out = {
        "metric": "DG element-updates/sec (all layers, per RK stage)",
        "value": round(value, 1), "unit": "element-updates/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic (analytic double-gyre IC)",
        "config": {"workload": f"{args.config}: double-gyre {base_cfg['nelx']}x{base_cfg['nely']} elements per GPU, "
                               f"N={case.scalars['ngl'] - 1}, {case.scalars['nlayers']} layers, "
                               f"N_btp={case.scalars['N_btp']}, kstages={case.scalars['kstages']}",
                   "elements": case.scalars["nelem"], "nlayers": case.scalars["nlayers"],
                   "nop": case.scalars["ngl"] - 1, "parallelism": parallelism,
                   "summation": args.summation, "stage_path": path},
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(build_case(make_config(args.config)), args.cpu_steps)
    if rank == 0:
        print(json.dumps(out))
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

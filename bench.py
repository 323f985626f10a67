"""Benchmark of the MI355X MLSWE time-step engine (h-NUMO ti_rk_bcl hot path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config dg25L3]

One "step" is one baroclinic time step ti_rk_bcl (ti_rk_bcl.F90:9-87): two barotropic
SSP(5,3) sub-cycles of N_btp*kstages stages each plus the layer predictor-corrector,
on device-resident state (hipGraph replay).  Metric (BASELINE.json): DG element-updates
per second, one element-update = one element advanced by one barotropic stage with all
layers, EU/s = E * 2*N_btp*kstages / T_step.  Inputs are the analytic double-gyre initial
condition (data: synthetic IC, no files).

Workloads (BASELINE.json configs):
  N=1   dg25L3  -- configs[1], the double gyre at 25x25 elements, N=4, 3 layers (the metric's
                   1-GPU configuration); the line also carries "c4_single_gpu", the C4 mesh
                   below on this one GPU (the strong-scaling base of the N>1 lines), and
                   "c3_single_gpu", configs[2] (dg25N7L3: N=7, 3 layers, 25x25 elements), and
                   "c5_single_gpu", configs[4]'s mesh (lake200: the lake at rest, 2 layers) on this GPU.
  N>1   dg316L3 -- configs[3] (C4), the double gyre at 316x316 = 99,856 elements, N=4,
                   3 layers, dt=40 s, dt_btp=2 s, split over the N GPUs (strong scaling:
                   rank grid 2x1, 2x2, 4x2 of 158x316 / 158x158 / 79x158 element blocks).
  --weak        -- labelled extra: N blocks of 25x25 elements (weak scaling).
  --config lake200 at N>1 -- configs[4] (C5), the lake at rest on 200x200 elements, 2 layers, on
                   a Morton processor-face partition (the C5 reference fixture's).
  --emulate W:R -- the N>1 code path on ONE GPU (torch.distributed.run --nproc-per-node 1): rank R
                   of the W-rank partition as its own neighbour (the self-neighbour contract,
                   hnumo/facepart.py self_neighbour: its per-neighbour processor-face lists kept,
                   each addressed to itself -- one RCCL send/recv pair per real neighbour at the
                   real offsets and sizes -- and the processor faces' side-2 statics mirrored
                   from side 1 so the mirror is well balanced), with the real run's nccl process
                   group, id broadcast, RCCL engine, two-stream schedule, timed loop, halo check
                   and strong-scaling base -- the per-GPU cost of a W-GPU run and the setup time
                   of every phase, measured where no W-GPU node is available.
Multi-GPU runs one rank per GPU (torch.distributed.run).  Each rank holds one block of the
brick partitioned the way h-NUMO itself partitions -- processor faces (hnumo/facepart.py,
p4est.c:1686-1712): the reference's halo contract, with the stage traces exchanged over RCCL
point-to-point (xGMI) on a second stream while the interior elements run (csrc/engine.hip
`trace_exchange`, the overlap of mod_rhs_btp.F90:40-46).  --halo ghost uses the one-element
ghost layer of hnumo/partition.py instead.  value = element-updates of all ranks / max time
over ranks.  If the RCCL halo cannot be set up (or fails) on any rank, the run fails (exit
status 1, an {"error": ...} line on stderr): it never substitutes another kind of number.
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


def _run_reference(parts_or_case, steps: int, nranks: int):
    """Time the reference Fortran (oracle/_ref/ref_driver, built from the reference sources in
    the build container): one process on core 0, or `mpiexec -n nranks` on a processor-face
    partition (the reference's own MPI halo exchange), one rank per core.  Returns seconds
    (max over ranks of the reference's own MPI_Wtime around the step loop) or None."""
    from hnumo import bundle as B
    ref = os.path.join(REPO, "oracle", "_ref", "ref_driver")
    if not os.path.exists(ref):
        return None

    def _stack():
        import resource
        resource.setrlimit(resource.RLIMIT_STACK, (resource.RLIM_INFINITY, resource.RLIM_INFINITY))

    env = dict(os.environ, OMP_NUM_THREADS="1")
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "b.bin"), os.path.join(d, "o.bin")
        if nranks == 1:
            B.write_bundle(fin, parts_or_case, "step", steps)
            cmd = ["taskset", "-c", "0", ref, fin, fout]
        else:
            for r, pc in enumerate(parts_or_case):
                B.write_bundle(f"{fin}.{r}", pc, "step", steps)
            cmd = [os.environ.get("HNUMO_MPIEXEC", "/opt/conda/bin/mpiexec"), "-launcher", "fork", "-bind-to", "core",
                   "-n", str(nranks), ref, fin, fout]
        r = subprocess.run(cmd, cwd=d, env=env, preexec_fn=_stack, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            print(f"[bench] reference run failed ({r.returncode}): {r.stderr[-500:]}", file=sys.stderr)
            return None
        t = [float(line.split()[1]) for line in r.stdout.splitlines() if line.startswith("REF_TIME")]
        return max(t) if t else None


def cpu_baseline(case, steps: int, cores: int, repeats: int = 3):
    """The reference Fortran timed on this host: `cores` MPI ranks (one per core) on a Morton
    processor-face partition of the same workload -- the reference's own multi-rank path --
    `repeats` times (value = the median; the host cores are shared, so min / max are reported
    beside it), and one rank on one core.  Falls back to the C restatement (oracle, 1 core)."""
    from hnumo.facepart import face_partition
    from hnumo.roofline import element_updates_per_step
    eu = element_updates_per_step(case)
    S = case.scalars
    sample = f"{case.cfg['name']} ({S['nelem']} elements, N={S['ngl'] - 1}, L={S['nlayers']})"
    out = None
    try:
        one = _run_reference(case, steps, 1)
        many_steps = steps * max(1, cores // 2)
        many = None
        if cores > 1:
            parts = [face_partition(case, cores, r, "morton") for r in range(cores)]
            runs = [t for t in (_run_reference(parts, many_steps, cores) for _ in range(repeats)) if t]
            if runs:
                many = sorted(runs)[len(runs) // 2]
        if many:
            rates = sorted(eu * many_steps / t for t in runs)
            out = {"value": eu * many_steps / many, "unit": "element-updates/s", "cores": cores, "kind": "reference",
                   "sample": sample + f", {many_steps} baroclinic steps of the reference Fortran (amdflang -O2) under "
                                      f"mpiexec -n {cores} (Morton processor-face partition, its own MPI halo), "
                                      f"one rank per core: {many:.2f} s (median of {len(runs)} runs)",
                   "spread": {"runs": len(runs), "min": round(rates[0], 1), "max": round(rates[-1], 1)}}
        if one:
            single = {"value": eu * steps / one, "cores": 1,
                      "sample": sample + f", {steps} baroclinic steps, 1 rank on core 0: {one:.2f} s"}
            if out:
                out["single_core"] = single
            else:
                out = dict(single, unit="element-updates/s", kind="reference")
    except Exception as exc:  # pragma: no cover - diagnostic only
        print(f"[bench] reference baseline failed: {exc}", file=sys.stderr)
    if out:
        return out
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    o = O.Oracle(case)
    q, qb, qp = o.state()
    t0 = time.perf_counter()
    for _ in range(steps):
        o.ti_rk_bcl(q, qb, qp)
    t = time.perf_counter() - t0
    return {"value": eu * steps / t, "unit": "element-updates/s", "cores": 1, "kind": "port",
            "sample": sample + f", {steps} baroclinic steps of the C restatement (oracle/hnumo_oracle.c, -O2), {t:.2f} s"}


def single_gpu_line(cfg: str, workload: str, steps: int = 3, case=None, device: int = 0, breakdown: bool = True):
    """Another BASELINE config on this one GPU, reported beside the N=1 configs[1] line: the C4
    mesh (dg316L3, 99,856 elements; the base of the N>1 strong-scaling lines) and C3 (dg25N7L3,
    N=7).  Also the strong-scaling base of an N>1 run (rank 0's GPU, the whole mesh)."""
    import torch
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine
    from hnumo.roofline import element_updates_per_step
    if case is None:
        case = build_case(make_config(cfg), dense=False)
    eng = Engine(case, device=device)
    eng.set_resident(True)
    q, qb, qp = eng.state()
    eng.ti_rk_bcl(q, qb, qp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.bench_steps(steps)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    k_ms = eng.time_stage_kernel(1)
    path = eng.stage_path
    stats = eng.persistent_stats
    env = eng.overrides
    bd = step_breakdown(eng, case, 1) if breakdown else None
    from hnumo.roofline import HBM_PEAK_GBS, stage_bytes
    eng.close()
    ach = stage_bytes(case) / (k_ms * 1e-3) / 1e9
    out = {"workload": f"{workload} on 1 GPU, {path} stage path",
           "value": round(element_updates_per_step(case) * steps / t, 1), "unit": "element-updates/s",
           "steps": steps, "ms_per_step": round(1e3 * t / steps, 3),
           "stage_kernel_us": round(k_ms * 1e3, 2), "stage_kernel_frac": round(ach / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_stage": int(stage_bytes(case)), "persistent_fallbacks": stats["aborts"],
           "engine_env": env}
    out.update(_profiled(cfg, "btp_subcycle_kernel" if path == "persistent" else "btp_stage_kernel", k_ms))
    if bd:
        out.update(bd)
    return out


def step_breakdown(eng, case, nsteps: int = 2) -> dict:
    """Per-kernel microseconds of one step (hnumo_step_breakdown: direct launches with an event
    after each on the engine stream; the state advances) and the sub-cycle-only rate: element-
    updates of the two barotropic sub-cycles over their own time."""
    from hnumo.roofline import element_updates_per_step
    try:
        bd = eng.step_breakdown(nsteps)
    except Exception as exc:  # pragma: no cover - diagnostic only
        return {"step_breakdown_error": f"{type(exc).__name__}: {exc}"}
    sub = sum(v for k, v in bd.items() if k in ("btp_subcycle", "btp_stage", "subcycle_prologue", "grad_trace",
                                                "btp_finalize"))
    tot = sum(bd.values())
    return {"step_breakdown_us": {k: round(v, 2) for k, v in bd.items()},
            "step_breakdown_total_us": round(tot, 2),
            "step_breakdown_note": f"direct launches, an event after each ({nsteps} steps averaged); spans "
                                   "between events, so they include the launch gaps the captured graph avoids",
            "subcycle_us_per_step": round(sub, 2),
            "subcycle_eu_per_s": round(element_updates_per_step(case) / (sub * 1e-6), 1) if sub > 0 else None,
            "glue_us_per_step": round(tot - sub, 2)}


def stream_copy(device: int = 0) -> dict | None:
    """The measured HBM denominator (achieved bandwidth against the nominal peak
    AND a stream copy on the same GPU): hnumo_stream_copy_bw over 2 x 2 GiB buffers."""
    from hnumo.engine import Engine
    try:
        gbs, var = Engine.stream_copy_bw(device, 2 << 30, 10)
    except Exception as exc:  # pragma: no cover - diagnostic only
        print(f"[bench] stream copy failed: {exc}", file=sys.stderr)
        return None
    kind = {0: "grid-stride, default policy", 1: "grid-stride, non-temporal", 2: "one-pass, non-temporal"}[int(var)]
    return {"gbs": round(gbs, 1),
            "how": f"hnumo_stream_copy_bw: 16-byte copy kernels 2 GiB -> 2 GiB, read + written bytes, 10 launches "
                   f"back to back per variant, the fastest ({kind}); this GPU, this run"}


def c4_cpu_baseline(gcase, cores: int, repeats: int = 3) -> dict | None:
    """The reference Fortran on the C4 workload itself: ONE baroclinic step of the 316x316 mesh under
    `mpiexec -n cores` on a Morton processor-face partition (its own MPI halo), each rank reading
    the dense tables of its own elements (facepart.add_dense_tables); `repeats` runs, the median
    reported with the spread (the host cores are shared)."""
    from hnumo.facepart import add_dense_tables, face_partition
    from hnumo.roofline import element_updates_per_step
    try:
        t0 = time.perf_counter()
        parts = [add_dense_tables(face_partition(gcase, cores, r, "morton")) for r in range(cores)]
        runs = [t for t in (_run_reference(parts, 1, cores) for _ in range(repeats)) if t]
        wall = time.perf_counter() - t0
    except Exception as exc:  # pragma: no cover - diagnostic only
        print(f"[bench] C4 reference baseline failed: {exc}", file=sys.stderr)
        return None
    if not runs:
        return None
    eu = element_updates_per_step(gcase)
    t = sorted(runs)[len(runs) // 2]
    rates = sorted(eu / x for x in runs)
    return {"value": round(eu / t, 1), "unit": "element-updates/s", "cores": cores, "kind": "reference",
            "sample": f"dg316L3 (C4, {gcase.scalars['nelem']} elements), 1 baroclinic step of the reference Fortran "
                      f"(amdflang -O2) under mpiexec -n {cores} (Morton processor-face partition, its own MPI "
                      f"halo), one rank per core: {t:.2f} s (MPI_Wtime, max over ranks; median of {len(runs)} runs; "
                      f"{wall:.0f} s in all with the per-rank dense tables and bundles)",
            "spread": {"runs": len(runs), "min": round(rates[0], 1), "max": round(rates[-1], 1)}}


def _profiled(cfg: str, kname: str, k_ms: float) -> dict:
    """roofline.traffic and the rocprofv3 duration of the stage kernel from the committed profile
    summary (profiles/roofline_pmc.json, written by tools/profile_summary.py from a rocprofv3
    --kernel-trace --stats run and the FETCH_SIZE / WRITE_SIZE passes of the same bench command;
    the persistent kernel's stage-less trial launch excluded), and the DRAM rate those bytes
    make over this run's measured kernel time.  Empty if no summary matches config and kernel."""
    path = os.path.join(REPO, "profiles", "roofline_pmc.json")
    try:
        d = json.load(open(path)).get(cfg)
    except Exception:
        return {}
    if not d or d.get("kernel") != kname or "hbm_bytes_per_stage" not in d:
        return {}
    from hnumo.roofline import HBM_PEAK_GBS, kernel_src_sha16
    cur = kernel_src_sha16()
    if d.get("kernel_src_sha16") != cur:
        # a summary taken from other kernel sources is not this kernel's traffic
        return {"traffic_stale": f"{d['source']} was measured on kernel sources {d.get('kernel_src_sha16')}, "
                                 f"these are {cur}: PMC fields omitted"}
    dram = d["hbm_bytes_per_stage"] / (k_ms * 1e-3) / 1e9
    return {"traffic": d["hbm_bytes_per_stage"], "traffic_source": f"{d['source']} (kernel sources {cur})",
            "rocprof_stage_us": d["stage_us"], "traffic_over_algorithmic": d["traffic_over_algorithmic"],
            "dram_achieved": round(dram, 1), "dram_frac": round(dram / HBM_PEAK_GBS, 4)}


def _limiter(frac: float, dram_frac: float | None, E: int) -> str:
    """What the measurements say limits the stage kernel: the DRAM bytes it really moves (PMC)
    against the algorithmic bytes' rate at the same kernel time."""
    if dram_frac is None:
        return "unmeasured (no PMC traffic summary for this config)"
    if dram_frac >= 0.6:
        return f"HBM: DRAM traffic at {dram_frac:.0%} of peak"
    why = (f"{E} elements on 256 CUs ({E / 256.0:.1f} per CU), state and statics resident in LDS across the "
           "stages" if E < 4096 else "instruction issue and latency with 5 workgroups per CU, the LDS arena's limit (SQ "
           "counters: profiles/roofline_pmc.json sq_per_element_stage; DESIGN.md section 9)")
    return f"not HBM: DRAM traffic at {dram_frac:.1%} of peak while the algorithmic bytes run at {frac:.1%}; {why}"


def _claim_stdout():
    """The JSON line is the only thing on stdout: libraries that print to fd 1 (RCCL's version
    banner at communicator set-up, the HIP runtime) are sent to stderr; the line goes to a private
    copy of the original stdout."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: 20 at N=1 (dg25L3), 5 at N>1 (C4)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, help="default: dg25L3 at N=1, dg316L3 (C4) at N>1; lake200 = C5")
    ap.add_argument("--weak", action="store_true", help="N>1: N blocks of the 1-GPU mesh (weak scaling)")
    ap.add_argument("--halo", default="faces", choices=["faces", "ghost"],
                    help="N>1: processor faces (the reference's contract) or a one-element ghost layer")
    ap.add_argument("--order", default=None, choices=["block", "morton"],
                    help="N>1 processor-face partition: block (default; C4's 4x2 blocks) or morton (default for lake200)")
    ap.add_argument("--emulate", default=None, metavar="W:R",
                    help="one GPU: rank R of a W-rank run as its own neighbour (see the module docstring)")
    ap.add_argument("--emulate-lists", default="peers", choices=["peers", "one"],
                    help="--emulate: keep the rank's per-neighbour processor-face lists (peers: one RCCL send/recv "
                         "pair per real neighbour, the real run's message shape) or merge them into one list")
    ap.add_argument("--emulate-halo", default=None, choices=["mirror", "frozen"],
                    help="--emulate: what the rank's processor faces receive -- its own traces (mirror; default "
                         "except lake configs) or the first message of each exchange site again (frozen: the "
                         "at-rest neighbour of an at-rest lake; hnumo_debug_frozen_halo)")
    ap.add_argument("--cpu-steps", type=int, default=8)
    ap.add_argument("--cpu-cores", type=int, default=16,
                    help="MPI ranks (= host cores) of the reference CPU baseline (the GPU box's share is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c4-cpu", action="store_true", help="N=1: skip the reference C4 step on the host cores")
    ap.add_argument("--no-c4", action="store_true", help="N=1: skip the c4/c3/c5_single_gpu figures")
    ap.add_argument("--no-base", action="store_true", help="N>1: skip the strong-scaling base (whole mesh on rank 0's GPU)")
    ap.add_argument("--summation", default="reference", choices=["reference", "factored"],
                    help="stage summation order (hnumo_set_summation); only 'reference' meets the 1e-10 bar")
    args = ap.parse_args()
    json_out = _claim_stdout()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    emu = None
    if args.emulate:
        if world != 1:
            sys.exit("--emulate runs on one GPU (one rank)")
        W, R = (int(x) for x in args.emulate.split(":"))
        if not (W > 1 and 0 <= R < W):
            sys.exit("--emulate W:R needs W > 1 and 0 <= R < W")
        emu = (W, R)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    nparts, prank = emu if emu else (world, rank)   # the partition this process runs
    multi = nparts > 1
    import torch
    dist = None
    setup = {}
    if multi:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        t0 = time.perf_counter()
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        setup["init_process_group_s"] = round(time.perf_counter() - t0, 2)

    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine
    from hnumo.roofline import HBM_PEAK_GBS, element_updates_per_step, stage_bytes, step_bytes

    weak = multi and args.weak
    cfg_name = args.config or ("dg316L3" if multi and not weak else "dg25L3")
    order = args.order or ("morton" if cfg_name.startswith("lake") else "block")
    emu_halo = args.emulate_halo or ("frozen" if cfg_name.startswith("lake") else "mirror")
    steps = args.steps if args.steps is not None else (20 if not multi or weak else 5)
    base_cfg = make_config(cfg_name)
    eng, parallelism, scaling = None, "single", "weak"
    case, gcase, live_halo = None, None, False
    if multi:
        from hnumo.partition import partition, rank_grid
        px, py = rank_grid(nparts) if (order == "block" or args.halo == "ghost" or weak) else (nparts, 1)
        if weak:
            x0, x1 = base_cfg["xdims"]
            y0, y1 = base_cfg["ydims"]
            gcfg = make_config(cfg_name, nelx=base_cfg["nelx"] * px, nely=base_cfg["nely"] * py,
                               xdims=(x0, x0 + (x1 - x0) * px), ydims=(y0, y0 + (y1 - y0) * py))
        else:
            gcfg = base_cfg
            scaling = "strong"
        t0 = time.perf_counter()
        gcase = build_case(gcfg, dense=False)
        setup["case_build_s"] = round(time.perf_counter() - t0, 2)
        obj = [Engine.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        err = None
        try:
            t0 = time.perf_counter()
            if args.halo == "faces":
                from hnumo.facepart import face_partition
                case = face_partition(gcase, nparts, prank, order)
                if emu:
                    from hnumo.facepart import self_neighbour
                    case = self_neighbour(case, per_peer=args.emulate_lists == "peers")
            else:
                if emu:
                    raise ValueError("--emulate needs the processor-face halo")
                case = partition(gcase, nparts, prank)
            setup["partition_s"] = round(time.perf_counter() - t0, 2)
            t0 = time.perf_counter()
            eng = Engine(case, device=local_rank, comm_id=obj[0], summation=args.summation)
            if emu and emu_halo == "frozen":
                eng.debug_frozen_halo(True)
            setup["engine_create_s"] = round(time.perf_counter() - t0, 2)
            eng.set_resident(True)
            q, qb, qp = eng.state()
            t0 = time.perf_counter()
            eng.ti_rk_bcl(q, qb, qp)                 # first step: uploads, captures the graph, exchanges
            setup["first_step_s"] = round(time.perf_counter() - t0, 2)
        except Exception as exc:  # pragma: no cover - depends on the node
            err = f"{type(exc).__name__}: {exc}"
        bad = torch.tensor([1 if err else 0], device="cuda")
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if bad.item():
            # no substitute number (independent replicas would be another kind of measurement)
            if rank == 0 or err:
                print(json.dumps({"error": "multi-GPU halo setup failed", "rank": rank,
                                  "detail": err or "on another rank"}), file=sys.stderr)
            if eng is not None:
                eng.close()
            dist.destroy_process_group()
            sys.exit(1)
        else:
            how = ("processor-face halo (reference contract) over RCCL p2p, traces on a 2nd stream overlapped with "
                   "interior elements" if args.halo == "faces" else "one-element ghost halo over RCCL p2p")
            if order == "block" or args.halo == "ghost" or weak:
                bx, by = gcfg["nelx"] // px, gcfg["nely"] // py
                parallelism = (f"domain decomposition {px}x{py} blocks of {bx}x{by} elements "
                               f"({gcfg['nelx']}x{gcfg['nely']} total), {how}")
            else:
                parallelism = (f"domain decomposition: {nparts} Morton (Z-order) pieces of the "
                               f"{gcfg['nelx']}x{gcfg['nely']} elements, {how}")
            if emu:
                parallelism = (f"EMULATED on one GPU: rank {prank} of [{parallelism}] as its own neighbour "
                               f"({args.emulate_lists} lists, {emu_halo} halo)")
            live_halo = True
    if eng is None:
        if case is None:
            case = build_case(base_cfg, dense=False)
        eng = Engine(case, device=local_rank, summation=args.summation)
        eng.set_resident(True)
        q, qb, qp = eng.state()
        eng.ti_rk_bcl(q, qb, qp)                   # uploads the state, builds the graph
    else:
        q, qb, qp = eng.state()
    if args.warmup > 1:
        eng.bench_steps(args.warmup - 1)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    _, k_ms, _ = eng.bench_steps(steps)               # synchronises the engine stream; checks the flags
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # the timed run's own persistent-path counters and stage path, read before any diagnostic step
    # below (step_breakdown, the halo check) can add aborts or re-probes of its own
    timed_stats = eng.persistent_stats
    timed_path = eng.stage_path
    eu_local = element_updates_per_step(case) * steps
    if dist is not None:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        n = torch.tensor([eu_local], device="cuda", dtype=torch.float64)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        eu_total = float(n.item())
    else:
        eu_total = float(eu_local)
    path = timed_path
    kname = "btp_subcycle_kernel" if path == "persistent" else "btp_stage_kernel"
    k_src = "graph event nodes around the corrector sub-cycle"
    if not (k_ms and k_ms > 0):
        k_ms = eng.time_stage_kernel(2)
        k_src = "events around 2 direct corrector sub-cycles" + (" (incl. halo exchanges)" if multi else "")
    if path == "persistent":
        k_src += "; one launch per sub-cycle, time per stage = launch time / (N_btp*kstages)"
    eng.sync(q, qb, qp)
    if not (abs(qb).max() < 1e30):
        raise RuntimeError("non-finite state after benchmark")
    halo_check = None
    if live_halo:
        # the halo proves itself: one step from the IC over the live RCCL transport against the
        # same step computed on this GPU alone (hnumo/halocheck.py); a mismatch is an error
        from hnumo import halocheck as HC
        t0 = time.perf_counter()
        mine = HC.owned(case, HC.step_from_ic(eng))
        if emu:
            # the self-neighbour partition's own local-exchange-group step is what the RCCL run must
            # equal; the real run's check (all W partitions as a local group) is built and stepped
            # too, to time it, but not compared (a real rank's neighbours are other ranks)
            _, ref = HC.reference_faces_cases([case], 0, local_rank, frozen=emu_halo == "frozen")
            ref = HC.owned(case, ref)
            t1 = time.perf_counter()
            HC.reference_faces(gcase, nparts, prank, order, local_rank)
            setup["halocheck_real_run_s"] = round(time.perf_counter() - t1, 2)
            against = "the same self-neighbour partition as a local exchange group on this GPU (device copies)"
        elif args.halo == "faces":
            _, ref = HC.reference_faces(gcase, world, rank, order, local_rank)
            ref = HC.owned(case, ref)
            against = "the same processor-face partitions as one local exchange group on each GPU (device copies)"
        else:
            ref = HC.reference_ghost(gcase, case, local_rank)
            against = "the whole mesh as one rank on each GPU"
        setup["halocheck_s"] = round(time.perf_counter() - t0, 2)
        same, rel = HC.compare(mine, ref)
        bad = torch.tensor([0 if same else 1], device="cuda")
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        relt = torch.tensor([rel], device="cuda", dtype=torch.float64)
        dist.all_reduce(relt, op=dist.ReduceOp.MAX)
        halo_check = {"halo_bitwise": not bad.item(), "steps_from_ic": 1, "against": against,
                      "max_rel_diff": float(relt.item())}
        if bad.item():
            if rank == 0:
                print(json.dumps({"error": "multi-GPU halo check failed", "halo_check": halo_check}), file=sys.stderr)
            raise RuntimeError(f"halo check failed: the RCCL run differs from {against} (max rel {relt.item():.3e})")

    value = eu_total / elapsed
    ms_per_step = 1e3 * elapsed / steps
    sb = stage_bytes(case)
    roof = None
    bd = None
    copy_bw = None
    if not multi:
        bd = step_breakdown(eng, case, 2)
        copy_bw = stream_copy(local_rank)
    if k_ms and k_ms > 0:
        achieved = sb / (k_ms * 1e-3) / 1e9
        step_ach = step_bytes(case) * steps / elapsed / 1e9
        E = case.scalars["nelem"]
        # the roofline the kernel is priced against is HBM (no MFMA work on this path); what the
        # measurements say limits it is `limiter` (from the PMC traffic, below)
        roof = {"bound": "hbm",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": kname, "kernel_avg_us": round(k_ms * 1e3, 3),
                "algorithmic_bytes_per_launch": int(sb), "timing": k_src,
                "step_achieved": round(step_ach, 1), "step_frac": round(step_ach / HBM_PEAK_GBS, 4),
                "step_bytes": int(step_bytes(case)),
                "step_model": "E*(2*N_btp*kstages*B_stage + B_bcl_step)/T_step per GPU (hnumo/roofline.py)"}
        if copy_bw:
            roof["peak_measured"] = copy_bw["gbs"]
            roof["frac_measured"] = round(achieved / copy_bw["gbs"], 4)
            roof["step_frac_measured"] = round(step_ach / copy_bw["gbs"], 4)
            roof["peak_measured_how"] = copy_bw["how"]
        roof.update(_profiled(cfg_name, kname, k_ms) if not multi or weak else {})
        roof["limiter"] = _limiter(roof["frac"], roof.get("dram_frac"), E)
        if bd:
            roof.update(bd)
    S = case.scalars
    if multi and not weak:
        what = "C5" if cfg_name.startswith("lake") else "C4"
        wl = (f"{cfg_name} ({what}): {base_cfg['test_case']} {base_cfg['nelx']}x{base_cfg['nely']} = "
              f"{base_cfg['nelx'] * base_cfg['nely']} elements split over {nparts} GPUs")
    else:
        wl = f"{cfg_name}: {base_cfg['test_case']} {base_cfg['nelx']}x{base_cfg['nely']} elements per GPU"
    out = {
        "metric": "DG element-updates/sec (all layers, per RK stage)",
        "value": round(value, 1), "unit": "element-updates/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "emulated" if emu else scaling, "vs_baseline": None, "dtype": "f64",
        "data": f"synthetic (analytic {base_cfg['test_case']} IC)",
        "config": {"workload": wl + f", N={S['ngl'] - 1}, {S['nlayers']} layers, "
                               f"N_btp={S['N_btp']}, kstages={S['kstages']}",
                   "elements": int(eu_total / steps / (2 * S["N_btp"] * S["kstages"])),
                   "elements_per_gpu": int(eu_local / steps / (2 * S["N_btp"] * S["kstages"])),
                   "nlayers": S["nlayers"], "nop": S["ngl"] - 1, "parallelism": parallelism,
                   "summation": args.summation, "stage_path": path},
        "roofline": roof,
    }
    if halo_check is not None:
        out["halo_bitwise"] = halo_check["halo_bitwise"]
        out["halo_check"] = halo_check
    # the persistent path's in-launch residency check: launches that gave up (and were redone on
    # per-stage launches), trial re-probes, and re-probes that found the grid resident again
    out["persistent"] = timed_stats
    # every HNUMO_* environment setting the engine read (hnumo_overrides; experiment knobs are
    # honoured only with HNUMO_EXPERIMENTS=1): empty on a clean box
    out["engine_env"] = eng.overrides
    eng.close()
    if multi and not weak and not args.no_base:
        # the strong-scaling base: the whole mesh on rank 0's GPU alone, timed in this run, so the
        # N>1 line carries the 1-GPU number of the SAME workload (the N=1 line is configs[1])
        base = None
        if rank == 0:
            t0 = time.perf_counter()
            try:
                base = single_gpu_line(cfg_name, f"{cfg_name} (whole mesh) on rank 0's GPU", 3, case=gcase,
                                       device=local_rank, breakdown=False)
            except Exception as exc:  # pragma: no cover - diagnostic only
                base = {"error": f"{type(exc).__name__}: {exc}"}
            setup["strong_scaling_base_s"] = round(time.perf_counter() - t0, 2)
        dist.barrier()
        if rank == 0 and base is not None:
            out["strong_scaling_base"] = base
            if "value" in base:
                v = value if not emu else gcase.scalars["nelem"] * 2 * S["N_btp"] * S["kstages"] * 1e3 / ms_per_step
                out["speedup_vs_base"] = round(v / base["value"], 3)
                # strong-scaling efficiency of THIS workload (the driver's 1 -> N curve divides by the
                # N=1 line, which is configs[1], a different mesh)
                out["efficiency_vs_base"] = round(v / base["value"] / nparts, 3)
    if emu:
        # value is ONE rank block's rate on one GPU, not a measured N-GPU (or whole-mesh) rate
        out["emulated"] = True
        E_g = gcase.scalars["nelem"]
        out["emulation"] = {
            "world": nparts, "rank": prank, "order": order, "lists": args.emulate_lists, "halo": emu_halo,
            "messages_per_exchange": len(case.fneighbours),
            "rank_elements": S["nelem"], "processor_faces": int(sum(n.faces.size for n in case.fneighbours)),
            "projection_eu_per_s": round(E_g * 2 * S["N_btp"] * S["kstages"] * 1e3 / ms_per_step, 1),
            "note": f"this GPU ran rank {prank}'s block at {ms_per_step:.3f} ms per step with every exchange going to "
                    f"itself; if each of the {nparts} GPUs runs its block in that time, the whole-mesh rate is the "
                    "projection (xGMI transfer time of the real messages not included)"}
    if multi:
        out["setup_s"] = setup
    if rank == 0 and not multi and not args.no_c4 and args.config is None:
        for key, cfg, wl, n in [("c4_single_gpu", "dg316L3", "dg316L3 (C4: 316x316 elements, N=4, 3 layers)", 3),
                                ("c3_single_gpu", "dg25N7L3", "dg25N7L3 (C3: 25x25 elements, N=7, 3 layers)", 5),
                                ("c5_single_gpu", "lake200", "lake200 (C5: the lake at rest, 200x200 elements, "
                                                             "N=4, 2 layers, wetting/drying BC path)", 3)]:
            try:
                c = build_case(make_config(cfg), dense=False)
                out[key] = single_gpu_line(cfg, wl, n, case=c)
                if key == "c4_single_gpu" and not args.no_cpu_baseline and not args.no_c4_cpu:
                    ncores = max(1, min(args.cpu_cores, len(os.sched_getaffinity(0))))
                    cb = c4_cpu_baseline(c, ncores)
                    if cb:
                        out[key]["cpu_baseline"] = cb
                del c
            except Exception as exc:  # pragma: no cover - diagnostic only
                out[key] = {"error": f"{type(exc).__name__}: {exc}"}
    if rank == 0 and not multi and not args.no_cpu_baseline:
        ncores = max(1, min(args.cpu_cores, len(os.sched_getaffinity(0))))
        out["cpu_baseline"] = cpu_baseline(build_case(make_config(cfg_name)), args.cpu_steps, ncores)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""A/B timing of engine builds (HNUMO_LIB) on a list of configurations: per-stage / persistent
stage time, one-step time and a hash of the state after 2 steps (equal hashes = same bits).
Usage (GPU): HNUMO_LIB=<so> python tools/ab_stage.py cfg[@k=v,...][:persist|:stage] ..."""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.roofline import stage_bytes  # noqa: E402

lib = os.environ.get("HNUMO_LIB", "default")
for arg in sys.argv[1:]:
    cfg, _, mode = arg.partition(":")
    os.environ["HNUMO_PERSISTENT"] = "0" if mode == "stage" else "1"
    from hnumo.engine import Engine
    # cfg@k=v,k=v: integer overrides of the configuration (e.g. dg316L3@nelx=79,nely=158)
    cfg, _, ov = cfg.partition("@")
    over = {k: int(v) for k, v in (x.split("=") for x in ov.split(",") if x)}
    case = build_case(make_config(cfg, **over), dense=False)
    e = Engine(case)
    e.set_resident(True)
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    e.ti_rk_bcl(q, qb, qp)
    e.sync(q, qb, qp)
    h = hashlib.sha256(q.tobytes() + qb.tobytes() + qp.tobytes()).hexdigest()[:16]
    ms = e.time_stage_kernel(2)
    t0 = time.perf_counter()
    e.bench_steps(3)
    t = (time.perf_counter() - t0) / 3
    print(f"{os.path.basename(lib)} {arg} path={e.stage_path}: stage {ms*1e3:.2f} us, "
          f"frac {stage_bytes(case)/(ms*1e-3)/8e12:.3f}, step {t*1e3:.2f} ms, state {h}", flush=True)
    e.close()

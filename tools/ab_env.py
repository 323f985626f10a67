"""A/B timing of engine environment knobs on one configuration (the case is built once):
per-stage / persistent stage time, one-step time and a hash of the state after 2 steps (equal
hashes = same bits).
Usage (GPU): python tools/ab_env.py cfg[:persist|:stage] "K=V,K=V" "K=V" ...   ("" = defaults)"""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.roofline import stage_bytes  # noqa: E402

cfg, _, mode = sys.argv[1].partition(":")
os.environ["HNUMO_PERSISTENT"] = "0" if mode == "stage" else "1"
from hnumo.engine import Engine  # noqa: E402
os.environ["HNUMO_EXPERIMENTS"] = "1"   # the engine honours HNUMO_* experiment knobs only with this

case = build_case(make_config(cfg), dense=False)
reps = int(os.environ.get("AB_REPS", "1"))
for _ in range(reps):
    for spec in sys.argv[2:]:
        kv = [x.split("=", 1) for x in spec.split(",") if x]
        old = {k: os.environ.get(k) for k, _ in kv}
        for k, v in kv:
            os.environ[k] = v
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
        print(f"{cfg}:{mode} [{spec}] path={e.stage_path}: stage {ms*1e3:.2f} us, "
              f"frac {stage_bytes(case)/(ms*1e-3)/8e12:.3f}, step {t*1e3:.2f} ms, state {h}", flush=True)
        e.close()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

"""Per-stage kernel timing for arena sizings (HNUMO_STAGE_NB) at a configuration. GPU only."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.roofline import stage_bytes  # noqa: E402
os.environ["HNUMO_EXPERIMENTS"] = "1"   # the engine honours HNUMO_* experiment knobs only with this

cfg = sys.argv[1] if len(sys.argv) > 1 else "dg316L3"
nbs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "4"]
case = build_case(make_config(cfg), dense=False)
ref = None
for nb in nbs:
    os.environ["HNUMO_STAGE_NB"] = nb
    os.environ["HNUMO_PERSISTENT"] = "0"
    from hnumo.engine import Engine
    e = Engine(case)
    e.set_resident(True)
    q, qb, qp = e.state()
    e.ti_rk_bcl(q, qb, qp)
    ms = e.time_stage_kernel(1)
    t0 = time.perf_counter()
    e.bench_steps(2)
    t = (time.perf_counter() - t0) / 2
    e.sync(q, qb, qp)
    import numpy as np
    same = "ref" if ref is None else bool(np.array_equal(ref, qb))
    ref = qb.copy() if ref is None else ref
    print(f"{cfg} NB={nb}: stage {ms*1e3:.1f} us, frac {stage_bytes(case)/(ms*1e-3)/8e12:.3f}, step {t*1e3:.1f} ms, bitwise {same}",
          flush=True)
    e.close()

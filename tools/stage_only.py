"""Runs only the fused stage kernel (corrector sub-cycles of dg25L3) -- for counter profiles."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.engine import Engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "dg25L3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
case = build_case(make_config(cfg), dense=False)
eng = Engine(case)
eng.set_resident(True)
q, qb, qp = eng.state()
try:
    eng.ti_rk_bcl(q, qb, qp)
except Exception as ex:  # HNUMO_STAGE_DBG timing experiments break the physics
    print("warm-up step:", ex)
print(f"{cfg}: stage avg {eng.time_stage_kernel(n) * 1e3:.2f} us")

"""Stage-kernel time under HNUMO_STAGE_DBG phase switches (timing only: the switches break the
physics), one case build, one engine per setting.  GPU only; diagnostics.
Usage: python tools/dbg_sweep.py <cfg> <dbg> [<dbg> ...]   (bits: 1 no face projections,
2 no Laplacian, 4 no volume sums, 32 no time averages)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
from hnumo.case import build_case, make_config  # noqa: E402
os.environ["HNUMO_EXPERIMENTS"] = "1"   # the engine honours HNUMO_* experiment knobs only with this

cfg = sys.argv[1]
case = build_case(make_config(cfg), dense=False)
for d in sys.argv[2:]:
    os.environ["HNUMO_STAGE_DBG"] = d
    from hnumo.engine import Engine
    e = Engine(case)
    e.set_resident(True)
    q, qb, qp = e.state()
    try:
        e.ti_rk_bcl(q, qb, qp)
    except Exception as ex:  # the switches break the physics
        print("  warm-up:", str(ex)[:80])
    ms = e.time_stage_kernel(2)
    print(f"{cfg} dbg={d}: stage {ms * 1e3:.2f} us", flush=True)
    e.close()

"""Per-phase clock breakdown of btp_stage_kernel (HNUMO_STAGE_PROF=1). GPU only."""
import os
import sys

os.environ["HNUMO_STAGE_PROF"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
import numpy as np  # noqa: E402
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.engine import Engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "dg25L3"
case = build_case(make_config(cfg), dense=False)
eng = Engine(case)
eng.set_resident(True)
q, qb, qp = eng.state()
eng.ti_rk_bcl(q, qb, qp)
ms = eng.time_stage_kernel(1)
pr = eng.stage_profile().astype(np.int64)
d = np.diff(pr[:, :6], axis=1)
names = ["A loads", "B quad/grad/face", "D terms+sums", "E1 update", "E2 out+traces"]
print(f"{cfg}: stage avg {ms*1e3:.1f} us (direct events)")
for i, n in enumerate(names):
    print(f"  {n:14s} mean {d[:, i].mean():9.0f} clk  max {d[:, i].max():9.0f}")
dk = np.diff(np.concatenate([pr[:, 2:3], pr[:, 6:10]], axis=1), axis=1)
for k in range(dk.shape[1]):
    if dk[:, k].mean() > 0:
        print(f"    D{k:<12d} mean {dk[:, k].mean():9.0f} clk")
tot = pr[:, 5] - pr[:, 0]
print(f"  total per block mean {tot.mean():.0f} clk, max {tot.max():.0f}")
w0, w1 = pr[:, 10], pr[:, 11]
t0 = w0.min()
print(f"  wall (100MHz ticks): block start spread {np.percentile(w0 - t0, [0, 50, 90, 100])}, "
      f"block dur mean {(w1 - w0).mean():.0f} max {(w1 - w0).max():.0f}, span {(w1.max() - t0)}")

"""Per-phase clock breakdown of btp_stage_kernel (HNUMO_STAGE_PROF=1). GPU only; diagnostics."""
import os
import sys

os.environ["HNUMO_STAGE_PROF"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
import numpy as np  # noqa: E402
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.engine import Engine  # noqa: E402
os.environ["HNUMO_EXPERIMENTS"] = "1"   # the engine honours HNUMO_* experiment knobs only with this

cfg = sys.argv[1] if len(sys.argv) > 1 else "dg25L3"
case = build_case(make_config(cfg), dense=False)
eng = Engine(case)
eng.set_resident(True)
q, qb, qp = eng.state()
try:
    eng.ti_rk_bcl(q, qb, qp)
except Exception as ex:  # HNUMO_STAGE_DBG experiments break the physics; timing still counts
    print("warm-up step:", ex)
ms = eng.time_stage_kernel(1)
pr = eng.stage_profile().astype(np.int64)
print(f"{cfg}: stage avg {ms*1e3:.1f} us (direct events)")
for name, a, b in [("A loads", 0, 21), ("A2", 21, 1), ("B", 1, 2), ("D all", 2, 3), ("E1 update", 3, 4), ("E2 out", 4, 5)]:
    d = pr[:, b] - pr[:, a]
    print(f"  {name:12s} mean {d.mean():8.0f} clk  max {d.max():8.0f}")
prev = pr[:, 2]
for k in range(6):
    cur = pr[:, 6 + k]
    # a D-phase slot is printed only if this build wrote it: its clock lies between the previous
    # mark and the end of D in every block (unwritten slots hold stale values from other runs)
    if (cur >= prev).all() and (cur <= pr[:, 3]).all():
        print(f"    D{k}        mean {(cur - prev).mean():8.0f} clk")
        prev = cur
for w in range(4):
    print(f"    B wave{w} done mean {(pr[:, 12 + w] - pr[:, 1]).mean():8.0f} clk")
tot = pr[:, 5] - pr[:, 0]
print(f"  total per block mean {tot.mean():.0f} clk, max {tot.max():.0f}")
w0, w1 = pr[:, 30], pr[:, 31]
t0 = w0.min()
print(f"  wall (100MHz ticks): start spread {np.percentile(w0 - t0, [0, 50, 90, 100])}, "
      f"block dur mean {(w1 - w0).mean():.0f} max {(w1 - w0).max():.0f}, span {(w1.max() - t0)}")
hw = pr[:, 16:20]
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
xcc = pr[:, 20] & 15
print("  placement (first 12 blocks): xcc, se, cu, simd of waves 0-3")
for e in list(range(8)) + [256, 257, 512, 513]:
    if e < len(pr):
        print(f"    blk {e:4d}: xcc {xcc[e]} se {se[e, 0]} cu {cu[e, 0]:2d} simd {simd[e].tolist()}")
key = xcc * 1000 + se[:, 0] * 100 + cu[:, 0]
u, c = np.unique(key, return_counts=True)
hist = {int(k): int(n) for k, n in zip(*np.unique(c, return_counts=True))}
print(f"  distinct CUs used {len(u)}, blocks per CU over the launch -> number of CUs: {hist}")
# SIMD sharing of the blocks' role waves on each CU (persistent: all blocks resident together):
# for wave w, the CUs on which two or more blocks run their wave w on the same SIMD
if getattr(eng, "stage_path", "") == "persistent":
    for w in range(4):
        coll = 0
        for k in u:
            sims = simd[key == k, w]
            coll += int(len(sims) != len(set(sims.tolist())))
        print(f"    wave {w}: CUs with two blocks' wave {w} on one SIMD: {coll} of {len(u)}")

# (slots 24-29: the persistent sub-cycle only; a per-stage launch leaves them unwritten)
if getattr(eng, "stage_path", "") == "persistent" and (pr[:, 26] > 0).all():
    nst = pr[:, 26].astype(float)
    aw, wk, wt = pr[:, 24] / nst, pr[:, 25] / nst, pr[:, 27] / nst
    print(f"  trace wait per stage (longest thread): mean {wt.mean():.0f} clk, p10 {np.percentile(wt, 10):.0f}, "
          f"p90 {np.percentile(wt, 90):.0f}; work without it: mean {(wk - wt).mean():.0f}, max {(wk - wt).max():.0f}")
    for x in range(8):
        sel = xcc == x
        print(f"    xcc {x}: work-wait mean {(wk - wt)[sel].mean():.0f}, wait {wt[sel].mean():.0f}")
    bpc = c[np.searchsorted(u, key)]
    print(f"  persistent: per stage A(+waits) mean {aw.mean():.0f} clk, work mean {wk.mean():.0f} clk")
    ph = [pr[:, k] / nst for k in (8, 9, 10, 11, 29)]
    print("  persistent per-stage phase means: A2 %.0f | B %.0f | D %.0f (wave-0 volume sums %.0f) | E %.0f clk"
          % (ph[0].mean(), ph[1].mean(), ph[2].mean(), ph[4].mean(), ph[3].mean()))
    if (pr[:, 23] > 0).all() and (pr[:, 28] > 0).all():  # SLATE (N=7): the last stage's D split
        print("  last stage, from D's start: volume sums done %.0f clk, the last wave's D work done %.0f clk"
              % ((pr[:, 28] - pr[:, 2]).mean(), (pr[:, 23] - pr[:, 2]).mean()))
    for k in sorted(set(bpc.tolist())):
        sel = bpc == k
        print(f"    CUs with {k} blocks: {sel.sum()} blocks, A(+waits) {aw[sel].mean():.0f}, work {wk[sel].mean():.0f} "
              f"(max {wk[sel].max():.0f}) clk, trace wait {wt[sel].mean():.0f}, work-wait {(wk - wt)[sel].mean():.0f}")

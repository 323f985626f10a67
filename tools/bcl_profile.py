"""Phase clocks of the baroclinic element kernels (mass_elem, cons_elem, mom_elem) from an
HNUMO_BCL_PROF=1 build (diagnostics).  Usage (GPU): HNUMO_LIB=<prof .so> python tools/bcl_profile.py [cfg]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
import numpy as np  # noqa: E402
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.engine import Engine, lib  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "dg25L3"
case = build_case(make_config(cfg), dense=False)
eng = Engine(case)
eng.set_resident(True)
q, qb, qp = eng.state()
for _ in range(2):
    eng.ti_rk_bcl(q, qb, qp)
buf = np.zeros(4 * 8192 * 8, dtype=np.uint64)
L = lib()
L.hnumo_bcl_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert L.hnumo_bcl_prof(buf.ctypes.data, buf.size) == 0
E = case.scalars["nelem"]
pr4 = buf.reshape(4, 8192, 8).astype(np.int64)
pr = pr4[:, :E]
names = {0: ("mass_elem", ["loads", "quad", "node sums", "faces+store", "final"]),
         1: ("cons_elem", ["loads", "-", "quad", "node", "final"]),
         2: ("mom_elem", ["loads", "ph1 interp", "ph2 couple+lap", "ph3 weak", "ph4 tail"]),
         3: ("mom_flux_face", ["loads", "quad lane", "-", "-", "end"])}
NF = case.scalars["nface"] if "nface" in case.scalars else E
for k, (nm, ph) in names.items():
    a = pr4[k, :NF] if k == 3 else pr[k]
    tot = a[:, 5] - a[:, 0]
    w0, w1 = a[:, 6], a[:, 7]
    print(f"{nm}: block clocks mean {tot.mean():.0f} max {tot.max():.0f}; wall (100 MHz) start spread "
          f"{(w0.max() - w0.min())}, block span mean {(w1 - w0).mean():.0f}, kernel span {(w1.max() - w0.min())}")
    prev = a[:, 0]
    for i, p in enumerate(ph):
        cur = a[:, i + 1]
        if p != "-" and (cur > 0).all():
            d = cur - prev
            print(f"    {p:16s} mean {d.mean():8.0f}  max {d.max():8.0f}")
            prev = cur
    if k != 3 and E > 256:
        # the CUs of blocks b % 256 < E % 256 hold one block more (round-robin dealing, 256 CUs)
        heavy = (np.arange(E) % 256) < (E % 256)
        span = w1 - w0
        print(f"    block span (100 MHz) on CUs holding one more: {span[heavy].mean():.0f}, the others: "
              f"{span[~heavy].mean():.0f}; start of the last-started block {w0.max() - w0.min()}")
        marks = [0] + [i + 1 for i, p in enumerate(ph) if p != "-"]  # (phases with a mark of their own)
        for b in np.argsort(-tot)[:6]:
            ds = [int(a[b, marks[i + 1]] - a[b, marks[i]]) for i in range(len(marks) - 1)]
            print(f"    slow block {b:4d} ({'3' if heavy[b] else '2'} on its CU): clocks {tot[b]}, phases {ds}, "
                  f"wall start +{w0[b] - w0.min()} end +{w1[b] - w0.min()}")
eng.close()

"""Kernel timeline of one replayed dg25L3 step from a rocprofv3 --kernel-trace CSV (diagnostics):
each kernel's duration and the idle gap before it, over the last `--steps` steps of the trace.
Usage: python tools/step_timeline.py <kernel_trace.csv> [nsteps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nst = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts with the predictor's first kernel after a corrector's mom_elem; take the last steps
names = [r["Kernel_Name"] for r in rows]
ends = [i for i, n in enumerate(names) if n.startswith("void hnumo::mom_elem_kernel")]
# two mom_elem per step (predictor, corrector): the last nst steps span ends[-2*nst]+1 .. ends[-1]
lo = ends[-2 * nst - 1] + 1 if len(ends) > 2 * nst else 0
hi = ends[-1]
sel = rows[lo:hi + 1]
t0 = int(sel[0]["Start_Timestamp"])
prev_end = None
busy = 0
agg = {}
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    nm = r["Kernel_Name"].split("(")[0].replace("void hnumo::", "")
    if nst == 1:
        print(f"{(s - t0) / 1e3:9.2f} us  gap {gap:7.2f}  dur {(e - s) / 1e3:9.2f}  {nm}")
    a = agg.setdefault(nm, [0, 0.0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e3
    a[2] += gap
    busy += e - s
    prev_end = e
span = (int(sel[-1]["End_Timestamp"]) - t0) / 1e3
print(f"span {span:.2f} us over {nst} step(s); kernels busy {busy / 1e3:.2f} us; idle {span - busy / 1e3:.2f} us")
for nm, (c, d, g) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {nm:60s} x{c:3d}  {d / nst:8.2f} us/step  gaps before {g / nst:6.2f} us/step")

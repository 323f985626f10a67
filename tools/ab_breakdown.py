"""A/B of an engine environment knob by the per-kernel step breakdown (hnumo_step_breakdown: an
event after every launch of two direct steps): which kernels a knob moves, and by how much, with
the state hash after 2 steps (equal hashes = same bits).  The case is built once.
Usage (GPU): python tools/ab_breakdown.py cfg[:stage] KNOB v1 v2 [...]   (AB_REPS=n repeats)"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
from hnumo.case import build_case, make_config  # noqa: E402

cfg, _, mode = sys.argv[1].partition(":")
if mode == "stage":
    os.environ["HNUMO_PERSISTENT"] = "0"
from hnumo.engine import Engine  # noqa: E402
os.environ["HNUMO_EXPERIMENTS"] = "1"   # the engine honours HNUMO_* experiment knobs only with this

knob, values = sys.argv[2], sys.argv[3:]
case = build_case(make_config(cfg), dense=False)
for _ in range(int(os.environ.get("AB_REPS", "1"))):
    for v in values:
        os.environ[knob] = v
        e = Engine(case)
        e.set_resident(True)
        q, qb, qp = e.state()
        e.ti_rk_bcl(q, qb, qp)
        e.ti_rk_bcl(q, qb, qp)
        e.sync(q, qb, qp)
        h = hashlib.sha256(q.tobytes() + qb.tobytes() + qp.tobytes()).hexdigest()[:16]
        bd = e.step_breakdown(2)
        ks = " ".join(f"{k} {u:.1f}" for k, u in sorted(bd.items(), key=lambda kv: -kv[1]))
        print(f"{cfg} {knob}={v}: state {h} | us/step: {ks}", flush=True)
        e.close()

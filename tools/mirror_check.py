"""Self-neighbour mirror diagnostics (bench.py --emulate): rank R of a W-rank processor-face
partition run as its own neighbour, against the same rank inside the real W-rank local exchange
group on this GPU, step by step from the initial condition.

    python tools/mirror_check.py <cfg> <W> <R> <order> [steps] [nelx]

Prints per step: finite?, the max |U|, |V| of the barotropic state, and the max relative
difference of the mirror rank's state from the real rank's (the mirror feeds each processor face
its own side's traces, so they part once the state moves)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))


def main():
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine, group_ti_rk_bcl, local_group
    from hnumo.facepart import face_partition, self_neighbour
    cfg, W, R, order = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    ov = {}
    if len(sys.argv) > 6:
        ov = dict(nelx=int(sys.argv[6]), nely=int(sys.argv[6]))
    g = build_case(make_config(cfg, **ov), dense=False)
    parts = [face_partition(g, W, r, order) for r in range(W)]
    real = [Engine(p) for p in parts]
    local_group(real)
    rs = [e.state() for e in real]
    variants = {}
    for name, pp, fz in (("peers+mirror", True, False), ("one+mirror", False, False), ("peers+frozen", True, True)):
        pc = self_neighbour(face_partition(g, W, R, order), per_peer=pp)
        e = Engine(pc)
        if fz:
            e.debug_frozen_halo(True)
        local_group([e])
        variants[name] = (e, e.state())
    print(f"{cfg} W={W} R={R} {order}: rank elements {parts[R].scalars['nelem']}, "
          f"neighbours {[n.rank for n in parts[R].fneighbours]} ({[n.faces.size for n in parts[R].fneighbours]} faces)")
    for s in range(steps):
        group_ti_rk_bcl(real, rs)
        ref = rs[R]
        line = [f"step {s + 1}: real |U|max {np.abs(ref[1][2:4]).max():.3e}"]
        for name, (e, st) in variants.items():
            try:
                group_ti_rk_bcl([e], [st])
                rc = "ok"
            except Exception as exc:
                rc = f"{type(exc).__name__}: {str(exc)[:60]}"
            fin = all(np.isfinite(x).all() for x in st)
            rel = max(float(np.abs(x - y).max()) / (float(np.abs(y).max()) or 1.0) for x, y in zip(st, ref))
            line.append(f"{name}: rc {rc} finite {fin} |U|max {np.abs(st[1][2:4]).max():.3e} rel {rel:.3e}")
        print(" | ".join(line), flush=True)
    for e, _ in variants.values():
        e.close()
    for e in real:
        e.close()


if __name__ == "__main__":
    main()

"""Self-neighbour mirror diagnostics, one barotropic RHS (create_rhs_btp) at the initial condition:
rank R of a W-rank processor-face partition as its own neighbour against the same elements in the
whole mesh run as one rank.  At the initial condition a continuous state's traces are the same
from either side of a face, so the two RHS must agree up to the processor faces' orientation
(rounding); the elements where they do not are printed with their processor faces.

    python tools/mirror_rhs.py <cfg> <W> <R> <order> [key=value ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))


def main():
    from hnumo.case import build_case, make_config
    from hnumo.engine import Engine
    from hnumo.facepart import face_partition, self_neighbour
    cfg, W, R, order = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    ov = {}
    for kv in sys.argv[5:]:   # config overrides k=v (e.g. kstages=1 dt=1.8: one barotropic stage)
        k, v = kv.split("=")
        ov[k] = int(v) if v.isdigit() else float(v)
    g = build_case(make_config(cfg, **ov), dense=False)
    pc = self_neighbour(face_partition(g, W, R, order))
    e = Engine(pc, comm_id=Engine.rccl_unique_id())   # (the RCCL self-neighbour engine: a lone call)
    if os.environ.get("MIRROR_FROZEN") == "1":
        e.debug_frozen_halo(True)
    q, qb, qp = e.state()
    r_m = e.create_rhs_btp(qb, qp)
    eg = Engine(g)
    q, qb, qp = eg.state()
    r_g = eg.create_rhs_btp(qb, qp)
    P = pc.scalars["ngl"] ** 2
    Q = pc.scalars["nq"] ** 2
    gi = (pc.elems[:, None] * P + np.arange(P)[None, :]).ravel()
    gq = (pc.elems[:, None] * Q + np.arange(Q)[None, :]).ravel()
    r_g = r_g[:, gi]
    E = pc.scalars["nelem"]
    sc = np.abs(r_g).max() or 1.0
    print(f"{cfg} W={W} R={R} {order}: {E} elements; create_rhs_btp at the IC: max rel diff "
          f"{np.abs(r_m - r_g).max() / sc:.3e}")
    from hnumo import bundle as Bd
    proc = np.concatenate([n.faces for n in pc.fneighbours])

    def cmp(tag, st_m, st_g):
        out = []
        for nm, a, b in zip(("q", "qb", "qp"), st_m, st_g):
            b = b[:, gi, ...]
            d = np.abs(a - b).max() / (np.abs(b).max() or 1.0)
            out.append(f"{nm} {d:.2e}")
        for nm, shp in Bd.FIELDS:
            if shp.endswith("npoin") or shp.endswith("npoin_q"):
                a, b = e.field(nm), eg.field(nm)
                idx = gi if shp.endswith("npoin") else gq
                b = b[..., idx]
                d = np.abs(a - b).max() / (np.abs(b).max() or 1.0)
                if d > 1e-12:
                    out.append(f"{nm} {d:.2e}")
        print(f"  {tag}: " + ", ".join(out), flush=True)

    st_m, st_g = e.state(), eg.state()
    e.btp_bcl_coeffs(st_m[2])
    eg.btp_bcl_coeffs(st_g[2])
    cmp("btp_bcl_coeffs", st_m, st_g)
    # the face coefficients: local face lf is global face pc.faces[lf] (sides exchanged if flipped)
    flip = np.zeros(pc.scalars["nface"], bool)
    flip[np.asarray(pc.flipped, dtype=int)] = True
    isproc = np.zeros(pc.scalars["nface"], bool)
    isproc[proc] = True
    for nm, side_ax in (("Q_uu_dp_edge", None), ("Q_uv_dp_edge", None), ("Q_vv_dp_edge", None), ("H_bcl_edge", None),
                        ("btp_graduv_dpp_face", 1), ("sum_layer_mass_flux_face", None)):
        a, b = e.field(nm), eg.field(nm)[..., pc.faces]
        if side_ax is not None:
            bs = np.swapaxes(b, side_ax, 0)
            bs = np.where(flip, bs[::-1], bs)
            b = np.swapaxes(bs, side_ax, 0)
        d = np.abs(a - b).reshape(-1, a.shape[-1]).max(axis=0) / (np.abs(b).max() or 1.0)
        msg = f"{nm}: processor faces {d[isproc].max():.2e}, others {d[~isproc].max() if (~isproc).any() else 0:.2e}"
        if side_ax is not None:
            for sd in (0, 1):
                dd = np.abs(np.take(a, sd, side_ax) - np.take(b, sd, side_ax)).reshape(-1, a.shape[-1]).max(axis=0)
                msg += f"; side {sd + 1} proc {dd[isproc].max() / (np.abs(b).max() or 1.0):.2e}"
        print("    " + msg, flush=True)
    st_m, st_g = e.state(), eg.state()
    e.ti_barotropic_ssprk(st_m[1], st_m[2])
    eg.ti_barotropic_ssprk(st_g[1], st_g[2])
    cmp("ti_barotropic_ssprk", st_m, st_g)
    st_m, st_g = e.state(), eg.state()
    for nm, f in (("predict", "predict"), ("ti_rk_bcl", "ti_rk_bcl")):
        st_m, st_g = e.state(), eg.state()
        try:
            getattr(e, f)(*st_m)
        except Exception as exc:
            print(f"  {nm}: mirror {exc}")
        getattr(eg, f)(*st_g)
        cmp(nm, st_m, st_g)
    e.close()
    eg.close()


if __name__ == "__main__":
    main()

"""Configurations, static operator tables and initial conditions for the MLSWE engine.

Host-side setup; nothing here is timed.  The reference builds these fields once at
start-up in ``mod_initial_create`` (mod_initial.F90:88-190).  This module restates
that pipeline for the brick mesh of ``mesh.py``:

* metrics at quad points / nodes (metrics_quad.F90:60-126, metrics.F90:113) for an
  affine element, lumped LGL mass ``massinv = 1/jac`` (create_mass.F90:5-39);
* dense per-quad-point tables ``psih, dpsidx, dpsidy, indexq, wjac`` and their nodal
  twins (Tensor_product.F90:1-128) -- used only by the CPU oracle, the HIP engine works
  from the 1-D basis and the per-point metrics;
* initial conditions ``bump``, ``lakeAtrest``, ``double-gyre`` (+ a labelled 3-layer
  double-gyre variant) (initial_conditions.F90:93-416), reference pressure at quad
  points and faces (mod_initial_mlswe.F90:170-277), wave-speed edge coefficients
  (:355-401), bottom topography traces and gradient (:29-120,
  mod_Tensorproduct.F90:57-110), wind stress / Coriolis / implicit Coriolis
  coefficients (mod_initial_mlswe.F90:280-352), SSP(5,3) tables (:582-681).

All arrays are float64 / int32 numpy arrays in Fortran order, with the reference's
dimensions (dead face sub-indices compacted, see mesh.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from .basis import Basis
from .mesh import BrickMesh
from .quadmesh import QuadMesh, read_inp, warped_brick

GRAVITY = 9.806                    # set by every IC and by wind_stress_coriolis (mod_initial_mlswe.F90:306)
PI = math.pi                       # mod_constants pi = pi_trig


# --------------------------------------------------------------------------- configs
CONFIGS = {
    # C1: shipped bump namelist (CI/bump/numo3d.in); 10x10 and 16x16 variants
    "bump10": dict(test_case="bump", nelx=10, nely=10, nop=4, nlayers=2,
                   xdims=(0.0, 2000.0), ydims=(0.0, 2000.0), dt=100.0, dt_btp=1.8,
                   method_visc=0, visc=0.0, botfr=0, cd=0.0, f0=0.0, beta=0.0),
    # (16x16: the 10x10 time steps scaled by the element size, 10/16 -- at dt_btp 1.8 the
    # reference goes unstable, its state NaN after one step)
    "bump16": dict(test_case="bump", nelx=16, nely=16, nop=4, nlayers=2,
                   xdims=(0.0, 2000.0), ydims=(0.0, 2000.0), dt=62.5, dt_btp=1.125,
                   method_visc=0, visc=0.0, botfr=0, cd=0.0, f0=0.0, beta=0.0),
    # C5: lake at rest, well-balanced
    "lake10": dict(test_case="lakeAtrest", nelx=10, nely=10, nop=4, nlayers=2,
                   xdims=(0.0, 2000.0), ydims=(0.0, 2000.0), dt=100.0, dt_btp=1.8,
                   method_visc=0, visc=0.0, botfr=0, cd=0.0, f0=0.0, beta=0.0),
    # C5 at its performance size: the lake at rest on 200x200 elements (the 10x10 steps scaled with
    # the element size; the reference fixture lake200_mpi4m_step1 runs it on 4 Morton ranks)
    "lake200": dict(test_case="lakeAtrest", nelx=200, nely=200, nop=4, nlayers=2,
                    xdims=(0.0, 2000.0), ydims=(0.0, 2000.0), dt=5.0, dt_btp=0.09,
                    method_visc=0, visc=0.0, botfr=0, cd=0.0, f0=0.0, beta=0.0),
    # C2: shipped double-gyre namelist (Examples/double_gyre/numo3d.in), L=2
    "dg25": dict(test_case="double-gyre", nelx=25, nely=25, nop=4, nlayers=2,
                 xdims=(0.0, 2.0e6), ydims=(0.0, 2.0e6), dt=500.0, dt_btp=25.0,
                 method_visc=3, visc=50.0, botfr=1, cd=1.0e-7, f0=0.93e-4, beta=2.0e-11),
    # C2 3-layer performance variant (synthetic interfaces)
    "dg25L3": dict(test_case="double-gyre-3", nelx=25, nely=25, nop=4, nlayers=3,
                   xdims=(0.0, 2.0e6), ydims=(0.0, 2.0e6), dt=500.0, dt_btp=25.0,
                   method_visc=3, visc=50.0, botfr=1, cd=1.0e-7, f0=0.93e-4, beta=2.0e-11),
    # C3: N=7, dt scaled for CFL
    "dg25N7L3": dict(test_case="double-gyre-3", nelx=25, nely=25, nop=7, nlayers=3,
                     xdims=(0.0, 2.0e6), ydims=(0.0, 2.0e6), dt=180.0, dt_btp=9.0,
                     method_visc=3, visc=50.0, botfr=1, cd=1.0e-7, f0=0.93e-4, beta=2.0e-11),
    # method_visc == 1 (quad-point LDG viscosity): not in a shipped namelist
    "bump10q": dict(test_case="bump", nelx=10, nely=10, nop=4, nlayers=2,
                    xdims=(0.0, 2000.0), ydims=(0.0, 2000.0), dt=100.0, dt_btp=1.8,
                    method_visc=1, visc=25.0, botfr=0, cd=0.0, f0=0.0, beta=0.0),
    "dg8L3q": dict(test_case="double-gyre-3", nelx=8, nely=8, nop=4, nlayers=3,
                   xdims=(0.0, 2.0e6), ydims=(0.0, 2.0e6), dt=500.0, dt_btp=25.0,
                   method_visc=1, visc=50.0, botfr=1, cd=1.0e-7, f0=0.93e-4, beta=2.0e-11),
    # ad_mlswe > 0 (implicit vertical shear stress between the layers):
    # not in a shipped namelist; A_D = 1e-2 m^2/s, max_shear_dz 10 m / 50 m
    "bump10s": dict(test_case="bump", nelx=10, nely=10, nop=4, nlayers=2,
                    xdims=(0.0, 2000.0), ydims=(0.0, 2000.0), dt=100.0, dt_btp=1.8,
                    method_visc=0, visc=0.0, botfr=0, cd=0.0, f0=0.0, beta=0.0,
                    ad_mlswe=1.0e-2, max_shear_dz=10.0),
    "dg8L3s": dict(test_case="double-gyre-3", nelx=8, nely=8, nop=4, nlayers=3,
                   xdims=(0.0, 2.0e6), ydims=(0.0, 2.0e6), dt=500.0, dt_btp=25.0,
                   method_visc=3, visc=50.0, botfr=1, cd=1.0e-7, f0=0.93e-4, beta=2.0e-11,
                   ad_mlswe=1.0e-2, max_shear_dz=50.0),
    # f3 (meshes beyond the brick): general bilinear quadrilaterals with mixed edge orientations
    # (hnumo/quadmesh.py; "mesh": ("warp", amplitude, rotate corners) or ("inp", path))
    "qmbump8": dict(test_case="bump", nelx=8, nely=8, nop=4, nlayers=2,
                    xdims=(0.0, 2000.0), ydims=(0.0, 2000.0), dt=100.0, dt_btp=1.8,
                    method_visc=0, visc=0.0, botfr=0, cd=0.0, f0=0.0, beta=0.0, mesh=("warp", 0.15, True)),
    "qmdg8L3": dict(test_case="double-gyre-3", nelx=8, nely=8, nop=4, nlayers=3,
                    xdims=(0.0, 2.0e6), ydims=(0.0, 2.0e6), dt=500.0, dt_btp=25.0,
                    method_visc=3, visc=50.0, botfr=1, cd=1.0e-7, f0=0.93e-4, beta=2.0e-11,
                    mesh=("warp", 0.15, True)),
    # C4: ~1e5 elements, dt scaled for CFL
    "dg316L3": dict(test_case="double-gyre-3", nelx=316, nely=316, nop=4, nlayers=3,
                    xdims=(0.0, 2.0e6), ydims=(0.0, 2.0e6), dt=40.0, dt_btp=2.0,
                    method_visc=3, visc=50.0, botfr=1, cd=1.0e-7, f0=0.93e-4, beta=2.0e-11),
}


def make_config(name: str, **overrides) -> dict:
    cfg = dict(CONFIGS[name])
    cfg.setdefault("kstages", 5)
    cfg.setdefault("ad_mlswe", 0.0)
    cfg.setdefault("max_shear_dz", 0.0)     # mod_input.F90:127
    cfg.setdefault("shear_corrector", 0)    # HNUMO_SHEAR_CORRECTOR_REFERENCE (include/hnumo_engine.h)
    cfg.setdefault("x_boundary", (4, 4))
    cfg.setdefault("y_boundary", (4, 4))
    cfg["name"] = name
    cfg.update(overrides)
    return cfg


def ssprk_coefficients(kstages: int):
    """SSP RK tables (mod_initial_mlswe.F90:582-681, 'rk35' branch)."""
    a = np.zeros((kstages, 3), order="F")
    b = np.zeros(kstages)
    if kstages == 5:
        a[0] = (1.0, 0.0, 0.0); b[0] = 0.377268915331368
        a[1] = (0.0, 1.0, 0.0); b[1] = 0.377268915331368
        a[2] = (0.355909775063326, 0.644090224936674, 0.0); b[2] = 0.242995220537396
        a[3] = (0.367933791638137, 0.632066208361863, 0.0); b[3] = 0.238458932846290
        a[4] = (0.0, 0.762406163401431, 0.237593836598569); b[4] = 0.287632146308408
    elif kstages == 3:
        a[0] = (1.0, 0.0, 0.0); b[0] = 1.0
        a[1] = (3.0 / 4.0, 1.0 / 4.0, 0.0); b[1] = 1.0 / 4.0
        a[2] = (1.0 / 3.0, 2.0 / 3.0, 0.0); b[2] = 2.0 / 3.0
    elif kstages == 2:
        a[0] = (1.0, 0.0, 0.0); b[0] = 1.0
        a[1] = (0.5, 0.5, 0.0); b[1] = 0.5
    elif kstages == 1:
        a[0] = (1.0, 0.0, 0.0); b[0] = 1.0
    else:
        raise ValueError(f"kstages={kstages} not supported")
    return a, b


@dataclass
class Case:
    """Every input of ``ti_rk_bcl`` for one configuration (see include/hnumo_engine.h)."""
    cfg: dict
    basis: Basis
    mesh: BrickMesh
    arrays: dict = field(default_factory=dict)   # name -> np.ndarray (Fortran order)
    scalars: dict = field(default_factory=dict)

    def __getitem__(self, k):
        return self.arrays[k]


def _interp_nodes_to_quad(basis: Basis, nodal_e):
    """Reference-order interpolation nodes->quad (loop m outer, n inner; hi = psiqx(n,iq)*psiqy(m,jq)).

    nodal_e: (nelem, ngl(j), ngl(i)).  Returns (nelem, nq(jq), nq(iq)).
    Restates e.g. mod_initial_mlswe.F90:193-217.
    """
    psiq = basis.psiq
    ngl, nq = basis.ngl, basis.nq
    out = np.zeros((nodal_e.shape[0], nq, nq))
    for jq in range(nq):
        for iq in range(nq):
            acc = np.zeros(nodal_e.shape[0])
            for m in range(ngl):
                for n in range(ngl):
                    hi = psiq[n, iq] * psiq[m, jq]
                    acc = acc + nodal_e[:, m, n] * hi
            out[:, jq, iq] = acc
    return out


def _brick_metrics(A, basis: Basis, mesh: BrickMesh):
    """Metrics of the affine brick (metrics_quad.F90:60-126, metrics.F90:113)."""
    ngl, nq, nelem = basis.ngl, basis.nq, mesh.nelem
    x_ksi, y_eta = 0.5 * mesh.dx, 0.5 * mesh.dy
    xj = x_ksi * y_eta * 1.0 - x_ksi * 0.0 * 0.0 - (0.0 * 0.0 * 1.0 - 0.0 * 0.0 * 0.0) \
        + (0.0 * 0.0 * 0.0 - 0.0 * 0.0 * y_eta)
    ksi_x = (y_eta * 1.0 - 0.0 * 0.0) / xj
    ksi_y = -(0.0 * 1.0 - 0.0 * 0.0) / xj
    eta_x = -(0.0 * 1.0 - 0.0 * 0.0) / xj
    eta_y = (x_ksi * 1.0 - 0.0 * 0.0) / xj
    wq2 = np.outer(basis.wnq, basis.wnq)            # [jq, iq] -> wnqx(i)*wnqy(j)
    wg2 = np.outer(basis.wgl, basis.wgl)
    jacq_e = (basis.wnq[None, :] * basis.wnq[:, None]) * 1.0 * abs(xj)   # [jq, iq]
    jac_e = (basis.wgl[None, :] * basis.wgl[:, None]) * 1.0 * abs(xj)    # [j, i]
    del wq2, wg2
    A["ksiq_x"] = np.full((nq, nq, nelem), ksi_x, order="F")
    A["ksiq_y"] = np.full((nq, nq, nelem), ksi_y, order="F")
    A["etaq_x"] = np.full((nq, nq, nelem), eta_x, order="F")
    A["etaq_y"] = np.full((nq, nq, nelem), eta_y, order="F")
    A["jacq"] = np.asfortranarray(np.broadcast_to(jacq_e.T[:, :, None], (nq, nq, nelem)))
    A["ksi_x"] = np.full((ngl, ngl, nelem), ksi_x, order="F")
    A["ksi_y"] = np.full((ngl, ngl, nelem), ksi_y, order="F")
    A["eta_x"] = np.full((ngl, ngl, nelem), eta_x, order="F")
    A["eta_y"] = np.full((ngl, ngl, nelem), eta_y, order="F")
    A["jac"] = np.asfortranarray(np.broadcast_to(jac_e.T[:, :, None], (ngl, ngl, nelem)))
    # lumped mass: mass(ip) = jac(i,j,e) (one element per DG node), massinv = 1/mass
    A["massinv"] = 1.0 / A["jac"].reshape(-1, order="F")



def build_case(cfg: dict, dense: bool = True) -> Case:
    """Build mesh, tables and ICs.  ``dense`` adds the reference's dense tables (oracle only)."""
    nop, L = cfg["nop"], cfg["nlayers"]
    basis = Basis(nop)
    ngl, nq = basis.ngl, basis.nq
    mspec = cfg.get("mesh")
    if mspec is None:
        mesh = BrickMesh(cfg["nelx"], cfg["nely"], tuple(cfg["xdims"]), tuple(cfg["ydims"]),
                         ngl, nq, tuple(cfg["x_boundary"]), tuple(cfg["y_boundary"]))
        mesh.finalize_face_jacobians(basis.wgl, basis.wnq)
    else:
        # f3: a general conforming quadrilateral grid (hnumo/quadmesh.py)
        if mspec[0] == "warp":
            V, Qd, bc = warped_brick(cfg["nelx"], cfg["nely"], cfg["xdims"], cfg["ydims"], mspec[1], mspec[2],
                                     cfg["x_boundary"][0])
        elif mspec[0] == "inp":
            V, Qd, bc = read_inp(mspec[1])
        else:
            raise ValueError(mspec)
        mesh = QuadMesh(V, Qd, bc, ngl, nq)
    nelem, npoin, npoin_q, nface = mesh.nelem, mesh.npoin, mesh.npoin_q, mesh.nface
    P, Q = ngl * ngl, nq * nq
    A = {}

    if isinstance(mesh, QuadMesh):
        # ---------------- metrics, normals, face Jacobians of a general grid (quadmesh.py)
        G = mesh.geometry(basis)
        for k in ("normal_vector", "normal_vector_q", "jac_face", "jac_faceq"):
            setattr(mesh, k, G.pop(k))
        A.update(G)
        A["massinv"] = 1.0 / A["jac"].reshape(-1, order="F")
    else:
        _brick_metrics(A, basis, mesh)

    # ---------------- mesh arrays
    for k in ("face", "imapl", "imapr", "imapl_q", "imapr_q", "normal_vector", "normal_vector_q", "jac_face",
              "jac_faceq"):
        A[k] = getattr(mesh, k)
    A["psiq"] = np.asfortranarray(basis.psiq)
    A["dpsiq"] = np.asfortranarray(basis.dpsiq)
    A["psi"] = np.asfortranarray(basis.psi)
    A["dpsi"] = np.asfortranarray(basis.dpsi)
    A["wgl"] = basis.wgl.copy()
    A["wnq"] = basis.wnq.copy()

    # ---------------- dense tables (Tensor_product.F90:50-126), oracle only
    if dense:
        _dense_tables(A, basis, mesh)

    # ---------------- initial conditions (initial_conditions.F90)
    coord = mesh.node_coords(basis.xgl)
    x, y = coord[0], coord[1]
    xmin, xmax, ymin, ymax = x.min(), x.max(), y.min(), y.max()
    tc = cfg["test_case"]
    z_int = np.zeros((npoin, L + 1), order="F")
    alpha = np.zeros(L)
    tau_wind_df = np.zeros((2, npoin), order="F")
    Ly = cfg["ydims"][1] - cfg["ydims"][0]
    if tc == "bump":
        H_bot = 40.0
        zbot_df = np.full(npoin, -H_bot)
        for k in range(L + 1):
            z_int[:, k] = -(k) * H_bot / float(L)
        xm = 0.5 * (xmax + xmin)
        yl = 0.5 * (ymax + ymin)
        Lb, amp = 250.0, 1.0
        r = np.sqrt((x - xm) ** 2 + (y - yl) ** 2)
        msk = r < Lb
        z_int[msk, 1] = z_int[msk, 1] + 0.5 * amp * (1.0 + np.cos(PI * r[msk] / Lb))
        alpha[0] = 0.9737e-3
        alpha[1] = 0.9735e-3
    elif tc == "lakeAtrest":
        H_bot = 40.0
        zbot_df = np.full(npoin, -H_bot)
        xm = 0.5 * (cfg["xdims"][0] + cfg["xdims"][1])
        yl = 0.5 * (cfg["ydims"][0] + cfg["ydims"][1])
        Lb = 250.0
        r = np.sqrt((x - xm) ** 2 + (y - yl) ** 2)
        msk = r < Lb
        zbot_df[msk] = zbot_df[msk] + 3.0 * (1.0 + np.cos(PI * r[msk] / Lb))
        for k in range(L + 1):
            if L < 5:
                z_int[:, k] = -(k) * H_bot / float(L)
            else:
                z_int[:, k] = -(k) * 32 / float(L - 1)
                z_int[:, L] = -H_bot
        rho_0 = 1027.01037
        alpha[0] = 1.0 / rho_0
        for k in range(2, L + 1):
            alpha[k - 1] = 1.0 / (rho_0 + k * 0.2110 / float(L))
    elif tc in ("double-gyre", "double-gyre-3"):
        H_bot = 9928.0
        zbot_df = np.full(npoin, -H_bot)
        if tc == "double-gyre":
            assert L == 2, "shipped double-gyre IC is 2-layer (initial_conditions.F90:171-191)"
            z_int[:, 1] = -1489.5
            z_int[:, 2] = -H_bot
            alpha[0] = 9.7370e-04
            alpha[1] = 9.7350e-04
        else:
            # labelled 3-layer variant: interfaces 0, -500, -1489.5, -9928
            assert L == 3
            z_int[:, 1] = -500.0
            z_int[:, 2] = -1489.5
            z_int[:, 3] = -H_bot
            alpha[0] = 9.7370e-04
            alpha[1] = 9.7360e-04
            alpha[2] = 9.7350e-04
        tau_wind_df[0] = -0.1 * np.cos(2.0 * PI * y / Ly)
    else:
        raise ValueError(tc)
    # interfaces not below the bottom (initial_conditions.F90:310-317)
    for k in range(L + 1):
        z_int[:, k] = np.maximum(zbot_df, z_int[:, k])
    g = GRAVITY
    pbprime_df = np.zeros(npoin)
    for k in range(L):
        pbprime_df = pbprime_df + (g / alpha[k]) * (z_int[:, k] - z_int[:, k + 1])

    # pbprime at quad points / faces (interpolate_pbprime_init, mod_initial_mlswe.F90:170-277)
    pbq = _interp_nodes_to_quad(basis, pbprime_df.reshape(nelem, ngl, ngl))
    pbprime = pbq.reshape(-1)
    pbprime_face = _quad_face_traces(mesh, pbprime)
    pbprime_df_face = _node_face_traces(mesh, pbprime_df)
    one_over_pbprime_edge = np.zeros((nq, nface), order="F")
    pos = pbprime_face[0] > 0.0
    one_over_pbprime_edge[pos] = 1.0 / pbprime_face[0][pos]
    one_over_pbprime_df = np.where(pbprime_df > 0.0, 1.0 / np.where(pbprime_df > 0, pbprime_df, 1.0), 0.0)
    one_over_pbprime = np.where(pbprime > 0.0, 1.0 / np.where(pbprime > 0, pbprime, 1.0), 0.0)

    # layer state (initial_conditions.F90:378-416); one_plus_eta_temp starts at zero
    q_df = np.zeros((3, npoin, L), order="F")
    qprime_df = np.zeros((3, npoin, L), order="F")
    ope = np.zeros(npoin)
    for k in range(L):
        q_df[0, :, k] = (g / alpha[k]) * (z_int[:, k] - z_int[:, k + 1])
        ope = ope + q_df[0, :, k] / pbprime_df
    for k in range(L):
        qprime_df[0, :, k] = q_df[0, :, k] / ope
    # u_df = v_df = 0 -> q_df(2:3) = 0
    qb_df = np.zeros((4, npoin), order="F")
    for k in range(L):
        qb_df[0] = qb_df[0] + q_df[0, :, k]
        qb_df[2] = qb_df[2] + q_df[1, :, k]
        qb_df[3] = qb_df[3] + q_df[2, :, k]
    qb_df[1] = qb_df[0] - pbprime_df
    for k in range(L):
        qprime_df[1, :, k] = q_df[1, :, k] / q_df[0, :, k] - qb_df[2] / qb_df[0]
        qprime_df[2, :, k] = q_df[2, :, k] / q_df[0, :, k] - qb_df[3] / qb_df[0]

    # edge wave-speed coefficients (mod_initial_mlswe.F90:355-401)
    cm = np.sqrt(alpha[L - 1] * pbprime_face[1])
    cp = np.sqrt(alpha[L - 1] * pbprime_face[0])
    ok = (cm > 0.0) | (cp > 0.0)
    den = np.where(ok, cm + cp, 1.0)
    z = np.zeros((nq, nface), order="F")
    coeff_pbpert_L = np.where(ok, cm / den, z)
    coeff_pbpert_R = np.where(ok, cp / den, z)
    coeff_pbub_LR = np.where(ok, 1.0 / den, z)
    coeff_mass_pbub_L = np.where(ok, cp / den, z)
    coeff_mass_pbub_R = np.where(ok, cm / den, z)
    coeff_mass_pbpert_LR = np.where(ok, cm * cp / den, z)

    # bottom topography (bot_topo_derivatives, mod_initial_mlswe.F90:29-120; zbot starts at 0)
    zbot = _interp_nodes_to_quad(basis, zbot_df.reshape(nelem, ngl, ngl)).reshape(-1)
    zbot_face = _quad_face_traces(mesh, zbot)
    grad_zbot_quad = _gradient_quad(basis, A, zbot_df, nelem)

    # wind stress + Coriolis (mod_initial_mlswe.F90:280-352)
    dt = float(cfg["dt"])
    N_btp = int(math.ceil(dt / cfg["dt_btp"]))
    dt_btp = dt / float(N_btp)
    ym = 0.5 * cfg["ydims"][1]
    coriolis_df = cfg["f0"] + cfg["beta"] * (y - ym)
    cor_e = coriolis_df.reshape(nelem, ngl, ngl)
    tw1 = tau_wind_df[0].reshape(nelem, ngl, ngl)
    tw2 = tau_wind_df[1].reshape(nelem, ngl, ngl)
    coriolis_quad = _interp_nodes_to_quad(basis, cor_e).reshape(-1)
    tau_wind = np.zeros((2, npoin_q), order="F")
    tau_wind[0] = _interp_nodes_to_quad(basis, tw1).reshape(-1)
    tau_wind[1] = _interp_nodes_to_quad(basis, tw2).reshape(-1)
    fdt_bcl = dt * coriolis_df
    fdt2_bcl = 0.5 * fdt_bcl
    a_bcl = 1.0 / (1.0 + fdt2_bcl ** 2)
    b_bcl = fdt2_bcl / (1.0 + fdt2_bcl ** 2)
    ssprk_a, ssprk_beta = ssprk_coefficients(cfg["kstages"])

    A.update(dict(
        pbprime=pbprime, pbprime_df=pbprime_df, one_over_pbprime=one_over_pbprime,
        one_over_pbprime_df=one_over_pbprime_df, pbprime_face=pbprime_face,
        pbprime_df_face=pbprime_df_face, one_over_pbprime_edge=one_over_pbprime_edge,
        coeff_pbpert_L=coeff_pbpert_L, coeff_pbpert_R=coeff_pbpert_R, coeff_pbub_LR=coeff_pbub_LR,
        coeff_mass_pbub_L=coeff_mass_pbub_L, coeff_mass_pbub_R=coeff_mass_pbub_R,
        coeff_mass_pbpert_LR=coeff_mass_pbpert_LR, alpha=alpha, tau_wind=tau_wind,
        coriolis_quad=coriolis_quad, grad_zbot_quad=grad_zbot_quad, zbot_df=zbot_df,
        zbot_face=zbot_face, fdt2_bcl=fdt2_bcl, a_bcl=a_bcl, b_bcl=b_bcl,
        ssprk_a=ssprk_a, ssprk_beta=ssprk_beta, coord=coord,
        q_df=q_df, qb_df=qb_df, qprime_df=qprime_df,
    ))
    for k, v in list(A.items()):
        if v.dtype != np.int32:
            A[k] = np.asfortranarray(v, dtype=np.float64)
        else:
            A[k] = np.asfortranarray(v)
    S = dict(nelem=nelem, npoin=npoin, npoin_q=npoin_q, nface=nface, ngl=ngl, nq=nq, nlayers=L,
             kstages=cfg["kstages"], N_btp=N_btp, dt=dt, dt_btp=dt_btp,
             method_visc=cfg["method_visc"], visc=float(cfg["visc"]), botfr=cfg["botfr"],
             cd=float(cfg["cd"]), ad=float(cfg["ad_mlswe"]), gravity=g,
             max_shear_dz=float(cfg["max_shear_dz"]), shear_corrector=int(cfg["shear_corrector"]))
    return Case(cfg=cfg, basis=basis, mesh=mesh, arrays=A, scalars=S)


# ------------------------------------------------------------------------ helpers
def _quad_face_traces(mesh: BrickMesh, fq):
    """(2,nq,nface) traces of a quad-point field via imapl_q/imapr_q (mod_initial_mlswe.F90:219-251)."""
    nq, Q = mesh.nq, mesh.nqq
    el = mesh.face[6].astype(np.int64) - 1
    er = mesh.face[7].astype(np.int64)
    il, jl = mesh.imapl_q[0].astype(np.int64) - 1, mesh.imapl_q[1].astype(np.int64) - 1
    Il = el[None, :] * Q + jl * nq + il
    out = np.zeros((2, nq, mesh.nface), order="F")
    out[0] = fq[Il]
    inter = er > 0
    ir, jr = mesh.imapr_q[0].astype(np.int64) - 1, mesh.imapr_q[1].astype(np.int64) - 1
    Ir = (np.maximum(er, 1) - 1)[None, :] * Q + jr * nq + ir
    out[1] = np.where(inter[None, :], fq[np.where(inter[None, :], Ir, 0)], out[0])
    return out


def _node_face_traces(mesh: BrickMesh, fn):
    """(2,ngl,nface) traces of a nodal field via imapl/imapr (mod_initial_mlswe.F90:253-274)."""
    ngl, P = mesh.ngl, mesh.npts
    el = mesh.face[6].astype(np.int64) - 1
    er = mesh.face[7].astype(np.int64)
    il, jl = mesh.imapl[0].astype(np.int64) - 1, mesh.imapl[1].astype(np.int64) - 1
    Il = el[None, :] * P + jl * ngl + il
    out = np.zeros((2, ngl, mesh.nface), order="F")
    out[0] = fn[Il]
    inter = er > 0
    ir, jr = mesh.imapr[0].astype(np.int64) - 1, mesh.imapr[1].astype(np.int64) - 1
    Ir = (np.maximum(er, 1) - 1)[None, :] * P + jr * ngl + ir
    out[1] = np.where(inter[None, :], fn[np.where(inter[None, :], Ir, 0)], out[0])
    return out


def _gradient_quad(basis: Basis, A, q_df, nelem):
    """compute_gradient_quad (mod_Tensorproduct.F90:57-110), reference loop order."""
    ngl, nq = basis.ngl, basis.nq
    psiq, dpsiq = basis.psiq, basis.dpsiq
    qe = q_df.reshape(nelem, ngl, ngl)
    ex = A["ksiq_x"].reshape(nq, nq, nelem, order="F")
    ey = A["ksiq_y"].reshape(nq, nq, nelem, order="F")
    nx = A["etaq_x"].reshape(nq, nq, nelem, order="F")
    ny = A["etaq_y"].reshape(nq, nq, nelem, order="F")
    out = np.zeros((2, nelem, nq, nq))
    for jq in range(nq):
        for iq in range(nq):
            e_x, e_y, n_x, n_y = ex[iq, jq], ey[iq, jq], nx[iq, jq], ny[iq, jq]
            g1 = np.zeros(nelem)
            g2 = np.zeros(nelem)
            for m in range(ngl):
                for n in range(ngl):
                    h_e = dpsiq[n, iq] * psiq[m, jq]
                    h_n = psiq[n, iq] * dpsiq[m, jq]
                    g1 = g1 + (h_e * e_x + h_n * n_x) * qe[:, m, n]
                    g2 = g2 + (h_e * e_y + h_n * n_y) * qe[:, m, n]
            out[0, :, jq, iq] = g1
            out[1, :, jq, iq] = g2
    return np.asfortranarray(out.reshape(2, -1))


def _dense_tables(A, basis: Basis, mesh: BrickMesh):
    """psih/dpsidx/dpsidy/indexq/wjac and nodal twins (Tensor_product.F90:50-126)."""
    ngl, nq, nelem = basis.ngl, basis.nq, mesh.nelem
    P, Q = ngl * ngl, nq * nq
    psiq, dpsiq, psi, dpsi = basis.psiq, basis.dpsiq, basis.psi, basis.dpsi
    ex = A["ksiq_x"].reshape(nq, nq, nelem, order="F")
    ey = A["ksiq_y"].reshape(nq, nq, nelem, order="F")
    nx = A["etaq_x"].reshape(nq, nq, nelem, order="F")
    ny = A["etaq_y"].reshape(nq, nq, nelem, order="F")
    psih = np.zeros((P, nelem, nq, nq))
    dpdx = np.zeros((P, nelem, nq, nq))
    dpdy = np.zeros((P, nelem, nq, nq))
    idxq = np.zeros((P, nelem, nq, nq), dtype=np.int32)
    base = np.arange(nelem) * P
    for jq in range(nq):
        for iq in range(nq):
            ip = 0
            for m in range(ngl):
                for n in range(ngl):
                    idxq[ip, :, jq, iq] = base + m * ngl + n + 1
                    psih[ip, :, jq, iq] = psiq[n, iq] * psiq[m, jq]
                    h_e = dpsiq[n, iq] * psiq[m, jq]
                    h_n = psiq[n, iq] * dpsiq[m, jq]
                    dpdx[ip, :, jq, iq] = h_e * ex[iq, jq] + h_n * nx[iq, jq]
                    dpdy[ip, :, jq, iq] = h_e * ey[iq, jq] + h_n * ny[iq, jq]
                    ip += 1
    A["psih"] = np.asfortranarray(psih.reshape(P, -1))
    A["dpsidx"] = np.asfortranarray(dpdx.reshape(P, -1))
    A["dpsidy"] = np.asfortranarray(dpdy.reshape(P, -1))
    A["indexq"] = np.asfortranarray(idxq.reshape(P, -1))
    A["wjac"] = A["jacq"].reshape(-1, order="F").copy()
    # nodal twins (Tensor_product.F90:89-124)
    exn = A["ksi_x"].reshape(ngl, ngl, nelem, order="F")
    eyn = A["ksi_y"].reshape(ngl, ngl, nelem, order="F")
    nxn = A["eta_x"].reshape(ngl, ngl, nelem, order="F")
    nyn = A["eta_y"].reshape(ngl, ngl, nelem, order="F")
    ddx = np.zeros((P, nelem, ngl, ngl))
    ddy = np.zeros((P, nelem, ngl, ngl))
    idxd = np.zeros((P, nelem, ngl, ngl), dtype=np.int32)
    for jq in range(ngl):
        for iq in range(ngl):
            ip = 0
            for m in range(ngl):
                for n in range(ngl):
                    idxd[ip, :, jq, iq] = base + m * ngl + n + 1
                    h_e = dpsi[n, iq] * psi[m, jq]
                    h_n = psi[n, iq] * dpsi[m, jq]
                    ddx[ip, :, jq, iq] = h_e * exn[iq, jq] + h_n * nxn[iq, jq]
                    ddy[ip, :, jq, iq] = h_e * eyn[iq, jq] + h_n * nyn[iq, jq]
                    ip += 1
    A["dpsidx_df"] = np.asfortranarray(ddx.reshape(P, -1))
    A["dpsidy_df"] = np.asfortranarray(ddy.reshape(P, -1))
    A["index_df"] = np.asfortranarray(idxd.reshape(P, -1))
    A["wjac_df"] = A["jac"].reshape(-1, order="F").copy()

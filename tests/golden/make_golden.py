"""Generates the golden vectors in tests/golden/ by running the REFERENCE Fortran hot path
(oracle/_ref/ref_driver, built from /root/reference/src by oracle/build_ref.sh) on the
inputs that h-numo_amd/hnumo/case.py builds.  Run in the build container only:

    python tests/golden/make_golden.py

Each fixture stores the sha256 of the input bundle, so a change to the setup code is
detected instead of silently comparing against stale outputs.
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "h-numo_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))
import oracle as O  # noqa: E402
from hnumo import bundle as B  # noqa: E402
from hnumo.case import build_case, make_config  # noqa: E402
from util import partition_inputs_sha256  # noqa: E402

# (fixture name, config, mode, nsteps, node stride for the stored state)
GOLDEN = [
    ("bump10_rhs", "bump10", "rhs", 1, 1),
    ("bump10_btp", "bump10", "btp", 1, 1),
    ("bump10_step2", "bump10", "step", 2, 1),
    ("lake10_step1", "lake10", "step", 1, 1),
    ("dg25_step1", "dg25", "step", 1, 7),
    ("dg25L3_step1", "dg25L3", "step", 1, 7),
    ("bump10q_step1", "bump10q", "step", 1, 1),
    ("dg8L3q_step1", "dg8L3q", "step", 1, 1),
    # C3 at N=7 (8x8 elements: the 25x25 bundle's dense tables are ~0.5 GB)
    ("dg8N7L3_step1", "dg25N7L3", "step", 1, 1, dict(nelx=8, nely=8)),
    # C3 at its stated size (25x25, N=7), strided like dg25_step1
    ("dg25N7L3_step1", "dg25N7L3", "step", 1, 7),
    # branches the shipped namelists do not exercise: quadratic drag + no-slip
    # walls, linear drag + beta plane + mixed walls, 3-layer lake, quad-point LDG + no-slip
    ("bump10_b2ns_step1", "bump10", "step", 1, 1,
     dict(botfr=2, cd=1e-3, visc=25.0, method_visc=3, y_boundary=(2, 2))),
    ("bump10_mixed_step1", "bump10", "step", 1, 1,
     dict(botfr=1, cd=1e-7, f0=1e-4, beta=1e-11, x_boundary=(2, 4))),
    ("lake10L3_step1", "lake10", "step", 1, 1, dict(nlayers=3)),
    ("bump10q_ns_step1", "bump10q", "step", 1, 1, dict(y_boundary=(2, 2), botfr=2, cd=1e-3)),
    ("dg8L3q_mixed_step1", "dg8L3q", "step", 1, 1, dict(x_boundary=(2, 4))),
    # f3: general bilinear quadrilaterals, neighbours along shared edges in both directions
    ("qmbump8_step2", "qmbump8", "step", 2, 1),
    ("qmdg8L3_step1", "qmdg8L3", "step", 1, 1),
    # C1 at its stated size (~256 elements)
    ("bump16_step1", "bump16", "step", 1, 1),
    # ad_mlswe > 0: the predictor (ref_driver mode 4, momentum_mass with the implicit vertical
    # shear stress); the harness zero-fills rhs_layer_shear_stress's never-assigned tau_u(nlayers+1)
    # as the reference's -finit-real=zero build does (oracle/zero_init_wrap.c)
    ("bump10s_predict", "bump10s", "predict", 1, 1),
    ("dg8L3s_predict", "dg8L3s", "predict", 1, 1),
]
FIELDS_KEPT = ["ope_ave", "H_ave", "Qu_ave", "btp_mass_flux_ave", "uvb_face_ave", "H_face_ave",
               "graduvb_ave", "Q_uu_dp", "H_bcl_edge", "btp_graduv_dpp_face"]


def state_sha256(a) -> str:
    """sha256 of a state array's float64 values in C order (the tests hash the engine's the same way)."""
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def bundle_hash(case, mode, nsteps):
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "b.bin")
        B.write_bundle(p, case, mode, nsteps)
        return hashlib.sha256(open(p, "rb").read()).hexdigest()


# Multi-rank: the reference run under mpiexec on a processor-face partition (hnumo/facepart.py;
# the reference's own halo exchange over MPI).  (name, config, overrides, nranks, order, nsteps)
GOLDEN_MPI = [
    ("bump10_mpi3m_step2", "bump10", {}, 3, "morton", 2),
    ("lake10_mpi2b_step1", "lake10", {}, 2, "block", 1),
    ("dg8L3_mpi2b_step2", "dg8L3q", dict(method_visc=3), 2, "block", 2),
    ("dg8L3_mpi4m_step2", "dg8L3q", dict(method_visc=3), 4, "morton", 2),
    # method_visc == 1: the quad-point LDG fluxes cross the processor faces every stage
    # (create_communicator_quad) and every baroclinic Laplacian (bcl_create_communicator)
    ("bump10q_mpi2b_step1", "bump10q", {}, 2, "block", 1),
    ("dg8L3q_mpi4m_step2", "dg8L3q", {}, 4, "morton", 2),
    # C5 (lake at rest) on 4 ranks
    ("lake10_mpi4m_step2", "lake10", {}, 4, "morton", 2),
    # the BASELINE configs at their stated sizes (VERDICT r03 "next" 1), each rank's state stored
    # at a node stride (the dense tables are built per rank: add_dense_tables):
    # C5: lake at rest 200x200 on 4 Morton ranks (dt scaled with the element size, test_lake_gpu.py)
    ("lake200_mpi4m_step1", "lake10", dict(nelx=200, nely=200, dt=5.0, dt_btp=0.09), 4, "morton", 1, 61),
    # C4: double gyre 316x316 on the 4x2 block partition of the 8-GPU metric
    ("dg316L3_mpi8b_step1", "dg316L3", {}, 8, "block", 1, 97),
]


def make_mpi(only=None):
    from hnumo.facepart import add_dense_tables, face_partition
    for entry in GOLDEN_MPI:
        name, cfg, ov, R, order, nsteps = entry[:6]
        stride = entry[6] if len(entry) > 6 else 1
        if only and name not in only:
            continue
        if stride == 1:
            case = build_case(make_config(cfg, **ov))
            parts = [face_partition(case, R, r, order) for r in range(R)]
        else:
            case = build_case(make_config(cfg, **ov), dense=False)
            parts = [add_dense_tables(face_partition(case, R, r, order)) for r in range(R)]
            del case
        outs = O.run_reference_mpi(parts, "step", nsteps)
        keep = {"config": np.array(cfg), "overrides": np.array(json.dumps(ov)), "nranks": np.array(R),
                "order": np.array(order), "nsteps": np.array(nsteps), "mode": np.array("step"),
                "stride": np.array(stride)}
        for r, (pc, o) in enumerate(zip(parts, outs)):
            keep[f"bundle_sha256_r{r}"] = np.array(bundle_hash(pc, "step", nsteps))
            keep[f"nelem_r{r}"] = np.array(pc.scalars["nelem"])
            keep[f"inputs_sha256_r{r}"] = np.array(partition_inputs_sha256(pc))
            for k in ("q_df", "qb_df", "qprime_df"):
                keep[f"{k}_r{r}"] = o[k][:, ::stride, ...]
                # the whole array, bit for bit, in 32 bytes (state_sha256)
                keep[f"{k}_sha256_r{r}"] = np.array(state_sha256(o[k]))
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **keep)
        print(name, os.path.getsize(path))


def add_mpi_inputs_hash(only):
    """Adds inputs_sha256_r* to existing strided multi-rank fixtures (no reference run)."""
    from hnumo.facepart import face_partition
    for entry in GOLDEN_MPI:
        name, cfg, ov, R, order = entry[:5]
        if name not in only:
            continue
        path = os.path.join(HERE, name + ".npz")
        keep = dict(np.load(path, allow_pickle=False))
        case = build_case(make_config(cfg, **ov), dense=False)
        for r in range(R):
            keep[f"inputs_sha256_r{r}"] = np.array(partition_inputs_sha256(face_partition(case, R, r, order)))
        np.savez_compressed(path, **keep)
        print(name, os.path.getsize(path))


# a18: the reference's own set-up routines (ref_driver mode 6: initial_conditions,
# compute_reference_edge_variables, bot_topo_derivatives, compute_gradient_quad,
# wind_stress_coriolis, ssprk_coefficients) -- every table hnumo/case.py builds.
# (name, config, overrides, stride of the stored flattened arrays)
GOLDEN_SETUP = [
    ("setup_bump10", "bump10", {}, 1),
    ("setup_lake10L3", "lake10", dict(nlayers=3), 1),
    ("setup_dg25", "dg25", {}, 5),
    ("setup_dg8N7", "dg25", dict(nelx=8, nely=8, nop=7, dt=180.0, dt_btp=9.0), 2),
    ("setup_qmbump8", "qmbump8", {}, 1),
]


def make_setup(only=None):
    for name, cfg, ov, stride in GOLDEN_SETUP:
        if only and name not in only:
            continue
        case = build_case(make_config(cfg, **ov))
        out = O.run_reference(case, "setup", 1)
        keep = {"config": np.array(cfg), "overrides": np.array(json.dumps(ov)), "stride": np.array(stride),
                "bundle_sha256": np.array(bundle_hash(case, "setup", 1))}
        for k, _ in B.SETUP_OUT:
            keep["ref_" + k] = np.asarray(out[k]).reshape(-1, order="F")[::stride]
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **keep)
        print(name, os.path.getsize(path))


# f3: the reference's own geometry routines (ref_driver mode 7: metrics, metrics_quad,
# create_normals, create_normals_quad) on the node coordinates and faces hnumo/quadmesh.py builds
GOLDEN_GEOM = [
    ("geom_qmbump8", "qmbump8", {}),
]


def make_geom(only=None):
    for name, cfg, ov in GOLDEN_GEOM:
        if only and name not in only:
            continue
        case = build_case(make_config(cfg, **ov))
        out = O.run_reference(case, "geom", 1)
        keep = {"config": np.array(cfg), "overrides": np.array(json.dumps(ov)),
                "bundle_sha256": np.array(bundle_hash(case, "geom", 1))}
        for k, _ in B.GEOM_OUT:
            keep["ref_" + k] = np.asarray(out[k])
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **keep)
        print(name, os.path.getsize(path))


def overrides_of(g) -> dict:
    """Config overrides stored in a fixture (JSON; lists back to tuples)."""
    if "overrides" not in g:
        return {}
    return {k: tuple(v) if isinstance(v, list) else v for k, v in json.loads(str(g["overrides"])).items()}


def main(only=None):
    for entry in GOLDEN:
        name, cfg, mode, nsteps, stride = entry[:5]
        ov = entry[5] if len(entry) > 5 else {}
        if only and name not in only:
            continue
        case = build_case(make_config(cfg, **ov))
        out = O.run_reference(case, mode, nsteps)
        keep = {"bundle_sha256": np.array(bundle_hash(case, mode, nsteps)), "stride": np.array(stride),
                "mode": np.array(mode), "nsteps": np.array(nsteps), "config": np.array(cfg),
                "overrides": np.array(json.dumps(ov))}
        if mode == "rhs":
            keep["rhs"] = out["rhs"]
        keep["qb_df"] = out["qb_df"][:, ::stride]
        if mode in ("step", "predict"):
            keep["q_df"] = out["q_df"][:, ::stride, :]
            keep["qprime_df"] = out["qprime_df"][:, ::stride, :]
        if stride > 1:
            for k in ("q_df", "qb_df", "qprime_df"):
                if k in keep:
                    keep[k + "_sha256"] = np.array(state_sha256(out[k]))
        for f in FIELDS_KEPT:
            a = out[f]
            keep["field_" + f] = a.reshape(-1, order="F")[::stride]
        for k in ("ref_xgl", "ref_wgl", "ref_xnq", "ref_wnq", "ref_psiq", "ref_dpsiq", "ref_dpsi"):
            keep[k] = out[k]
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **keep)
        print(name, os.path.getsize(path))


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "mpi":
        make_mpi(args[1:] or None)
    elif args and args[0] == "mpi_inputs":
        add_mpi_inputs_hash(args[1:])
    elif args and args[0] == "setup":
        make_setup(args[1:] or None)
    elif args and args[0] == "geom":
        make_geom(args[1:] or None)
    else:
        main(args or None)

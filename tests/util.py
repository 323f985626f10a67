import numpy as np


def rel(a, b):
    """Normwise relative difference max|a-b| / max|b| (0 if both are zero)."""
    a = np.asarray(a)
    b = np.asarray(b)
    d = np.abs(a - b).max() if a.size else 0.0
    s = np.abs(b).max() if b.size else 0.0
    return float(d / s) if s > 0 else float(d)


def layer_mass(case, q_df):
    """compute_conserved (compute_conserved.F90:7-45) of h = (alpha_k/g) dp_k per layer
    (diagnostics.F90:40-45); psih_df is the identity at LGL nodes."""
    A, S = case.arrays, case.scalars
    w = A["jac"].reshape(-1, order="F")
    return np.array([np.sum(w * (A["alpha"][k] / S["gravity"]) * q_df[0, :, k]) for k in range(S["nlayers"])])


def overrides_of(g) -> dict:
    """Config overrides stored in a golden fixture (JSON; lists back to tuples)."""
    import json
    if "overrides" not in g:
        return {}
    return {k: tuple(v) if isinstance(v, list) else v for k, v in json.loads(str(g["overrides"])).items()}


def state_sha256(a) -> str:
    """sha256 of a state array's float64 values in C order (tests/golden/make_golden.py hashes the
    reference's arrays the same way): whole-state bitwise parity for fixtures that store a strided
    sample only."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


DENSE_KEYS = ("psih", "dpsidx", "dpsidy", "indexq", "wjac", "dpsidx_df", "dpsidy_df", "index_df", "wjac_df")


def partition_inputs_sha256(pc) -> str:
    """sha256 over a rank's input arrays (sorted names, float64/int32 values in Fortran order) and
    its halo lists, without the dense tables (built from the same element metrics by
    hnumo.facepart.add_dense_tables).  The input-currency check of the fixtures whose full
    reference bundles are too large to rebuild in the CPU suite (C4, C5 at their stated sizes)."""
    import hashlib
    from hnumo.facepart import halo_lists
    h = hashlib.sha256()
    for k in sorted(pc.arrays):
        if k in DENSE_KEYS:
            continue
        a = np.asarray(pc.arrays[k])
        h.update(k.encode())
        h.update(np.asarray(a, dtype=a.dtype.newbyteorder("<")).ravel(order="F").tobytes())
    for a in halo_lists(pc):
        h.update(np.asarray(a, dtype="<i4").tobytes())
    for k in sorted(pc.scalars):
        h.update(f"{k}={pc.scalars[k]!r};".encode())
    return h.hexdigest()

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

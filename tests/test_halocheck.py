"""CPU tests of bench.py's multi-GPU halo check (hnumo/halocheck.py): the owned-part / global
slice bookkeeping it compares through, on ghost-element and processor-face partitions."""
import numpy as np
import pytest


@pytest.mark.parametrize("kind", ["ghost", "faces"])
def test_global_slice_inverts_gather(kind):
    from hnumo import halocheck as HC
    from hnumo.case import build_case, make_config
    from hnumo.facepart import face_partition
    from hnumo.partition import gather_owned, partition
    g = build_case(make_config("bump10"), dense=False)
    rng = np.random.default_rng(0)
    gstate = tuple(np.asfortranarray(rng.standard_normal(np.shape(g.arrays[k])))
                   for k in ("q_df", "qb_df", "qprime_df"))
    R = 4
    parts = [partition(g, R, r) if kind == "ghost" else face_partition(g, R, r, "morton") for r in range(R)]
    for k, name in enumerate(("q_df", "qb_df", "qprime_df")):
        local = [(pc, HC.global_slice(pc, gstate)[k]) for pc in parts]
        if kind == "ghost":
            back = gather_owned(local, name, g)
        else:
            from hnumo.facepart import gather_faces_state
            back = gather_faces_state(local, name, g)
        assert np.array_equal(back, gstate[k])
    for pc in parts:
        own = HC.owned(pc, HC.global_slice(pc, gstate))
        same, rel = HC.compare(own, HC.global_slice(pc, gstate))
        assert same and rel == 0.0


def test_compare_reports_difference():
    from hnumo import halocheck as HC
    a = (np.ones((3, 10, 2)), np.ones((4, 10)), np.ones((3, 10, 2)))
    b = (a[0].copy(), a[1].copy(), a[2].copy())
    b[1][2, 3] = 1.0 + 1e-15
    same, rel = HC.compare(a, b)
    assert not same and 0 < rel < 1e-14

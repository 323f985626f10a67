"""CPU checks of bench.py's host logic: the C5 performance config, the self-neighbour contract of
--emulate, and the command line (no GPU work)."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "h-numo_amd"))


def test_lake200_is_the_c5_fixture_configuration():
    """bench.py --config lake200 runs exactly the configuration the C5 reference fixture pins
    (tests/golden/make_golden.py: lake10 at 200x200, dt 5 s, dt_btp 0.09 s)."""
    from hnumo.case import make_config
    a = make_config("lake200")
    b = make_config("lake10", nelx=200, nely=200, dt=5.0, dt_btp=0.09)
    a.pop("name"), b.pop("name")
    assert a == b


def test_self_neighbour_lists_every_processor_face_once_under_rank_0():
    """facepart.self_neighbour (bench.py --emulate): per_peer keeps the real rank's per-neighbour
    lists (C4/8 rank 1 of the 4x2 blocks: neighbours 0, 2, 5), each addressed to rank 0 itself, in
    the same order and sizes; one-list mode merges them.  Every processor face is listed once."""
    from hnumo.case import build_case, make_config
    from hnumo.facepart import face_partition, halo_lists, self_neighbour
    g = build_case(make_config("dg8L3q"), dense=False)
    pc = face_partition(g, 8, 1, "block")
    assert [n.rank for n in pc.fneighbours] == [0, 2, 5]
    sizes = [n.faces.size for n in pc.fneighbours]
    faces = np.concatenate([n.faces for n in pc.fneighbours])
    sn = self_neighbour(face_partition(g, 8, 1, "block"))
    assert sn.nranks == 1 and sn.rank == 0
    assert [n.rank for n in sn.fneighbours] == [0, 0, 0] and [n.faces.size for n in sn.fneighbours] == sizes
    nbh_proc, num, lst, _ = halo_lists(sn)
    assert nbh_proc.tolist() == [1, 1, 1] and num.tolist() == sizes and np.array_equal(lst - 1, faces)
    one = self_neighbour(face_partition(g, 8, 1, "block"), per_peer=False)
    assert len(one.fneighbours) == 1 and np.array_equal(one.fneighbours[0].faces, faces)
    assert len(np.unique(faces)) == faces.size


def test_self_neighbour_mirrors_the_processor_faces_statics():
    """The mirror's side 2 is side 1 (the face receives its own traces): side-2 bathymetry statics
    copied from side 1 and the edge coefficients of mod_initial_mlswe.F90:355-401 with c_- = c_+ --
    on every processor face and nowhere else."""
    from hnumo.case import build_case, make_config
    from hnumo.facepart import face_partition, self_neighbour
    g = build_case(make_config("lake10"), dense=False)
    pc = face_partition(g, 4, 1, "morton")
    f = np.concatenate([n.faces for n in pc.fneighbours])
    # (the lake's bathymetry is continuous, so its two sides agree already: make side 2 differ, as a
    # discontinuous bathymetry would)
    for k in ("pbprime_face", "pbprime_df_face", "zbot_face"):
        pc.arrays[k][1][:, f] = 1.01 * pc.arrays[k][1][:, f] + 1.0
    ref = {k: np.array(v) for k, v in pc.arrays.items() if k.startswith(("pbprime", "zbot_face", "coeff_"))}
    other = np.setdiff1d(np.arange(pc.scalars["nface"]), f)
    sn = self_neighbour(pc)
    A = sn.arrays
    for k in ("pbprime_face", "pbprime_df_face", "zbot_face"):
        assert np.array_equal(A[k][1][:, f], A[k][0][:, f])
        assert not np.array_equal(A[k][1][:, f], ref[k][1][:, f])
        assert np.array_equal(A[k][:, :, other], ref[k][:, :, other])
    for a, b in (("coeff_pbpert_L", "coeff_pbpert_R"), ("coeff_mass_pbub_L", "coeff_mass_pbub_R")):
        assert np.array_equal(A[a][:, f], A[b][:, f])
    wet = A["pbprime_face"][0][:, f] > 0
    assert np.all(A["coeff_pbpert_L"][:, f][wet] == 0.5)
    for k in ("coeff_pbpert_L", "coeff_pbub_LR", "coeff_mass_pbpert_LR"):
        assert np.array_equal(A[k][:, other], ref[k][:, other])


def test_bench_cli_lists_the_emulation_and_baseline_switches():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                         check=True).stdout
    for flag in ("--emulate", "--emulate-lists", "--order", "--no-base", "--no-c4-cpu"):
        assert flag in out

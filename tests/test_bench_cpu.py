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
    import bench
    from hnumo.case import build_case, make_config
    from hnumo.facepart import face_partition
    g = build_case(make_config("dg8L3q"), dense=False)
    pc = face_partition(g, 4, 1, "block")
    faces = np.concatenate([n.faces for n in pc.fneighbours])
    sn = bench._self_neighbour(pc)
    assert sn.nranks == 1 and sn.rank == 0
    assert len(sn.fneighbours) == 1 and sn.fneighbours[0].rank == 0
    assert np.array_equal(sn.fneighbours[0].faces, faces)
    assert len(np.unique(faces)) == faces.size


def test_bench_cli_lists_the_emulation_and_baseline_switches():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                         check=True).stdout
    for flag in ("--emulate", "--order", "--no-base", "--no-c4-cpu"):
        assert flag in out

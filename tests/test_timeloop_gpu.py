"""The reference's CI case end to end on the engine: CI/bump/numo3d.in (bump 10x10, N=4, 2
layers, dt 100 s, dt_btp 1.8 s, 10800 s = 108 baroclinic steps) through the time loop of
hnumo/diagnostics.py (mod_time_loop.F90), checked as CI/bump/check.F90 checks the reference:
per-layer mass loss <= 1e-12.  The h/u/v extrema are compared with the reference's own FIN
files (tests/golden/*_mlswe_FIN.txt): the CI's file is matched to 1e-6 relative; the two
Examples/ files disagree with it at the 1e-2 level and are only reported."""
import io
import os

import pytest

from hnumo import diagnostics as D

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FINS = ["ci_bump_ref_mlswe_FIN.txt", "examples_bump_ref_mlswe_FIN.txt", "examples_bump_mlswe_ref_FIN.txt"]


def test_bump_ci_on_engine(case_factory, tmp_path):
    from hnumo.engine import Engine
    case = case_factory("bump10")
    e = Engine(case)
    D.time_loop(case, e, 10800.0, out_dir=str(tmp_path), dump_data=False, out=io.StringIO())
    e.close()
    fin = (tmp_path / "mlswe_FIN.txt").read_text()
    print(fin)
    worst = {}
    for name in FINS:
        ok, rep = D.ci_check(fin, open(os.path.join(GOLD, name)).read())
        assert ok, rep                                 # check.F90:58: mass loss <= 1e-12
        worst[name] = max(max(v) for r in rep.values() for k, v in r.items() if k != "mass_loss")
        print(name, "max relative difference of the h/u/v extrema: %.3e" % worst[name])
    # the CI's own reference file (the one check.F90 reads): h/u/v extrema of both layers agree
    # to 2e-7 relative after 108 steps (measured 1.8e-7; the Examples/ files are from other
    # code versions and differ by ~1e-2)
    assert worst[FINS[0]] < 1e-6

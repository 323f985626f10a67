"""The time loop's output formats and diagnostics (h-numo_amd/hnumo/diagnostics.py; SURVEY.md
§8f row f2): Fortran edit descriptors, mlswe_FIN.txt, the mlswe#### snapshot and its restart
reader, the layer mass, and the reference CI's check (CI/bump/check.F90).

Fixture data: tests/golden/*_mlswe_FIN.txt are the reference's own mlswe_FIN.txt files
(CI/bump/ref_mlswe_FIN.txt, Examples/bump/ref_mlswe_FIN.txt, Examples/bump/mlswe_ref_FIN.txt),
copied as data."""
import io
import os

import numpy as np
import pytest

from hnumo import diagnostics as D
from util import layer_mass, rel

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FINS = ["ci_bump_ref_mlswe_FIN.txt", "examples_bump_ref_mlswe_FIN.txt", "examples_bump_mlswe_ref_FIN.txt"]


def parse_fin(text):
    """(mass_loss[L], qmax(5,L), qmin(5,L)) from an mlswe_FIN.txt (dp rows left at 0)."""
    lines = text.splitlines()
    L = len(lines) // 6
    ml, qmax, qmin = [], np.zeros((5, L)), np.zeros((5, L))
    for k in range(L):
        ml.append(float(lines[6 * k + 1].split("=")[1]))
        for r, i in zip(range(2, 6), (0, 1, 2, 4)):
            t = lines[6 * k + r].split()
            qmax[i, k], qmin[i, k] = float(t[4]), float(t[5])
    return ml, qmax, qmin


def test_fortran_edit_descriptors():
    assert D.fmt_e(0.201449116645e2, 24, 12) == "      0.201449116645E+02"
    assert D.fmt_e(-0.132668287181e-2, 24, 12) == "     -0.132668287181E-02"
    assert D.fmt_e(0.18640037e-15, 16, 8) == "  0.18640037E-15"
    assert D.fmt_e(100.0, 23, 16, "D") == " 0.1000000000000000D+03"
    assert D.fmt_e(-0.0, 11, 4) == "-0.0000E+00"
    assert D.fmt_e(9.99996, 11, 4) == " 0.1000E+02"          # rounding carries into the exponent
    assert D.fmt_e(1.5e-120, 12, 4) == "  0.1500-119"          # 3-digit exponent drops the letter
    assert D.fmt_es(1.7857142857142858, 13, 5) == "  1.78571E+00"
    assert D.fmt_i(7, 8) == "       7"


@pytest.mark.parametrize("name", FINS)
def test_fin_layout_reproduces_reference_files(name):
    """mlswe_FIN.txt written from the numbers of each of the reference's FIN files is that file,
    byte for byte (print_diagnostics.F90:167-184 formats)."""
    ref = open(os.path.join(GOLD, name)).read()
    assert D.fin_text(*parse_fin(ref)) == ref


def test_ci_check_on_reference_files():
    """check.F90's acceptance (mass loss <= 1e-12 per layer) holds for each reference FIN file,
    and the reported field differences between them are the reference's own inconsistency
    (SURVEY.md §8c): 1e-4..1e-2 relative."""
    texts = [open(os.path.join(GOLD, n)).read() for n in FINS]
    ok, rep = D.ci_check(texts[1], texts[0])
    assert ok
    assert 1e-5 < rep[1]["h"][0] < 1e-2


@pytest.mark.ref
@pytest.mark.parametrize("name", ["bump10", "dg8L3q"])
def test_diagnostics_match_reference_fortran(name, case_factory, tmp_path):
    """The reference's own diagnostics (diagnostics.F90, compute_conserved.F90, courant.F90,
    print_diagnostics.F90, run by oracle/_ref/ref_driver mode 5 after 2 steps) against
    hnumo/diagnostics.py on the same state: the stdout reports (idone 0 and 1), the
    mass_mlswe.cons line and mlswe_FIN.txt are identical byte for byte."""
    import oracle as O
    case = case_factory(name)
    ref = O.run_reference(case, "diag", 2, workdir=str(tmp_path))
    L = case.scalars["nlayers"]
    qf0 = D.layer_fields(case, case.arrays["q_df"])
    mass0 = [D.conserved_mass(case, qf0[0, :, k]) for k in range(L)]
    qf = D.layer_fields(case, ref["q_df"])
    t = 2 * case.scalars["dt"]
    text0, cons, _ = D.print_diagnostics(case, qf, ref["qb_df"], t, 2, 0, mass0)
    text1, _, fin = D.print_diagnostics(case, qf, ref["qb_df"], t, 2, 1, mass0)
    out = ref["stdout"]
    assert out[out.index(" =====") - 1:].lstrip("\n") == text0 + text1
    assert (tmp_path / "mass_mlswe.cons").read_text() == cons + "\n"
    assert (tmp_path / "mlswe_FIN.txt").read_text() == fin


def test_conserved_mass_matches_layer_mass(case_factory):
    case = case_factory("bump10")
    q = case.arrays["q_df"]
    qf = D.layer_fields(case, q)
    m = [D.conserved_mass(case, qf[0, :, k]) for k in range(case.scalars["nlayers"])]
    assert rel(np.array(m), layer_mass(case, q)) < 1e-13


def test_snapshot_restart_round_trip(case_factory, tmp_path):
    """write_snapshot -> restart_state (mod_restart.F90:15-87).  D23.16 keeps 16 significant
    digits, so the round trip is exact to 1e-15 relative, not bitwise (the reference's
    restart has the same property)."""
    import oracle as O
    case = case_factory("bump10")
    o = O.Oracle(case)
    q, qb, qp = o.state()
    o.ti_rk_bcl(q, qb, qp)
    p = str(tmp_path / "mlswe0001")
    D.write_snapshot(p, case, q, qb)
    snap = D.read_snapshot(p)
    assert snap["nlayers"] == 2 and snap["npoin"] == case.scalars["npoin"]
    assert rel(snap["coord"], case.arrays["coord"][:2]) < 1e-15
    q2, qb2, qp2 = D.restart_state(case, p)
    for v in (0, 2, 3):
        assert rel(qb2[v], qb[v]) < 1e-15, v
    # qb(2) = qb(1) - pbprime_df (mod_restart.F90:45): the 16-digit rounding of qb(1) is
    # amplified by the cancellation (|pb'| ~ 1e-6 |pb|)
    assert np.abs(qb2[1] - qb[1]).max() < 1e-15 * np.abs(qb[0]).max()
    for v in range(3):
        assert rel(q2[v], q[v]) < 1e-14, v
    assert rel(qp2[0], qp[0]) < 1e-14
    # u' = u_k - u_bar is recomputed from the rounded state (a difference of nearly equal
    # velocities): bounded against |u_k|
    for v in (1, 2):
        assert np.abs(qp2[v] - qp[v]).max() < 1e-10 * np.abs(q[v] / q[0]).max(), v


def test_time_loop_outputs(case_factory, tmp_path):
    """mod_time_loop around the oracle for 3 steps with dump_data: snapshots 0..3, one
    mass_mlswe.cons line per report, the final report and mlswe_FIN.txt, mass loss <= 1e-12."""
    import oracle as O
    case = case_factory("bump10")
    o = O.Oracle(case)
    buf = io.StringIO()
    q, qb, qp = D.time_loop(case, o, 300.0, out_dir=str(tmp_path), dump_data=True, out=buf)
    for n in range(4):
        assert (tmp_path / f"mlswe{n:04d}").exists()
    cons = (tmp_path / "mass_mlswe.cons").read_text().splitlines()
    assert len(cons) == 4 and cons[-1].split()[0] == "3"
    fin = (tmp_path / "mlswe_FIN.txt").read_text()
    ok, _ = D.ci_check(fin, open(os.path.join(GOLD, FINS[0])).read())
    assert ok
    assert "**Simulation Finished**" in buf.getvalue()
    # restart from snapshot 2 and run to the end: the same final state as the straight run,
    # up to the 16-digit rounding of the snapshot, amplified by one step of dynamics
    o2 = O.Oracle(case)
    q2, qb2, qp2 = D.time_loop(case, o2, 300.0, out_dir=str(tmp_path), time_initial=200.0, restart_file_number=2,
                               lprint_diagnostics=False, lcheck_conserved=False, out=io.StringIO())
    assert rel(qb2[0], qb[0]) < 1e-13 and rel(q2[0], q[0]) < 1e-10

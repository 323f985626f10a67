"""Round-5 schedule choices that must not move a bit (engine.hip): the workgroup -> element
placement of the persistent sub-cycle and the element kernels (`HNUMO_PERSIST_PERM`,
`HNUMO_GLUE_PERM`), the first stage of a sub-cycle storing its time-average terms instead of
adding them to zeroed slots (`HNUMO_ACC_ZERO`), and the large-mesh element kernels
(`HNUMO_BCL_BIG`).  Each knob's old behaviour against the default, two steps, the whole state and
every parity field."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(case, monkeypatch, env):
    from hnumo.engine import Engine
    env = dict(env, HNUMO_EXPERIMENTS="1") if env else env   # experiment knobs need the gate
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = Engine(case)
    for k in env:
        monkeypatch.delenv(k)
    seen = {x.split("=")[0] for x in e.overrides}
    assert seen <= set(env) and bool(seen) == bool(env) and not any("ignored" in x for x in e.overrides)
    st = e.state()
    for _ in range(2):
        e.ti_rk_bcl(*st)
    from hnumo import bundle as B
    fields = {f: e.field(f) for f, _ in B.FIELDS}
    path = e.stage_path
    e.close()
    return st, fields, path


def _same(a, b):
    for x, y in zip(a[0], b[0]):
        assert np.array_equal(x, y)
    for f in a[1]:
        assert np.array_equal(a[1][f], b[1][f]), f


def test_placement_keeps_the_bits(case_factory, monkeypatch):
    """dg25L3 (625 elements on 256 CUs: 113 CUs hold three): boundary elements on the CUs holding
    two, for the persistent sub-cycle and the element kernels, against the identity placement."""
    case = case_factory("dg25L3")
    new = _run(case, monkeypatch, {})
    old = _run(case, monkeypatch, {"HNUMO_PERSIST_PERM": "0", "HNUMO_GLUE_PERM": "0"})
    assert new[2] == old[2] == "persistent"
    _same(new, old)


@pytest.mark.parametrize("cfg,kw", [("dg316L3", {"nelx": 48, "nely": 48}), ("dg25N7L3", {})])
def test_first_stage_store_and_large_mesh_kernels_keep_the_bits(cfg, kw, case_factory, monkeypatch):
    """A 48x48 double gyre (2,304 elements: per-stage launches, the large-mesh mass/cons kernels)
    and C3 (the persistent sub-cycle without register averages): the default against the zeroing
    pass before each sub-cycle and the small-mesh element kernels."""
    case = case_factory(cfg, **kw)
    new = _run(case, monkeypatch, {})
    old = _run(case, monkeypatch, {"HNUMO_ACC_ZERO": "1", "HNUMO_BCL_BIG": "0"})
    assert new[2] == old[2]
    _same(new, old)


def test_stray_experiment_knob_is_ignored_and_reported(case_factory, monkeypatch):
    """An experiment knob without HNUMO_EXPERIMENTS=1 changes nothing (a stray variable on a
    benchmark box) and is reported by hnumo_overrides; HNUMO_SUMMATION takes only its two words."""
    from hnumo.engine import Engine, EngineError
    case = case_factory("dg25L3")
    monkeypatch.setenv("HNUMO_PERSIST_LDS_PAD", "30000")   # honoured, this would drop persistence
    e = Engine(case)
    assert e.stage_path == "persistent"
    assert e.overrides == ["HNUMO_PERSIST_LDS_PAD=30000 (ignored: HNUMO_EXPERIMENTS!=1)"]
    e.close()
    monkeypatch.delenv("HNUMO_PERSIST_LDS_PAD")
    monkeypatch.setenv("HNUMO_SUMMATION", "fast")
    with pytest.raises(EngineError) as ex:
        Engine(case)
    assert ex.value.code == 4
    monkeypatch.setenv("HNUMO_SUMMATION", "reference")
    e = Engine(case)
    assert e.overrides == ["HNUMO_SUMMATION=reference"] and e.summation == "reference"
    e.close()

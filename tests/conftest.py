import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "h-numo_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "ref: needs the reference Fortran harness oracle/_ref (build container only)")


def pytest_collection_modifyitems(config, items):
    import shutil  # noqa: F401
    ref_ok = os.path.exists(os.path.join(REPO, "oracle", "_ref", "ref_driver"))
    for it in items:
        if "ref" in it.keywords and not ref_ok:
            it.add_marker(pytest.mark.skip(reason="oracle/_ref not built (no /root/reference here)"))


_cases = {}


@pytest.fixture(scope="session")
def case_factory():
    from hnumo.case import build_case, make_config

    def get(name, **kw):
        key = (name, tuple(sorted(kw.items())))
        if key not in _cases:
            _cases[key] = build_case(make_config(name, **kw))
        return _cases[key]

    return get

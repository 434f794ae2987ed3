"""The rejected k <= 8 kernel variants of rounds 1-2 (tools/zoo/kf_count_zoo.hip,
KF_COUNT_VARIANT) as their own library, tools/zoo/libkf2vec_zoo.so (built by
`python -m kf2vecfsw_amd.build --zoo`).  Not part of the product; run on a GPU
box with `pytest tools/zoo -m gpu` (the repo's pytest.ini collects tests/ only).

The zoo library is selected by a fixture of this directory only (the
`native` fixture below), never by an import-time environment change: a
`pytest` that also collects tests/ keeps loading the product library there."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import oracle, toy  # noqa: E402,F401  (fixtures shared with tests/)

ZOO_LIB = os.path.join(ROOT, "tools", "zoo", "libkf2vec_zoo.so")


@pytest.fixture(scope="session")
def native():
    """The zoo library as kf2vecfsw_amd._native's handle for this session."""
    if not os.path.exists(ZOO_LIB):
        pytest.skip("tools/zoo/libkf2vec_zoo.so not built (python -m kf2vecfsw_amd.build --zoo)")
    from kf2vecfsw_amd import _native
    mp = pytest.MonkeyPatch()
    mp.setattr(_native, "LIB_PATH", ZOO_LIB)
    mp.setattr(_native, "_lib", None)
    yield _native.lib()
    mp.undo()
    _native._lib = None

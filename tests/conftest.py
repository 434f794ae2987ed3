import gzip
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
TOY = os.path.join(GOLDEN, "toy")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (fna dir, kf dir) pairs of the reference toy example (toy_example/*, README.md:220-316)
TOY_PAIRS = [("train_tree_fna", "train_tree_kf"), ("test_fna", "test_kf")]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and the built HIP library")


def toy_fna():
    """[(file name, sample name, bytes, expected .kf bytes)] for the 7 pinned pairs."""
    out = []
    for fd, kd in TOY_PAIRS:
        for f in sorted(os.listdir(os.path.join(TOY, fd))):
            name = f[:-3]
            sample = name.rsplit(".f", 1)[0]
            data = gzip.open(os.path.join(TOY, fd, f)).read()
            exp = gzip.open(os.path.join(TOY, kd, sample + ".kf.gz")).read()
            out.append((name, sample, data, exp))
    return out


@pytest.fixture(scope="session")
def toy():
    return toy_fna()


@pytest.fixture(scope="session")
def native():
    from kf2vecfsw_amd import build
    build.build()
    from kf2vecfsw_amd import _native
    return _native.lib()


@pytest.fixture(scope="session")
def oracle():
    import kf_oracle
    kf_oracle.build()
    return kf_oracle


@pytest.fixture(autouse=True)
def _stall_dump():
    """A test that runs past KF_TEST_STALL_S seconds (170: before a 3-minute
    silence watchdog) dumps every thread's stack and ends the run, so a stall
    names its test and the line it waits on instead of ending silently."""
    import faulthandler
    faulthandler.dump_traceback_later(int(os.environ.get("KF_TEST_STALL_S", "170")), exit=True)
    yield
    faulthandler.cancel_dump_traceback_later()

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "gym-loadbalancing_amd")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_addoption(parser):
    parser.addoption("--lib", default=None,
                     help="run the tests against another build of liblbk8s.so (a diagnostic A/B build under "
                          "exp/; the product tests load the in-tree library)")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    lib = config.getoption("--lib")
    if lib:
        from lbk8s import _native
        _native.LIB_PATH = os.path.abspath(lib)


def golden_names(prefix=""):
    """Env-trajectory fixtures (nn_* hold network / learner goldens, eval_* evaluation loops)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN)
                  if f.endswith(".npz") and f.startswith(prefix) and not f.startswith(("nn_", "eval_")))


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle

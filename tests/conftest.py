"""Shared fixtures.  GPU tests are marked ``gpu`` and run only on the MI355X
box (``pytest -m gpu``); everything else runs on CPU (``-m "not gpu"``).
The oracles under oracle/ are test infrastructure: only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() use them, as the checker."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O

    if not os.path.exists(O.ORC_SO) or os.environ.get("PHT_REBUILD_ORACLE"):
        O.build()
    return O.OracleLib()


@pytest.fixture(scope="session")
def lib():
    import phasetype_amd as P

    return P.load()


@pytest.fixture(scope="session")
def gpu(lib):
    import phasetype_amd as P

    n = P.device_count()
    assert n > 0, "GPU tests need a HIP device: " + lib.pht_last_error().decode()
    return n

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP engine parity / smoke)")
    config.addinivalue_line("markers", "slow: long CPU test")


def golden_files():
    """Placement replay fixtures (tests/golden/gen_golden.py, gen_service.py)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz")
                  and not f.startswith(("steal_", "svc_steal_", "svcaddw_", "svcgraph_")))


def svc_second_graph_files():
    """Service-mode message streams with a second graph submitted (gen_service.py second-graph)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcgraph_") and f.endswith(".npz"))


def svc_add_worker_files():
    """Service-mode message streams with workers joining (tests/golden/gen_service.py add-workers)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcaddw_") and f.endswith(".npz"))


def svc_steal_files():
    """Service-mode message streams with confirmed steals (tests/golden/gen_service.py)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svc_steal_") and f.endswith(".npz"))


def steal_files():
    """WorkStealing balance fixtures (tests/golden/gen_steal.py)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("steal_") and f.endswith(".npz")
                  and f != STEAL_REFTESTS)


# the reference's own balance unit scenarios, many problems in one file (gen_steal_ref.py)
STEAL_REFTESTS = "steal_reftests.npz"


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN

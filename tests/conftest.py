import os
import sys

import pytest

# In-process virtual ranks (one DeviceSolver + HIP stream per rank, one host
# thread each) with the xGMI mailbox transport need every rank's stream on a
# hardware queue of its own plus one for the default stream: n ranks need
# GPU_MAX_HW_QUEUES >= n + 1 (tools/hwq_probe.py, profiles/hwq_probe_r06.md;
# DeviceSolver::p2p_import refuses fewer).  The GPU suite runs up to 8 such
# ranks, so it asks HIP for 16 queues before the first HIP call.  (Real
# multi-GPU runs are one process per GPU and need no such setting.)
os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIXTURES = os.path.join(ROOT, "tests", "fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def hf():
    import openhyperflow2d_amd as pkg

    pkg.native()
    return pkg


@pytest.fixture(scope="session")
def native(hf):
    return hf.native()


@pytest.fixture
def gpu(hf):
    if not hf.gpu_available():
        pytest.fail("GPU test requires a HIP device; the native HIP path must run (no CPU fallback)")
    return hf


def deck_path(name):
    return os.path.join(FIXTURES, "decks", name)


def read_deck(name):
    with open(deck_path(name), "r", errors="replace") as f:
        return f.read()

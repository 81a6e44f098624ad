import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402

# every handle the tests create starts with NaN-filled workspaces (lz_init)
os.environ.setdefault("LZ_POISON", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")


@pytest.fixture(scope="session")
def lz():
    return ge.load_package()


@pytest.fixture(scope="session")
def orc():
    return ge.load_oracle()


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "golden_matrix_a.npz"))


@pytest.fixture(scope="session")
def handle(lz):
    h = lz.Handle(0)
    yield h
    h.close()


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return torch


def golden_csr(lz, g, N, bug=False):
    tag = "_bug" if bug else ""
    return lz.CsrHost(int(g[f"N{N}_n"]), g[f"N{N}{tag}_row_ptr"], g[f"N{N}{tag}_col"], g[f"N{N}{tag}_val"])


@pytest.fixture(autouse=True)
def _poison_lds(request):
    """Before every GPU test, fill each CU's LDS with NaN bit patterns
    (lz_debug_poison_lds), so a kernel that reads LDS it never wrote fails
    deterministically rather than when the previous kernel left garbage."""
    if request.node.get_closest_marker("gpu") is not None:
        h = request.getfixturevalue("handle")
        request.getfixturevalue("torch_cuda")
        h.debug_poison_lds()
    yield

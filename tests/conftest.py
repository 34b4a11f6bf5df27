import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "torch-ngp_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# The -m gpu run stops at the first failure (-x), so the tests that establish
# the coverage rows run first: the benched step against the oracle on every
# BASELINE config, the reference operator surface (every _backend entry point
# against the oracle), the render loop, the reference's own gradcheck, the
# reference-executed golden fixtures, then the RCCL data-parallel path. The
# rest keep their order.
FIRST = ["test_gpu_e2e_oracle.py", "test_gpu_parity.py", "test_gpu_render.py", "test_gradcheck.py",
         "test_golden_reference.py", "test_gpu_rccl.py"]

_REPORT = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return FIRST.index(name) if name in FIRST else len(FIRST)
    items.sort(key=rank)  # stable: the order inside a file is kept


@pytest.fixture
def parity_report(request):
    """Append a one-line parity summary (config, sample count, errors); the
    lines are printed at the end of the run, where a log's tail shows them."""
    def add(line):
        _REPORT.append(f"{request.node.nodeid.split('::')[-1]}: {line}")
    return add


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if _REPORT:
        terminalreporter.section("parity summary")
        for line in _REPORT:
            terminalreporter.write_line(line)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")

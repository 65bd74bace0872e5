import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(__file__))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def orbpl():
    from _pkg import load_pkg
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    from _pkg import load_oracle
    o = load_oracle()
    o.lib()
    return o


@pytest.fixture(scope="session")
def synth(orbpl):
    import orbpl.synth as s
    return s


if os.environ.get("ORBPL_TEST_TORCH_FIRST"):
    # Load torch's bundled HIP runtime before liborbpl.so (both carry the
    # SONAME libamdhip64.so.7; the first one loaded serves the process).
    import torch  # noqa: F401
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda")

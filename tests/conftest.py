import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE.json) property checks")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def ctx():
    from tests.util import native_mode

    if native_mode():
        # torch-free (tests/util.py): the ROCm runtime the library was built against
        import raptor_amd as ra

        try:
            return ra.Context.native(0)
        except ra.AmgError as e:
            pytest.skip(f"no GPU ({e})")
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import raptor_amd as ra

    return ra.Context(0)


@pytest.fixture
def say(capfd, request):
    """Progress line on the terminal (capture bypassed) for the long full-size tests, so a
    phase that takes minutes is never mistaken for a hang."""
    import time

    t0 = time.perf_counter()

    def _say(msg):
        with capfd.disabled():
            print(f"[{request.node.name} {time.perf_counter() - t0:7.1f}s] {msg}", flush=True)

    return _say

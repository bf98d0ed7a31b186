import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def kats():
    import json

    return json.loads((ROOT / "tests" / "golden" / "kats.json").read_text())


@pytest.fixture(autouse=True)
def _gpu_errors_belong_to_their_test(request):
    """After every GPU test: wait for the device and read one value back, so
    an asynchronous device error is reported by the test that caused it, not
    by a later one."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return
    torch.cuda.synchronize()
    torch.zeros(1, device="cuda").cpu()

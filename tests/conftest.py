import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "halogen-pathtracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def built():
    """Build the oracle (test infra) and the HIP library (product) once per session."""
    import subprocess
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    so = ROOT / "halogen-pathtracer_amd" / "halogen" / "libhalogen_hip.so"
    if not so.exists():
        subprocess.run(["make", "-s", "-j4", "-C", str(ROOT / "halogen-pathtracer_amd")], check=True)
    return True


@pytest.fixture(scope="session")
def gpu(built):
    from halogen import abi
    if not abi.gpu_available():
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")
    return True

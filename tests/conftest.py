import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "surely-raytracing_amd"))
sys.path.insert(0, str(REPO / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


def _ensure_built():
    """Build the in-tree libraries if they are missing (host + oracle are quick; the HIP
    library cross-compiles for gfx950 without a GPU)."""
    need = [REPO / "build" / "librthost.so", REPO / "build" / "librtmi355x.so",
            REPO / "oracle" / "_build" / "liboracle_f64.so",
            REPO / "oracle" / "_build" / "liboracle_f32.so"]
    if all(p.exists() for p in need):
        return
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-C", str(REPO), f"-j{jobs}", "device", "host", "oracle"], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import surely_rt as rt

    n = rt.device_count()
    if n <= 0:
        pytest.fail("no HIP device visible: -m gpu tests must run on the GPU box")
    return n

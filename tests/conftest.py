import os
import subprocess
import sys
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "tests", "golden")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # scene-specialised kernels compile into a cache private to this test session, so no code
    # object from an earlier build or toolchain can stand in for the current sources
    os.environ.setdefault("BDPT_JIT_CACHE", tempfile.mkdtemp(prefix="bdpt-jit-test-"))
    # build the in-tree artefacts once if they are missing (cheap no-op otherwise)
    need = [os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "libbdpt.so"),
            os.path.join(REPO, "oracle", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.check_call(["make", "-s", "-j8"], cwd=REPO)


def _gpu_available() -> bool:
    try:
        import torch  # noqa: F401  (device probe only)
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _gpu_available():
        pytest.skip("no GPU")
    return 0


SCENES = os.path.join(REPO, "assets", "scenes")
GOLDEN = os.path.join(REPO, "tests", "golden")

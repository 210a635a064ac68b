import os
import subprocess
import sys

import pytest

# One HIP runtime per process: torch ships its own libamdhip64, and libapg
# binds to whichever copy is loaded first.  Load torch first (as bench.py
# does) so tests that mix libapg with torch device buffers see one runtime.
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libapg's HIP kernels)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _ensure_built():
    lib = os.path.join(ROOT, "allpathslg_amd", "libapg.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "allpathslg_amd", "csrc")], check=True)
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu_ctx():
    from allpathslg_amd import Context

    ctx = Context(device=0, timing=False)
    yield ctx
    ctx.close()

import os
import shutil
import subprocess
import sys

import pytest

try:  # torch first: libvrt.so then binds to torch's HIP runtime (one runtime
    import torch  # noqa: F401  per process; see DESIGN.md "Host runtime")
except Exception:  # pragma: no cover - CPU-only environments without torch
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def _ensure_built():
    """Build when a library is missing or libvrt.so's embedded source hash
    (vrt_build_id) differs from the tree's: the tests must exercise the
    sources at this HEAD, not a stale binary."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_id
    need = [os.path.join(ROOT, "voxelraytrace20190722_amd", "libvrt.so"),
            os.path.join(ROOT, "oracle", "liboracle.so")]
    if all(os.path.exists(p) for p in need) and not build_id.stale():
        return
    if shutil.which("make") is None:
        raise RuntimeError("libvrt.so missing or stale (build id) and `make` unavailable")
    subprocess.run(["make", "-j8"], cwd=ROOT, check=True)
    if build_id.stale():
        raise RuntimeError("libvrt.so build id still differs from the tree after make")


_ensure_built()


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gold():
    return golden

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "raytracing-clj_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library with at least one visible GPU (fails loudly otherwise)."""
    # torch's wheel bundles its own HIP runtime under the same soname
    # (libamdhip64.so.7) as /opt/rocm's, which librtclj.so links: whichever
    # loads first serves the process, and torch fails to initialise on the
    # /opt/rocm one ("No HIP GPUs are available"). Tests that use torch
    # buffers therefore load torch first, as bench.py does.
    import torch  # noqa: F401
    import rtclj

    n = rtclj.lib.rt_device_count()
    assert n > 0, "no GPU visible to librtclj.so (HIP); GPU tests must run on the MI355X box"
    return rtclj

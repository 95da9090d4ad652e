import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The small shapes of the tests would fall below the tile-count thresholds under which the q|k|v
# RoPE and the SwiGLU epilogues run as separate kernels (TP shard widths, kernels.py); keep the
# fused epilogues on for them, as at the real shapes (tests that want the split path set it).
for _k in ("PICOTRON_ROPE_FUSE_MIN_TILES", "PICOTRON_SWIGLU_FUSE_MIN_TILES", "PICOTRON_SWIGLU_BWD_MIN_TILES"):
    os.environ.setdefault(_k, "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the gfx950 kernels")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)

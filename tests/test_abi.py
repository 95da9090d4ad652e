"""The C-ABI library loads and exports every entry point include/picotron_hip.h declares (CPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "picotron_hip.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^int\s+(pt_\w+)\s*\(", txt, flags=re.M)))


def test_header_parses():
    names = declared()
    assert len(names) >= 12, names


def test_library_exports_every_declared_symbol():
    from picotron_amd import _C
    if not os.path.exists(_C.LIB_PATH):
        from picotron_amd import build
        build.build(verbose=False)
    lib = _C.load_library()
    for n in declared():
        assert hasattr(lib, n), f"missing export {n}"
    # the ctypes binding covers exactly the header
    assert sorted(_C.SIGNATURES) == declared()


def test_no_compute_without_gpu():
    import torch
    from picotron_amd import _C
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_C.HipKernelError):
        _C.lib()


def test_argument_errors_map_to_codes():
    """Host-side validation inside the ABI returns PT_E* before touching the device."""
    from picotron_amd import _C
    lib = _C.load_library()
    assert lib.pt_rmsnorm_fwd(None, None, None, None, None, None, 0, 0, 1e-5, 0, None) == -1
    assert lib.pt_gemm_pick_tile(4096, 2048, None, 0, None, 0) >= 0
    assert lib.pt_gemm_pick_tile(100, 100, None, 0, None, 0) == -1


def test_no_kernel_spills_to_scratch():
    """Every kernel of the library keeps its registers: no VGPR spill and no scratch (private
    segment) memory in any gfx950 code object (tools/spills.py reads the AMDGPU metadata notes)."""
    import glob
    import subprocess
    import sys
    objs = glob.glob(os.path.join(ROOT, "picotron_amd", "lib", "obj", "*.o"))
    if not objs or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"):
        pytest.skip("no built objects / ROCm LLVM tools")
    from picotron_amd import build
    build.build(verbose=False)   # the objects match the sources
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "spills.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 kernel(s) with VGPR spills or scratch memory" in r.stdout

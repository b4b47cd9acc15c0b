"""Every in-tree native library resolves all of its symbols (RTLD_NOW) — catches missing kernel
host stubs / unresolved references at build time instead of on the GPU box."""
import ctypes
import os
from pathlib import Path

import pytest

LIB = Path(__file__).resolve().parent.parent / "stereoalgorithms_amd" / "lib"
NAMES = ["libstereo_host.so", "libstereo_amd.so", "libRAFTStereo.so", "libHitNet.so", "libCREStereo.so",
         "libFastACVNet_plus.so"]


@pytest.mark.parametrize("name", NAMES)
def test_library_loads_with_all_symbols(name):
    path = LIB / name
    if not path.exists():
        pytest.skip(f"{name} not built")
    ctypes.CDLL(str(path), mode=os.RTLD_NOW | ctypes.RTLD_GLOBAL)


@pytest.mark.parametrize("lib,syms", [
    ("libRAFTStereo.so", ["Initialize", "RunRAFTStereo", "Version", "Release"]),
    ("libHitNet.so", ["Initialize", "RunHitNet", "Version", "Release"]),
    ("libCREStereo.so", ["Initialize", "RunCREStereo", "RunCREStereo_RectifyImage", "Version", "Release"]),
    ("libFastACVNet_plus.so", ["Initialize", "RunFastACVNet_plus", "RunFastACVNet_plus_RectifyImage", "Version",
                               "Release"]),
])
def test_reference_abi_symbols(lib, syms):
    path = LIB / lib
    if not path.exists():
        pytest.skip(f"{lib} not built")
    L = ctypes.CDLL(str(path), mode=os.RTLD_NOW | ctypes.RTLD_GLOBAL)
    for s in syms:
        assert hasattr(L, s), s
    L.Version.restype = ctypes.c_char_p
    assert L.Version(None).decode().endswith("_V1.0")

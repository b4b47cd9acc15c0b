"""The ctypes mirrors of the launch-argument structs (stereoalgorithms_amd/_native.py) match the C layouts in
csrc/include/sa/kernels.h: loading the library checks every struct's size against the native sizeof, so a field
added or removed on one side fails here (and at import on a GPU box) instead of shifting every later field."""
import ctypes as C

import pytest

from stereoalgorithms_amd import _native as N


@pytest.mark.skipif(not N.available(), reason="native library not built")
def test_struct_layouts_match_native():
    lib = N.dev()  # raises on a mismatch
    for st in (N.SaConvSrc, N.SaConvArgs, N.SaNormArgs, N.SaAgclArgs, N.SaEwArgs):
        assert lib.sa_struct_size(st.__name__.encode()) == C.sizeof(st)
    assert lib.sa_struct_size(b"NoSuchStruct") == -1
    # the retired projection epilogue (5) must not be reachable from Python
    assert 5 not in N.EPI.values()

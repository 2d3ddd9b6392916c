"""CPU-side checks of the C-ABI library: it builds for gfx950, loads, exports
every symbol include/ls_hip.h declares with the expected ABI, and its host-side
argument validation rejects bad descriptors (no GPU needed for those paths)."""
import ctypes as C
import os
import re

import pytest

from conftest import REPO
from latentsync_amd import _lib


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "ls_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|size_t|const char\*)\s+(ls_\w+)\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.EXPORTED)
    assert lib.ls_abi_version() == _lib.ABI_VERSION


def test_gfx950_code_object():
    path = _lib.LIB_PATH
    data = open(path, "rb").read()
    assert b"gfx950" in data


def test_conv_desc_validation_rejects_bad_channels():
    lib = _lib.load()
    d = _lib.ConvDesc()
    d.x1, d.w, d.y = 16, 16, 16  # never dereferenced: validation fails first
    d.C1, d.ksize, d.K, d.N, d.n_img, d.H, d.W, d.Ho, d.Wo, d.stride = 12, 3, 128, 32, 1, 4, 4, 4, 4, 1
    d.ld1 = 16
    assert lib.ls_conv2d(C.byref(d), None) == 1
    assert b"multiples of 8" in lib.ls_last_error()
    d.C1 = 16
    d.K = 64  # too small for 9*16
    assert lib.ls_conv2d(C.byref(d), None) == 1


def test_attention_validation():
    lib = _lib.load()
    d = _lib.AttnDesc()
    d.q = d.k = d.v = d.o = 16
    d.batch, d.z2, d.heads, d.nq, d.nk, d.head_dim = 1, 1, 1, 16, 16, 513
    assert lib.ls_attention(C.byref(d), None) == 1

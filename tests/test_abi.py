"""The C-ABI library: built, loadable without a GPU, exports every symbol include/*.h declares,
and its pure functions behave.  No compute calls here (no GPU on the CPU runner)."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from smallz4_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "smallz4_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sz4_[a-z0-9_]+)\s*\(", text)))


def test_library_built():
    assert os.path.exists(_native.LIB_PATH), "run __graft_entry__.build()"


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(_native.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 12
    for name in names:
        assert hasattr(lib, name), name
    # and the Python binding describes each of them
    assert set(names) == set(_native.SIGNATURES)


def test_library_is_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_pure_functions():
    lib = _native.lib()
    assert lib.sz4_version() == b"1.5"
    n = 100_000_000
    assert lib.sz4_bound(n, 65536) >= n + 4 * (n // 65536) + 11
    assert lib.sz4_lz4_bound(n, 0) >= n + n // 255
    assert lib.sz4_lz4_bound(0, 1) > 0
    assert lib.sz4_bound(10, 0) == 0


def test_null_context_is_rejected():
    lib = _native.lib()
    assert lib.sz4_compress_blocks_device(None, None, 0, 65536, 9, 0, None, 0, None, None) == -1
    assert lib.sz4_last_error(None) == b"no context"


def test_create_fails_cleanly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _native.lib()
    h = ctypes.c_void_p()
    assert lib.sz4_create(ctypes.byref(h), 0, 0) != 0


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_cpp_dropin_header_compiles(tmp_path):
    src = os.path.join(ROOT, "tests", "cpp", "dropin_demo.cpp")
    subprocess.run(["g++", "-std=c++11", "-fsyntax-only", "-Wall", "-I", os.path.join(ROOT, "include"), src],
                   check=True)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_c_decoder_dropin_header_compiles():
    """include/smallz4cat_amd.h (smallz4cat.c's interface over the C ABI) compiles as C99."""
    src = os.path.join(ROOT, "tests", "cpp", "unlz4_demo.c")
    subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"), src],
                   check=True)


def test_decoder_rejects_null_context():
    lib = _native.lib()
    size = ctypes.c_uint64()
    assert lib.sz4_unlz4(None, b"x", 1, None, 0, None, 0, ctypes.byref(size)) == -1
    assert lib.sz4_unlz4_device(None, None, 0, None, 0, None, 0, ctypes.byref(size), None) == -1

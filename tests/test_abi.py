"""C-ABI checks that need no GPU: the library loads, exports exactly what include/vfilter.h
declares, the ctypes binding covers every entry point, and calls without a device fail
loudly (there is no CPU fallback anywhere in the product path)."""
import os
import re
import subprocess

import numpy as np
import pytest

import vfilter
from vfilter import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vfilter.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vf_[a-z0-9_]+)\s*\(", text)))


def test_library_built_in_tree():
    assert os.path.exists(_lib.library_path()), "run `make` first"
    assert _lib.library_path().startswith(os.path.join(ROOT, "distributed-video-filter_amd"))


def test_exports_every_header_symbol():
    syms = header_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.library_path()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (vf_[a-z0-9_]+)$", out, flags=re.M))
    assert set(syms) == exported, (set(syms) ^ exported)
    lib = _lib.load_library()
    for s in syms:
        assert hasattr(lib, s)


def test_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_library_is_gfx950_code_object():
    """The embedded offload bundle is a gfx950 code object and nothing else."""
    blob = open(_lib.library_path(), "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}


def test_abi_version_and_status_strings():
    lib = _lib.load_library()
    assert lib.vf_get_abi_version() == _lib.ABI_VERSION == 3
    assert lib.vf_status_string(0) == b"VF_OK"
    assert b"gfx950" in lib.vf_status_string(_lib.VF_E_NODEVICE)
    assert lib.vf_status_string(-99) == b"unknown vfilter status"


def test_null_ctx_calls_fail_with_invalid():
    lib = _lib.load_library()
    assert lib.vf_invert_host(None, None, None, 10) == _lib.VF_E_INVALID
    assert b"ctx is NULL" in lib.vf_last_error(None)
    assert lib.vf_invert_device(None, None, None, 10, None) == _lib.VF_E_INVALID
    assert lib.vf_destroy(None) == _lib.VF_OK


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_no_device_fails_loudly():
    assert vfilter.device_count() == 0
    with pytest.raises(vfilter.VFilterError) as ei:
        vfilter.Context(0)
    assert ei.value.status == _lib.VF_E_NODEVICE
    with pytest.raises(vfilter.VFilterError):
        vfilter.bitwise_not(np.zeros((4, 4, 3), np.uint8), ctx=None)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setenv("VFILTER_LIB", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(vfilter.VFilterError, match="not found"):
        _lib.load_library()

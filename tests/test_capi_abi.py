"""CPU checks of the C-ABI boundary: the shared library loads, exports every entry point that
include/clipembed.h declares, and rejects bad configurations before touching a device."""
import ctypes
import os
import re

import pytest

from clipembed import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "clipembed.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:int|char|void)\s*\*?\s*(ce_[a-z0-9_]+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "ce_encode_image" in names and "ce_pacl_pool" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), f"{name} declared in clipembed.h but not exported"


def test_binding_covers_header():
    assert sorted(_lib.exported_symbols()) == declared_functions()


def test_version_and_error_string():
    L = _lib.lib()
    assert L.ce_version().decode().startswith("clipembed")
    assert isinstance(L.ce_last_error(), bytes)


def _cfg(**kw):
    c = _lib.Config()
    c.embed_dim, c.activation, c.image_size, c.patch_size = 768, 0, 336, 14
    c.vision = _lib.TowerConfig(1024, 24, 16, 4096)
    c.context_length, c.vocab_size = 77, 49408
    c.text = _lib.TowerConfig(768, 12, 12, 3072)
    c.pacl_dim = 0
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.mark.parametrize("bad,msg", [
    (dict(vision=_lib.TowerConfig(1000, 24, 16, 4096)), b"tower widths"),
    (dict(image_size=300), b"multiple of patch_size"),
    (dict(activation=7), b"unknown activation"),
    (dict(pacl_dim=100), b"pacl_dim"),
])
def test_create_rejects_bad_config(bad, msg):
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.ce_create(ctypes.byref(_cfg(**bad)), 0, ctypes.byref(h))
    assert rc == _lib.CE_ERR_INVALID
    assert msg in L.ce_last_error()
    assert not h.value


def test_null_arguments_are_errors():
    L = _lib.lib()
    assert L.ce_create(None, 0, None) == _lib.CE_ERR_INVALID
    assert L.ce_encode_image(None, None, None, 0, 1, 0, None, None, 0) == _lib.CE_ERR_INVALID
    assert L.ce_kernel_gemm_bf16(None, None, None, 1, 64, 64, None, 0, None, None, 0) == _lib.CE_ERR_INVALID
    assert L.ce_kernel_gemm_tn_bf16(None, None, 256, None, 256, 256, 256, 64, None, 256, 0, 1.0) == _lib.CE_ERR_INVALID
    assert L.ce_set_ln_fold(None, 1, None) == _lib.CE_ERR_INVALID
    assert b"null" in L.ce_last_error()

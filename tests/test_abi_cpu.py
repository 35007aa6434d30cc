"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/tiflash_amd.h declares; calls fail cleanly (no crash) when no GPU is visible."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tiflash_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*|size_t)\s+(tfg_\w+)\s*\(", text, re.M)))


def test_header_declares_the_surface():
    syms = declared_symbols()
    for s in ("tfg_filter", "tfg_agg_consume", "tfg_join_probe", "tfg_hash_partition", "tfg_weak_hash_update",
              "tfg_cmp_const", "tfg_arith"):
        assert s in syms
    assert len(syms) >= 40


def test_library_exports_every_declared_symbol(tfa):
    lib = tfa.lib()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", tfa.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (tfg_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_header_compiles_as_c():
    src = '#include "tiflash_amd.h"\nint main(void){ return TFG_OK; }\n'
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-x", "c", "-",
                        "-o", "/dev/null"], input=src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_errors_without_device(tfa):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    lib = tfa.lib()
    h = ctypes.c_void_p()
    rc = lib.tfg_ctx_create(0, None, ctypes.byref(h))
    assert rc == tfa.TFG_ERR_NO_DEVICE
    assert b"device" in lib.tfg_last_error()
    assert lib.tfg_type_width(tfa.DECIMAL128) == 16
    assert lib.tfg_type_width(99) == 0


def test_null_arguments_rejected_without_gpu(tfa):
    lib = tfa.lib()
    assert lib.tfg_filter(None, None, ctypes.c_int64(10), 0, None, None, None, None, None) == -1
    assert lib.tfg_agg_consume(None, None, None, None, None, None, ctypes.c_int64(1)) == -1
    assert lib.tfg_join_stats(None, None, None) == -1

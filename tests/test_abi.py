"""CPU: the C-ABI library loads, exports every symbol include/tadpole_hip.h
declares, and fails loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re

import numpy as np
import pytest

from tadpole_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "tadpole_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tp_[a-z_]+)\s*\(", txt)))


def test_header_symbols_exported():
    L = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.EXPORTS)


def test_version_and_status_codes():
    L = _lib.load()
    assert L.tp_version() == 2
    txt = open(os.path.join(ROOT, "include", "tadpole_hip.h")).read()
    for name, val in [("TP_OK", 0), ("TP_ERR_ARG", 1), ("TP_ERR_HIP", 2), ("TP_ERR_NO_BSTICK", 3),
                      ("TP_ERR_CAPACITY", 4), ("TP_ERR_NUMERIC", 5), ("TP_ERR_UNSUPPORTED", 6), ("TP_ERR_INTERNAL", 7)]:
        assert re.search(rf"{name}\s*=\s*{val}\b", txt)
        assert getattr(_lib, name) == val


def test_no_cpu_fallback_without_gpu():
    L = _lib.load()
    if L.tp_device_count() > 0:
        pytest.skip("a GPU is present")
    import tadpole_amd as tp
    with pytest.raises(tp.TadpoleError) as e:
        tp.TADpole(np.eye(8) + 1.0)
    assert e.value.status == _lib.TP_ERR_HIP
    assert "no HIP device" in str(e.value)


def test_r_error_message_entry():
    L = _lib.load()
    buf = ctypes.create_string_buffer(64)
    arr = (ctypes.c_char_p * 1)(ctypes.cast(buf, ctypes.c_char_p))
    n = ctypes.c_int(64)
    L.tp_last_error_r(arr, ctypes.byref(n))   # must not crash; fills a caller buffer

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


def test_run_time_switch_table():
    """tp_debug_knob (no GPU work): the 13 run-time switches and the four test
    hooks are accepted and return their previous value; the switches of
    earlier rounds, now compile-time constants (round 6), are refused with
    TP_ERR_ARG; knob 36 takes only the product kernels that remain."""
    switches = {1: 0, 5: 1, 8: 4096, 18: 1, 20: -1, 24: 1, 36: 5, 43: 2, 44: 1, 45: 1, 48: 0, 49: 3, 52: 3}
    for which, default in switches.items():
        assert _lib.debug_knob(which, default) == default, which
    for hook in (25, 30, 41, 51):
        old = _lib.debug_knob(hook, 0)
        _lib.debug_knob(hook, old)
    for gone in (0, 2, 3, 4, 6, 7, 9, 16, 17, 19, 28, 29, 32, 33, 34, 35, 37, 38, 39, 40, 46, 47, 50):
        with pytest.raises(Exception, match="unknown knob"):
            _lib.debug_knob(gone, 0)
    with pytest.raises(Exception, match="knob 36"):
        _lib.debug_knob(36, 2)
    assert _lib.debug_knob(36, 5) == 5

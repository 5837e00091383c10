"""ctypes binding of libtadpole_hip.so (include/tadpole_hip.h).

The library is the product: there is no CPU path behind it.  Loading fails
loudly when the shared object is missing; calls fail with TadpoleError when no
HIP device is present.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TADPOLE_LIB") or os.path.join(_HERE, "libtadpole_hip.so")   # override: debugging builds

TP_OK, TP_ERR_ARG, TP_ERR_HIP, TP_ERR_NO_BSTICK, TP_ERR_CAPACITY, TP_ERR_NUMERIC, TP_ERR_UNSUPPORTED, TP_ERR_INTERNAL = \
    range(8)
TP_FLAG_ROW_MAJOR = 1
TP_FLAG_CLEAN = 2
TP_FLAG_NO_MASK = 4
TP_FLAG_SHARDED = 8
TP_FLAG_SUBSET = 16
TP_FLAG_LDS_LEAN = 32
ABI_VERSION = 2   # tp_version() this binding is written for (timings_ms: 32 doubles)

#: every symbol include/tadpole_hip.h declares
EXPORTS = (
    "tp_version", "tp_device_count", "tp_shutdown", "tp_release_stream", "tp_last_error", "tp_last_error_r",
    "tp_mask", "tp_mask_dev", "tp_cor", "tp_pca", "tp_sweep", "tp_coniss", "tp_dist", "tp_ch",
    "tp_pipeline", "tp_pipeline_dev", "tp_sweep_dev", "tp_tsv_dims", "tp_read_tsv",
    "tp_comm_unique_id", "tp_comm_init", "tp_comm_destroy", "tp_set_virtual_shards", "tp_shard_plan",
    "tp_level_coords", "tp_read_tsv_dev", "tp_context_stats", "tp_progress_attach", "tp_upload_dev",
    "tp_upload_counts_dev", "tp_reserve_streams",
)


class TadpoleError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"[status {status}] {msg}")
        self.status = status


_lib = None

_I = ctypes.POINTER(ctypes.c_int)
_D = ctypes.POINTER(ctypes.c_double)
_V = ctypes.c_void_p


def load() -> ctypes.CDLL:
    """Load libtadpole_hip.so.

    One HIP runtime per process: torch-ROCm bundles its own libamdhip64.so.7
    (same SONAME as /opt/rocm's).  Importing torch first makes our DT_NEEDED
    entries bind to the runtime torch already mapped, so device pointers and
    streams from torch tensors are valid in the library.  Without torch (R,
    plain C) the library binds to /opt/rocm.
    """
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (maps torch's HIP runtime before ours)
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C tadpole_amd/csrc).  There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    L.tp_version.restype = ctypes.c_int
    L.tp_device_count.restype = ctypes.c_int
    L.tp_last_error.restype = ctypes.c_int
    L.tp_last_error.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.tp_mask.argtypes = [_D, _I, _D, _I, _I, _I, _D, _I, _I, _I]
    L.tp_cor.argtypes = [_D, _I, _I, _D, _I]
    L.tp_pca.argtypes = [_D, _I, _I, _I, _D, _D, _I]
    L.tp_sweep.argtypes = [_D, _I, _I, _I, _I, _I, _I, _D, _I, _I, _I, _I, _D, _I]
    L.tp_coniss.argtypes = [_D, _I, _I, _I, _I, _D, _I, _I]
    L.tp_dist.argtypes = [_D, _I, _I, _I, _D, _I]
    L.tp_ch.argtypes = [_D, _I, _I, _I, _I, _I, _D, _I]
    L.tp_pipeline.argtypes = [_D, _I, _I, _I, _D, _I, _I, _I, _I, _I, _I, _I, _I, _I, _D, _I, _I, _I,
                              _I, _D, _I, _D, _I]
    L.tp_pipeline_dev.argtypes = [_V, _I, _I, _I, _D, _I, _I, _V, _I, _I, _I, _I, _I, _I, _I, _D, _I,
                                  _I, _I, _I, _D, _I, _D, _I]
    _S = ctypes.POINTER(ctypes.c_char_p)
    L.tp_tsv_dims.argtypes = [_S, _I, _I, _I]
    L.tp_read_tsv.argtypes = [_S, _I, _I, _I, _I, _D, _I]
    L.tp_sweep_dev.argtypes = [_V, _I, _I, _I, _I, _V, _I, _I, _D, _I, _I, _I, _D, _D, _I]
    L.tp_release_stream.argtypes = [_I, _V, _I]
    L.tp_comm_unique_id.argtypes = [ctypes.c_char_p, _I]
    L.tp_comm_init.argtypes = [ctypes.c_char_p, _I, _I, _I, _I]
    L.tp_comm_destroy.argtypes = [_I]
    L.tp_set_virtual_shards.argtypes = [_I, _I, _I]
    L.tp_shard_plan.argtypes = [_I, _I, _I, _I, _I]
    L.tp_level_coords.argtypes = [_I, _I, _I, _I, _I, _I, _I]
    L.tp_read_tsv_dev.argtypes = [_S, _I, _I, _I, _I, _V, _V, _I]
    L.tp_context_stats.argtypes = [_I, _I, _I, _I]
    L.tp_progress_attach.argtypes = [_I, _V, _V, _I]
    L.tp_upload_dev.argtypes = [_V, ctypes.POINTER(ctypes.c_longlong), _V, _I, _I, _V, _I]
    L.tp_upload_counts_dev.argtypes = [_V, ctypes.POINTER(ctypes.c_longlong), _V, _I, _I, _V,
                                       ctypes.POINTER(ctypes.c_longlong), _I]
    if L.tp_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI version {L.tp_version()}, this binding needs {ABI_VERSION} (rebuild)")
    _lib = L
    return L


def last_error() -> str:
    L = load()
    buf = ctypes.create_string_buffer(1024)
    L.tp_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def check(status: ctypes.c_int):
    if status.value != TP_OK:
        raise TadpoleError(status.value, last_error())


def ip(x):
    """int* to a scalar c_int or an int32 ndarray (None -> NULL)."""
    if x is None:
        return None
    if isinstance(x, ctypes.c_int):
        return ctypes.pointer(x)
    assert x.dtype == np.int32 and (x.flags["C_CONTIGUOUS"] or x.flags["F_CONTIGUOUS"])
    return x.ctypes.data_as(_I)



def dp(x):
    if x is None:
        return None
    if isinstance(x, ctypes.c_double):
        return ctypes.pointer(x)
    assert x.dtype == np.float64
    return x.ctypes.data_as(_D)


def cint(v: int) -> ctypes.c_int:
    return ctypes.c_int(int(v))


def cdbl(v: float) -> ctypes.c_double:
    return ctypes.c_double(float(v))


def release_stream(stream, device: int = None) -> None:
    """tp_release_stream: free the library context (scratch buffers) of a
    caller stream -- a torch.cuda.Stream or a raw hipStream_t handle.  Safe
    while a call on it is still running (that call keeps it until it returns).
    The library also retires the least recently used idle stream context once
    a device has TP_MAX_STREAM_CONTEXTS of them (default 8)."""
    handle = int(getattr(stream, "cuda_stream", stream))
    if device is None:
        dev = getattr(stream, "device", None)
        device = dev.index if getattr(dev, "index", None) is not None else 0
    L = load()
    st = ctypes.c_int(0)
    L.tp_release_stream(ctypes.byref(ctypes.c_int(int(device))), ctypes.c_void_p(int(handle)), ctypes.byref(st))
    check(st)


def reserve_streams(streams, device: int = 0) -> None:
    """tp_reserve_streams: size the library contexts of these caller streams
    (torch.cuda.Stream or raw handles) alike -- every scratch buffer of each
    grows to that buffer's largest size over the set."""
    hs = [int(getattr(x, "cuda_stream", x)) for x in streams]
    arr = (ctypes.c_void_p * len(hs))(*hs)
    L = load()
    st = ctypes.c_int(0)
    L.tp_reserve_streams(ctypes.byref(ctypes.c_int(int(device))), arr, ctypes.byref(ctypes.c_int(len(hs))),
                         ctypes.byref(st))
    check(st)


def context_stats(device: int = 0):
    """tp_context_stats: (caller-stream contexts kept now, contexts created on
    ``device`` since the library was loaded)."""
    L = load()
    live, created, st = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    L.tp_context_stats(ctypes.byref(ctypes.c_int(int(device))), ctypes.byref(live), ctypes.byref(created),
                       ctypes.byref(st))
    check(st)
    return live.value, created.value


def debug_knob(which: int, value: int) -> int:
    """tp_debug_knob: set a library tuning switch (or, for 41, read and reset
    the scratch-regrowth counter); returns the previous value."""
    L = load()
    old, st = ctypes.c_int(0), ctypes.c_int(0)
    L.tp_debug_knob(ctypes.byref(ctypes.c_int(int(which))), ctypes.byref(ctypes.c_int(int(value))), ctypes.byref(old),
                    ctypes.byref(st))
    check(st)
    return old.value

"""Host -> device upload rates on this box: torch pinned -> device (raw DMA),
torch pageable .to(device), tp_upload_dev (pinned ring) on one stream, and
tp_upload_dev from 8 threads on 8 streams at once.
python tools/upload_bw.py [MB per matrix]"""
import ctypes
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
MB = int(sys.argv[1]) if len(sys.argv) > 1 else 800
n = MB * (1 << 20) // 8
host = np.random.default_rng(0).integers(0, 1000, n).astype(np.float64)
dev = torch.empty(n, dtype=torch.float64, device="cuda:0")


def upload(h, d, stream, th=1):
    st = ctypes.c_int(0)
    L.tp_upload_dev(ctypes.c_void_p(h.ctypes.data), ctypes.byref(ctypes.c_longlong(h.nbytes)),
                    ctypes.c_void_p(d.data_ptr()), ctypes.byref(ctypes.c_int(th)), ctypes.byref(ctypes.c_int(0)),
                    ctypes.c_void_p(stream.cuda_stream), ctypes.byref(st))
    _lib.check(st)


def rate(label, fn, nbytes, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    print(f"{label}: {nbytes / t / 1e9:.1f} GB/s ({t * 1e3:.1f} ms)", flush=True)


pin = torch.empty(n, dtype=torch.float64).pin_memory()
pin.numpy()[:] = host
rate("pinned -> device (torch)", lambda: dev.copy_(pin, non_blocking=True), host.nbytes)
rate("pageable -> device (torch .copy_)", lambda: dev.copy_(torch.from_numpy(host)), host.nbytes)
s0 = torch.cuda.Stream()
for th in (1, 4, 8):
    rate(f"tp_upload_dev 1 stream, {th} threads", lambda: upload(host, dev, s0, th), host.nbytes)
hosts = [host.copy() for _ in range(8)]
devs = [torch.empty(n, dtype=torch.float64, device="cuda:0") for _ in range(8)]
streams = [torch.cuda.Stream() for _ in range(8)]


def par(fn_one):
    ths = [threading.Thread(target=fn_one, args=(i,)) for i in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()


rate("tp_upload_dev 8 streams x 1 thread", lambda: par(lambda i: upload(hosts[i], devs[i], streams[i], 1)), 8 * host.nbytes, 2)
rate("tp_upload_dev 8 streams x 2 threads", lambda: par(lambda i: upload(hosts[i], devs[i], streams[i], 2)), 8 * host.nbytes, 2)
pins = []
for i in range(8):
    p = torch.empty(n, dtype=torch.float64).pin_memory()
    p.numpy()[:] = hosts[i]
    pins.append(p)


def dma8():
    for i in range(8):
        with torch.cuda.stream(streams[i]):
            devs[i].copy_(pins[i], non_blocking=True)


rate("pinned -> device, 8 streams (torch)", dma8, 8 * host.nbytes, 2)

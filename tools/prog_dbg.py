import sys, time, threading, ctypes
sys.path.insert(0, '/root/repo')
import numpy as np, torch
import tadpole_amd as tp
from tadpole_amd import _lib
from tadpole_amd.synth import synth_hic_par
m = synth_hic_par(8000, 5)
s = torch.cuda.Stream()
L = _lib.load()
prog = np.zeros(1, np.int32)
st = _lib.cint(0)
L.tp_progress_attach(ctypes.byref(_lib.cint(0)), ctypes.c_void_p(s.cuda_stream), prog.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
_lib.check(st)
seen = []
done = [False]
def run():
    tp.TADpole(torch.from_numpy(m).cuda(), stream=s)
    done[0] = True
t0 = time.perf_counter()
th = threading.Thread(target=run); th.start()
last = -1
while not done[0]:
    v = int(prog[0])
    if v != last:
        seen.append((round(time.perf_counter() - t0, 4), v)); last = v
    time.sleep(1e-4)
th.join()
print("seen", seen, "final", int(prog[0]))

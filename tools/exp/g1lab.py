"""g1dw4 laboratory driver (diagnostics): times tools/exp/libg1lab.so's switch
variants of the product g1dw4 kernel at the bench's size (2048 ROIs), interleaved."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libg1lab.so"))
P = ctypes.c_void_p
L.lab_g1.argtypes = [ctypes.c_int, P, ctypes.c_int64, P, ctypes.c_int64, P, P, P]
dev = torch.device("cuda:0")
M, N = 2048 * 100, 1024
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1 = (torch.randn(N, 512, device=dev, generator=g) / 22).bfloat16()
wdw = torch.randn(25, N, device=dev, generator=g) / 5
Y2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
flags = [int(f) for f in (sys.argv[1:] or ["0", "1", "2", "3", "10", "18"])]
names = {0: "full", 1: "full, A L2-resident", 2: "K loop only", 3: "K loop only, A L2-resident",
         10: "K loop DMA only", 4: "full, no Y2 stores", 32: "no depthwise FMAs (copy)", 64: "K loop + Y1 to LDS", 128: "stores to one L2-resident tile", 129: "stores to one tile, A same", 18: "K loop MFMA only", 19: "MFMA only, A same"}
res = {f: [] for f in flags}
for rep in range(4):
    for f in flags:
        for _ in range(3):
            assert L.lab_g1(f, P(X.data_ptr()), M, P(W1.data_ptr()), N, P(wdw.data_ptr()), P(Y2.data_ptr()), st) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            L.lab_g1(f, P(X.data_ptr()), M, P(W1.data_ptr()), N, P(wdw.data_ptr()), P(Y2.data_ptr()), st)
        e1.record()
        torch.cuda.synchronize()
        if rep > 0:
            res[f].append(e0.elapsed_time(e1) / 10 * 1e3)
for f in flags:
    v = sorted(res[f])
    print(f"{f:3d} {names.get(f, '?'):32s} median {v[len(v) // 2]:7.1f} us  min {v[0]:7.1f}")

"""gemm4 laboratory driver (diagnostics): times tools/exp/libg4lab.so's switch variants
of the product gemm4 DSC / transition tiles at the bench's size (2048 ROIs), interleaved.
usage: python tools/exp/g4lab.py dsc|trans flags..."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libg4lab.so"))
P = ctypes.c_void_p
i64 = ctypes.c_int64
L.lab_dsc.argtypes = [ctypes.c_int, P, i64, i64, P, P, P, P, P]
L.lab_trans.argtypes = [ctypes.c_int, P, i64, i64, P, P, P, P, P]
dev = torch.device("cuda:0")
R, Pr = 2048, 100
M = R * Pr
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
W2 = (torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16()
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
b = torch.randn(1024, device=dev, generator=g) / 10
s = torch.rand(R, 512, device=dev, generator=g)
C = torch.empty(M, 1024, device=dev, dtype=torch.bfloat16)
sums = torch.empty(R * 3 * 1024, device=dev, dtype=torch.int64)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
kern = sys.argv[1]
flags = [int(f) for f in sys.argv[2:]]
names = {0: "full", 1: "A L2-resident", 2: "K loop only", 3: "K loop only, A L2", 10: "K loop DMA only",
         18: "K loop MFMA only", 32: "full + A prefetch", 34: "K loop only + A prefetch",
         64: "no activation", 128: "no ROI sums", 256: "no output stores", 192: "no act, no sums",
         448: "no act, no sums, no stores"}


def run(f):
    if kern == "dsc":
        return L.lab_dsc(f, P(A.data_ptr()), M, Pr, P(W2.data_ptr()), P(b.data_ptr()), P(C.data_ptr()),
                         P(sums.data_ptr()), st)
    return L.lab_trans(f, P(A.data_ptr()), M, Pr, P(s.data_ptr()), P(Wt.data_ptr()), P(b.data_ptr()),
                       P(sums.data_ptr()), st)


res = {f: [] for f in flags}
for rep in range(4):
    for f in flags:
        for _ in range(3):
            assert run(f) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run(f)
        e1.record()
        torch.cuda.synchronize()
        if rep > 0:
            res[f].append(e0.elapsed_time(e1) / 10 * 1e3)
for f in flags:
    v = sorted(res[f])
    print(f"{kern} {f:3d} {names.get(f, '?'):28s} median {v[len(v) // 2]:7.1f} us  min {v[0]:7.1f}")

import ctypes, os, torch, json
H = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(H, "libdw_exp.so"))
L.dw_run.restype = ctypes.c_float
L.dw_run.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3
dev = torch.device("cuda:0")
K, C = 2048, 1024
x = torch.randn(K, 10, 10, C, device=dev).bfloat16()
w = torch.randn(25, C, device=dev)
y = torch.empty_like(x)
byt = 2 * x.numel() * 2
for rnd in range(2):
    for m, r, d in [(0, 16, 1), (1, 16, 1), (2, 16, 1), (3, 16, 1), (0, 4, 1), (0, 64, 1), (0, 16, 2), (0, 32, 2),
                    (0, 64, 3), (1, 16, 2), (3, 16, 2)]:
        t = L.dw_run(m, r, d, x.data_ptr(), w.data_ptr(), y.data_ptr(), K, C, 20)
        if rnd == 1:
            print(json.dumps({"mode": m, "rois": r, "depth": d, "us": round(t, 1), "GBps": round(byt / t / 1e3, 1)}))
# --- 2-row blocked variants, checked against the 1-row experiment kernel output
L2 = ctypes.CDLL(os.path.join(H, "libdw2_exp.so"))
L2.dw2_run.restype = ctypes.c_float
L2.dw2_run.argtypes = [ctypes.c_int] * 2 + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3
L.dw_run(0, 16, 1, x.data_ptr(), w.data_ptr(), y.data_ptr(), K, C, 1)
ref = y.clone()
for rnd in range(2):
    for bf, r in [(1, 16), (1, 32), (1, 64), (0, 16), (0, 32), (0, 64)]:
        y.zero_()
        t = L2.dw2_run(bf, r, x.data_ptr(), w.data_ptr(), y.data_ptr(), K, C, 20)
        if rnd == 1:
            print(json.dumps({"v": "2row", "bf16tile": bf, "rois": r, "us": round(t, 1),
                              "GBps": round(byt / t / 1e3, 1), "same": bool(torch.equal(y, ref))}))

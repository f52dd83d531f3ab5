import ctypes, os, torch, json, sys
H = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(H, "libgemm_exp.so"))
L.gemm_run.restype = ctypes.c_float
L.gemm_run.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4
dev = torch.device("cuda:0")
torch.manual_seed(0)
for (M, N, K) in [(204800, 512, 512), (204800, 1024, 512), (204800, 512, 1024)]:
    A = torch.randn(M, K, device=dev).bfloat16()
    B = (torch.randn(N, K, device=dev) / 20).bfloat16()
    bias = torch.randn(N, device=dev)
    ref = (A.float() @ B.float().t() + bias)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    # hipBLASLt via torch for reference timing
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    Bt = B.t()
    torch.addmm(bias.bfloat16(), A, Bt)
    e0.record(st)
    for _ in range(10):
        torch.addmm(bias.bfloat16(), A, Bt)
    e1.record(st); torch.cuda.synchronize()
    tb = e0.elapsed_time(e1) / 10 * 1e3
    fl = 2.0 * M * N * K
    print(json.dumps({"shape": [M, N, K], "impl": "hipblaslt", "us": round(tb, 1), "TFLOPs": round(fl / tb / 1e6, 1)}))
    for bn, epi, bk, sw in [(128, 0, 32, 0), (128, 0, 32, 1), (128, 2, 32, 0), (128, 0, 64, 0), (128, 0, 64, 1),
                            (128, 2, 64, 0), (256, 0, 32, 1), (256, 2, 32, 0), (256, 0, 64, 1), (256, 2, 64, 0)]:
        C.zero_()
        t = L.gemm_run(bn, epi, bk, sw, A.data_ptr(), B.data_ptr(), bias.data_ptr(), C.data_ptr(), M, N, K, 10)
        err = (C.float() - ref).abs().max().item() / ref.abs().max().item() if epi != 2 else None
        print(json.dumps({"shape": [M, N, K], "bn": bn, "epi": epi, "bk": bk, "swap": sw, "us": round(t, 1),
                          "TFLOPs": round(fl / t / 1e6, 1), "relerr": err}))

import ctypes, os, torch, json
H = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(H, "libgemm2_exp.so"))
L.gemm2_run.restype = ctypes.c_float
L.gemm2_run.argtypes = [ctypes.c_int] * 2 + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4
L1 = ctypes.CDLL(os.path.join(H, "libgemm_exp.so"))
L1.gemm_run.restype = ctypes.c_float
L1.gemm_run.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4
dev = torch.device("cuda:0")
torch.manual_seed(0)
for (M, N, K) in [(204800, 512, 512), (204800, 1024, 512), (204800, 512, 1024)]:
    A = torch.randn(M, K, device=dev).bfloat16()
    B = (torch.randn(N, K, device=dev) / 20).bfloat16()
    bias = torch.randn(N, device=dev)
    ref = (A.float() @ B.float().t() + bias)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    t = L1.gemm_run(128, 2, 32, 0, A.data_ptr(), B.data_ptr(), bias.data_ptr(), C.data_ptr(), M, N, K, 10)
    print(json.dumps({"shape": [M, N, K], "impl": "regstage_bn128_noepi", "us": round(t, 1), "TFLOPs": round(fl / t / 1e6, 1)}))
    for bn, epi in [(128, 2), (128, 0), (256, 2), (256, 0)]:
        C.zero_()
        t = L.gemm2_run(bn, epi, A.data_ptr(), B.data_ptr(), bias.data_ptr(), C.data_ptr(), M, N, K, 10)
        err = (C.float() - ref).abs().max().item() / ref.abs().max().item() if epi == 0 else None
        print(json.dumps({"shape": [M, N, K], "impl": f"glds_bn{bn}_epi{epi}", "us": round(t, 1),
                          "TFLOPs": round(fl / t / 1e6, 1), "relerr": err}))

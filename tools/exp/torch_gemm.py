"""hipBLASLt (torch.mm) bf16 times for the encoder GEMM shapes, for comparison
with the hand-written kernels (tools/exp only; not part of the product)."""
import torch, json
dev = torch.device("cuda")
R = 204800
for (M, K, N) in [(R, 512, 1024), (R, 1024, 1024), (R, 512, 512), (R, 1024, 512)]:
    A = torch.randn(M, K, device=dev).bfloat16(); B = torch.randn(N, K, device=dev).bfloat16()
    for _ in range(3): C = A @ B.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(10): C = A @ B.t()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    print(json.dumps(dict(M=M, K=K, N=N, us=round(us, 1), tflops=round(2 * M * N * K / us / 1e6, 1))))

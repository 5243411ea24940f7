"""Reference point: PyTorch-ROCm (hipBLASLt) fp16 GEMM of config 2's shape, random data,
and the reference's own fake-quant forward run through PyTorch on the GPU is NOT used here
(the reference cannot travel); this is only the vendor dense-GEMM ceiling for the shape."""
import torch

M, K, N = 16384, 4096 + 448, 4096
for k in (4096, K):
    a = torch.randn(M, k, device="cuda", dtype=torch.float16)
    w = torch.randn(N, k, device="cuda", dtype=torch.float16) * 0.02
    for _ in range(20):
        y = a @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        y = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 100
    print(f"torch fp16 GEMM {M}x{k}x{N}: {ms:.4f} ms, {2 * M * N * k / ms / 1e9:.1f} TFLOP/s")

"""Library bf16 GEMM rate (torch.matmul -> hipBLASLt) on the BERT encoder shapes, as the
yardstick for k_gemm3 (tokens M = 256 x 100; QKV, attention output, FFN1, FFN2)."""
import torch

M = 25600
for name, N, K in (("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    for epi in ("plain", "bias"):
        f = (lambda: a @ w.t()) if epi == "plain" else (lambda: torch.addmm(b, a, w.t()))
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name} {epi}: {us:.1f} us, {2 * M * N * K / us / 1e6:.0f} TF/s", flush=True)

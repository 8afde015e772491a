"""Library GEMM rate (torch.matmul -> hipBLASLt) on the BERT encoder shapes, as the
yardstick for k_gemm3 / k_gemm2_f32 (tokens M = 256 x 100; QKV, attention output,
FFN1, FFN2). Usage: python tools/blas_probe.py [bf16|f32] (f32: exact fp32, the
reference's arithmetic; no TF32 path exists on gfx950 and it is disabled here)."""
import sys

import torch

dt = {"bf16": torch.bfloat16, "f32": torch.float32}[sys.argv[1] if len(sys.argv) > 1 else "bf16"]
torch.backends.cuda.matmul.allow_tf32 = False
M = 25600
for name, N, K in (("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)):
    a = torch.randn(M, K, device="cuda", dtype=dt)
    w = torch.randn(N, K, device="cuda", dtype=dt)
    b = torch.randn(N, device="cuda", dtype=dt)
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
        print(f"{str(dt)[6:]} {name} {epi}: {us:.1f} us, {2 * M * N * K / us / 1e6:.0f} TF/s", flush=True)

"""Vendor-library reference for the matcher's GEMM shapes (config 2, one frame): torch.mm on
ROCm (hipBLASLt / rocBLAS) in fp32, timed with HIP events, vs our kernels' alone times."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda", 0)
shapes = {"qkv (M5120 N768 K256)": (5120, 768, 256), "mlp1 (M5120 N512 K512)": (5120, 512, 512),
          "mlp2 (M5120 N256 K512)": (5120, 256, 512), "score (M1024 N4096 K256)": (1024, 4096, 256),
          "big (M8192 N8192 K8192)": (8192, 8192, 8192)}
for name, (M, N, K) in shapes.items():
    a = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev)
    for _ in range(5):
        y = a @ w.t()
    torch.cuda.synchronize()
    it = 5 if M == 8192 else 200
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        y = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / it * 1e3
    print(f"{name:28s} {us:9.2f} us  {2 * M * N * K / us * 1e-6:7.1f} TF/s", flush=True)

"""hipBLASLt (torch.mm) bf16 yardstick at the implicit-GEMM shapes of ResNet-50 b256 convs."""
import torch
shapes = [  # (name, M, N, K)
    ("56x56 1x1 64->256", 256 * 3136, 256, 64),
    ("56x56 3x3 64->64", 256 * 3136, 64, 576),
    ("28x28 3x3 128", 256 * 784, 128, 1152),
    ("14x14 3x3 256", 256 * 196, 256, 2304),
    ("7x7 3x3 512", 256 * 49, 512, 4608),
    ("28x28 1x1 128->512", 256 * 784, 512, 128),
    ("14x14 1x1 256->1024", 256 * 196, 1024, 256),
    ("14x14 1x1 1024->256", 256 * 196, 256, 1024),
    ("7x7 1x1 512->2048", 256 * 49, 2048, 512),
    ("7x7 1x1 2048->512", 256 * 49, 512, 2048),
    ("square 8192", 8192, 8192, 8192),
]
for name, M, N, K in shapes:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        c = a @ b
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    print(f"{name:24s} M={M:7d} N={N:5d} K={K:5d} {us:8.1f} us {2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)

"""Calibration: torch.bmm (hipBLASLt/rocBLAS fp32) at the conv layers' GEMM
shapes (batch = K clients), to compare with the flr conv kernels' TF/s.
usage: gemm_calib.py"""
import torch

K = 128
SHAPES = [  # name, M, N, R (C[M,N] = A[M,R] B[R,N])
    ("l1 fwd", 64, 2048, 576), ("l1 wgrad", 576, 64, 2048),
    ("l2b fwd", 128, 512, 1152), ("l2b wgrad", 1152, 128, 512),
    ("l3b fwd", 256, 128, 2304), ("l3b wgrad", 2304, 256, 128),
    ("l4b fwd", 512, 32, 512), ("l4b wgrad", 512, 512, 32),
    ("stem fwd", 64, 8192, 148), ("stem wgrad", 64, 148, 8192),
]
for name, M, N, R in SHAPES:
    a = torch.randn(K, M, R, device="cuda")
    b = torch.randn(K, R, N, device="cuda")
    c = torch.bmm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.bmm(a, b, out=c)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 100
    print(f"{name:10s} M={M:5d} N={N:5d} R={R:5d}  {us:8.1f} us  {2.0 * K * M * N * R / us / 1e6:6.1f} TF/s", flush=True)

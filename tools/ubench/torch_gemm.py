"""Calibration (tool, not product): hipBLASLt bf16 GEMM rate (torch.matmul) on the
lifter's layer shapes at B = 8192 windows (TORCH_GEMM_B=65536 for the config-4 batch), for
comparison with the conv-GEMM kernels.  Under rocprofv3 --kernel-trace the kernel names show
hipBLASLt's tile configuration.  TORCH_GEMM_RELU=1: A = relu(randn), the post-ReLU operand the
block convs see (and gemm_check's VP3D_RELU_A=1): half its products are zero, which changes
the chip's power draw and so its clock."""
import os

import torch

B = int(os.environ.get("TORCH_GEMM_B", "8192"))

shapes = {  # name: (M, N, K)
    "expand": (B * 81, 1024, 128),
    "block1_k3": (B * 27, 1024, 3072),
    "block1_1x1": (B * 27, 1024, 1024),
    "block2_k3": (B * 9, 1024, 3072),
    "block3_k3": (B * 3, 1024, 3072),
}
for name, (M, N, K) in shapes.items():
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    if os.environ.get("TORCH_GEMM_RELU") == "1":
        a = torch.relu(a)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        torch.matmul(a, w.t())
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{name:12s} M={M:7d} N={N} K={K:5d}  {ms:.4f} ms  {2 * M * N * K / ms / 1e9:.1f} TFLOP/s", flush=True)

"""Measurement: back-to-back device copy time of observation-sized fp32 buffers (the floor for a kernel that
rewrites the (N, 450) observation each step).  Run on the GPU box: python tools/copy_floor.py"""
import torch
a = torch.randn(4096, 450, device="cuda:0"); b = torch.empty_like(a)
for n in (4096, 16384, 65536):
    a = torch.randn(n, 450, device="cuda:0"); b = torch.empty_like(a)
    for _ in range(20): b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200): b.copy_(a)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 200 * 1e3
    print("copy %d x 450 f32 (%.1f MB): %.2f us/copy incl. launch, %.2f TB/s r+w" % (n, a.numel() * 4 / 1e6, us, 2 * a.numel() * 4 / us / 1e6))

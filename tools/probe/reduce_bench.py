"""Micro-benchmark (tools only): the PPO learner's reductions on the GPU -- the split-K weight-gradient sum over 16
partial products (16, out, in) and the bias gradient over a 24 576-row minibatch (B, out) -- as torch.sum vs a GEMM
against a ones vector vs pairwise adds."""
import torch

dev = "cuda:0"


def t(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for (s, o, i) in [(16, 512, 450), (16, 256, 512), (16, 128, 256), (16, 12, 128)]:
    P = torch.randn(s, o, i, device=dev)
    ones = torch.ones(1, s, device=dev)

    def pair():
        x = P
        while x.shape[0] > 1:
            h = x.shape[0] // 2
            x = x[:h] + x[h:]
        return x[0]
    ref = P.sum(0)
    assert torch.allclose((ones @ P.view(s, -1)).view(o, i), ref, rtol=1e-4, atol=1e-4)
    print(f"splitK sum ({s},{o},{i}): sum(0) {t(lambda: P.sum(0)):.1f} us  ones@P {t(lambda: ones @ P.view(s, -1)):.1f} us"
          f"  pairwise {t(pair):.1f} us", flush=True)
for (n, o) in [(24576, 512), (24576, 1024), (24576, 256), (24576, 128), (24576, 12)]:
    G = torch.randn(n, o, device=dev)
    ones = torch.ones(1, n, device=dev)
    print(f"bias grad ({n},{o}): sum(0) {t(lambda: G.sum(0)):.1f} us  ones@G {t(lambda: ones @ G):.1f} us", flush=True)

"""Probe: device time of the acting pass's big bf16 GEMMs (98304 node rows)
in the layouts hipBLASLt can take: x @ W^T (W [out, in] as stored: the
fused path today), x @ WT (W^T materialised [in, out]), F.linear.
Usage: python tools/act_gemm_layouts.py"""
import torch


def t(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


N = 98304
for K, M in ((1024, 1024), (1024, 256), (256, 512)):
    x = torch.randn(N, K, device="cuda").bfloat16()
    W = torch.randn(M, K, device="cuda").bfloat16()
    WT = W.t().contiguous()
    fl = 2.0 * N * K * M
    for name, fn in (("x @ W^T", lambda: x @ W.t()), ("x @ WT ", lambda: x @ WT),
                     ("linear ", lambda: torch.nn.functional.linear(x, W))):
        us = t(fn)
        print(f"[{N} x {K}] @ [{K} x {M}]  {name}  {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")

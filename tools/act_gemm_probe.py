"""Probe: the acting pass's bf16 lin GEMMs (M = 4096 graphs x 24 nodes) in
both weight layouts (x @ W^T with W [out, in] as stored, and x @ W^T with
W^T materialised [in, out]).  Usage: python tools/act_gemm_probe.py"""
import torch


def t(fn, reps=30):
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


M = 4096 * 24
for (k, n) in ((1024, 1024), (1024, 256), (256, 512)):
    x = torch.randn(M, k, device="cuda").bfloat16()
    w = torch.randn(n, k, device="cuda").bfloat16()
    wt = w.t().contiguous()
    fl = 2.0 * M * n * k
    a = t(lambda: torch.mm(x, w.t()))
    b = t(lambda: torch.mm(x, wt))
    c = t(lambda: torch.nn.functional.linear(x, w))
    print(f"M={M} K={k} N={n}: x@W^T (stored) {a:7.1f} us ({fl / a / 1e6:6.0f} TF/s)  x@WT (contig) {b:7.1f} us "
          f"({fl / b / 1e6:6.0f} TF/s)  F.linear {c:7.1f} us", flush=True)

#!/usr/bin/env python3
"""Time the SAC update's big weight-gradient GEMM (dW = dY^T X, [6144 x 1024]
bf16 operands -> [1024 x 1024]) in a few formulations.  Usage: python tools/wgrad_probe.py"""
import torch


def bench(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    d = torch.device("cuda", 0)
    for (K, O, I) in ((6144, 1024, 1024), (6144, 256, 1024), (6144, 512, 256), (25600, 1024, 6)):
        dy = torch.randn(K, O, device=d).to(torch.bfloat16)
        x = torch.randn(K, I, device=d).to(torch.bfloat16)
        res = {"dyT@x": bench(lambda: dy.t() @ x), "(xT@dy)T": bench(lambda: (x.t() @ dy).t())}
        for S in (2, 4, 8):
            if K % S == 0:
                res[f"bmm{S}+sum"] = bench(lambda: torch.bmm(dy.view(S, K // S, O).transpose(1, 2),
                                                            x.view(S, K // S, I)).sum(0))
        try:
            res["mm out f32"] = bench(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        except Exception as ex:  # noqa: BLE001
            res["mm out f32"] = f"n/a ({type(ex).__name__})"
        res["dyT@x + cast f32"] = bench(lambda: (dy.t() @ x).float())
        print((K, O, I), {k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()

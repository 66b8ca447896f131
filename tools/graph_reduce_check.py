"""Does a HIP-graph replay of torch column reductions give the eager answer?

Captures y = x.sum(0) (the bias-gradient reduction of nn.Linear backward) for
a few shapes/dtypes, replays it with fresh inputs and compares each replay to
the eager result.  Usage: python tools/graph_reduce_check.py
"""
import torch


def check(shape, dtype, replays=6):
    x = torch.empty(shape, device="cuda", dtype=dtype)
    x.normal_()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            y = x.sum(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x.sum(0)
    worst = 0.0
    for r in range(replays):
        x.normal_()
        g.replay()
        ref = x.float().sum(0)
        err = ((y.float() - ref).abs() / (ref.abs() + 1.0)).max().item()
        fin = bool(torch.isfinite(y).all())
        worst = max(worst, err if fin else float("inf"))
    torch.cuda.synchronize()
    print(f"{str(shape):>16} {str(dtype):>16}: worst rel err over {replays} replays = {worst:.3e}", flush=True)
    return worst


def main():
    bad = 0
    for shape in [(6144, 1024), (98304, 1024), (6144, 256), (19456, 256), (256, 1024)]:
        for dtype in (torch.bfloat16, torch.float32):
            tol = 5e-2 if dtype == torch.bfloat16 else 1e-4
            bad += check(shape, dtype) > tol
    print("GRAPH REDUCE", "MISMATCH" if bad else "OK", flush=True)


if __name__ == "__main__":
    main()


def check_linear(in_f, out_f, rows, replays=6):
    """nn.Linear forward+backward under bf16 autocast, graph vs eager."""
    torch.manual_seed(0)
    lin = torch.nn.Linear(in_f, out_f).cuda()
    x = torch.randn(rows, in_f, device="cuda")
    gy = torch.randn(rows, out_f, device="cuda")

    def step():
        lin.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            y = lin(x)
        (y.float() * gy).sum().backward()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    worst = {"w": 0.0, "b": 0.0}
    for r in range(replays):
        x.normal_()
        gy.normal_()
        g.replay()
        torch.cuda.synchronize()
        gw, gb = lin.weight.grad.clone(), lin.bias.grad.clone()
        step()
        torch.cuda.synchronize()
        for k, a, b in (("w", gw, lin.weight.grad), ("b", gb, lin.bias.grad)):
            fin = bool(torch.isfinite(a).all())
            err = ((a - b).abs() / (b.abs() + 1.0)).max().item() if fin else float("inf")
            worst[k] = max(worst[k], err)
    print(f"linear {in_f}->{out_f} rows {rows}: worst grad rel err w {worst['w']:.3e} b {worst['b']:.3e}", flush=True)
    return max(worst.values())


if __name__ == "__main__":
    bad = 0
    for in_f, out_f, rows in [(4, 1024, 6144), (4, 1024, 98304), (1024, 1024, 6144), (256, 512, 6144),
                              (1030, 256, 19456), (256, 1, 19456)]:
        bad += check_linear(in_f, out_f, rows) > 5e-2
    print("GRAPH LINEAR", "MISMATCH" if bad else "OK", flush=True)

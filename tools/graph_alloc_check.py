"""Graph-output integrity under eager memory churn between replays.

Captures many small reductions of a parameter list (a torch.stack of 200
scalars, a python sum of scalars -- the shapes the SAC update's clipping and
diagnostics use), then between replays runs large eager allocations (like the
4096-env acting pass) and checks every replay's outputs against eager.
Usage: python tools/graph_alloc_check.py
"""
import torch


def main(churn_on=True, kind="sum"):
    torch.manual_seed(0)
    sizes = [(1024, 1024), (1024,), (256, 1024), (4, 1024), (1024, 4), (256,), (6,), (1, 256)] * 25
    params = [torch.randn(s, device="cuda") for s in sizes]

    def body():
        vec = torch.stack([(p * 2.0).abs().sum() for p in params])
        if kind == "sum":
            tot = sum((p > 0).sum() for p in params)
        else:
            tot = torch.stack([(p > 0).sum() for p in params]).sum()
        return vec, tot

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            body()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        vec, tot = body()
    bad = 0
    for r in range(8):
        for p in params:
            p.normal_()
        g.replay()
        churn = [torch.empty(100_000_000, device="cuda").fill_(float("nan")) for _ in range(4 if churn_on else 0)]
        ref_vec, ref_tot = body()
        torch.cuda.synchronize()
        okv = torch.allclose(vec, ref_vec, rtol=1e-5)
        okt = int(tot) == int(ref_tot)
        bad += not (okv and okt)
        print(f"replay {r}: vec {'ok' if okv else 'BAD'} tot {'ok' if okt else 'BAD'}", flush=True)
        del churn
    print(f"GRAPH ALLOC churn={churn_on} kind={kind}:", "MISMATCH" if bad else "OK", flush=True)


if __name__ == "__main__":
    for churn_on in (False, True):
        for kind in ("sum", "stack"):
            main(churn_on, kind)

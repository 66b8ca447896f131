"""Split-K factor of the float32 actor's weight-gradient GEMMs
(rl/fused_update.py _wgrad3: out = g^T x over the tripled 3 x 6144 contraction,
S bf16 partial products in one batched GEMM, summed in order) timed per S at
the update's shapes.  usage: python tools/wgrad3_split.py"""
import statistics

import torch


def main():
    dev = "cuda"
    K3 = 3 * 6144
    shapes = [(256, 1024), (1024, 1024), (512, 256)]   # (M = out rows, N = out cols): lin2, lin1, edge head
    for M, N in shapes:
        g = torch.randn(K3, M, device=dev).to(torch.bfloat16)
        x = torch.randn(K3, N, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev)
        res = []
        for S in (1, 2, 3, 4, 6, 8, 12, 16, 24, 36):
            if K3 % S:
                continue

            def run():
                if S == 1:
                    torch.mm(g.t(), x, out_dtype=torch.float32, out=out)
                else:
                    part = torch.bmm(g.view(S, K3 // S, M).transpose(1, 2), x.view(S, K3 // S, N),
                                     out_dtype=torch.float32)
                    torch.sum(part, 0, out=out)
            for _ in range(3):
                run()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 20 * 1e3)
            res.append((S, statistics.median(ts)))
        fl = 2.0 * M * N * K3
        print(f"M={M} N={N} K3={K3}: " + ", ".join(f"S={s}: {t:.1f} us ({fl / t / 1e6:.0f} TF/s)" for s, t in res),
              flush=True)


if __name__ == "__main__":
    main()

"""Are this library's kernels ordered within a branch of a multi-branch HIP graph?

Six side-stream branches, each a dependent chain alternating libtrafficrl
kernels (trx_bf16_round: an exact float32 copy, then the two-term bf16 split)
and torch kernels / a hipBLASLt GEMM, as the fused update's forwards
alternate them.  The static input changes before every replay; each branch's
result is compared with an eager run of the same body.

usage: python tools/trx_chain_race.py"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

N, K = 6144, 1024


def main():
    from trafficrl.models import fused
    dev = "cuda"
    torch.manual_seed(0)
    side = [torch.cuda.Stream() for _ in range(6)]
    xs = [torch.randn(N, K, device=dev) for _ in range(6)]
    ws = [torch.randn(K, K, device=dev).bfloat16() * 0.03 for _ in range(6)]

    def body():
        main_s = torch.cuda.current_stream()
        outs = []
        for k, st in enumerate(side):
            st.wait_stream(main_s)
            with torch.cuda.stream(st):
                y = torch.empty_like(xs[k])
                fused._round_into([(xs[k], y, True)])          # trx kernel: copy
                z = y * 0.5 + 1.0                               # torch kernel
                z3 = fused.split3([(z, "cols", "hhl")])[0]     # trx kernel
                hi, lo = z3[:, :K], z3[:, 2 * K:]
                g = F.linear(hi, ws[k])                         # hipBLASLt
                u = torch.empty(N, K, device=dev)
                fused._round_into([(g.float(), u, True)])       # torch cast, trx copy
                outs.append(u + lo.float())
        for st in side:
            main_s.wait_stream(st)
        for o in outs:
            o.record_stream(main_s)
        return outs

    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        body()
        body()
    torch.cuda.current_stream().wait_stream(s0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = body()
    bad = 0
    for r in range(30):
        for x in xs:
            x.add_(0.25)
        g.replay()
        torch.cuda.synchronize()
        ref = body()
        torch.cuda.synchronize()
        bad += sum(int(not torch.equal(a, b)) for a, b in zip(outs, ref))
    print(f"trx/torch/hipBLASLt chains: {bad}/180 branch outputs differ from eager", flush=True)


if __name__ == "__main__":
    main()

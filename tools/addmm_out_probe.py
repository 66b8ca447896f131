"""torch.mm / addmm(out_dtype=float32) from bf16 operands with transposed views,
and the update's three-product split GEMM (rl/fused_update.py _mm3) against a
float64 reference.  usage: python tools/addmm_out_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def main():
    from trafficrl.models import fused
    from trafficrl.rl import fused_update as FU
    torch.manual_seed(0)
    M, K, N = 640, 384, 256
    A = torch.randn(M, K, device="cuda")
    Bm = torch.randn(K, N, device="cuda")
    At = A.t().contiguous()       # [K, M]
    Bt = Bm.t().contiguous()      # [N, K]
    ref = (A.double() @ Bm.double())
    for name, a, b in (("a b", A, Bm), ("a^T' b", At.t(), Bm), ("a b^T'", A, Bt.t()), ("a^T' b^T'", At.t(), Bt.t())):
        ab, bb = a.bfloat16(), b.bfloat16()
        r = torch.mm(ab, bb, out_dtype=torch.float32)
        want = ab.double() @ bb.double()
        print(f"mm out_dtype {name:10s} max err {float((r.double() - want).abs().max()):.3e}", flush=True)
    for name, a, b in (("a b", A, Bm), ("a^T' b", At.t(), Bm), ("a b^T'", A, Bt.t()), ("a^T' b^T'", At.t(), Bt.t())):
        src_a = At if a.stride(0) == 1 else A
        src_b = Bt if b.stride(0) == 1 else Bm
        sa, sb = fused.split_bf16([src_a, src_b])
        if a.stride(0) == 1:
            sa = (sa[0].t(), sa[1].t())
        if b.stride(0) == 1:
            sb = (sb[0].t(), sb[1].t())
        r = FU._mm3(sa, sb)
        rel = float((r.double() - ref).abs().max() / ref.abs().max())
        print(f"_mm3 {name:10s} max rel err {rel:.3e}", flush=True)
    hi, lo = fused.split_bf16([A])[0]
    print("split: hi exact", bool(torch.equal(hi, A.bfloat16())), "residual rel",
          float(((hi.double() + lo.double()) - A.double()).abs().max() / A.abs().max()), flush=True)


if __name__ == "__main__":
    main()

"""torch.mm / addmm(out_dtype=float32) from bf16 operands with transposed views,
and the update's three-term split GEMM (models/fused.py split3 +
rl/fused_update.py _mm3) against a float64 reference.  usage: python tools/addmm_out_probe.py"""
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
    # the three-term operands: a [M, K] by columns ("hhl"), b [K, N] by rows ("lhh"); and the
    # transposed forms the update uses (a = x^T from x's row stack, b = W^T from W's columns)
    a3, b3 = fused.split3([(A, "cols", "hhl"), (Bm, "rows", "lhh")])
    at3, bt3 = fused.split3([(At, "rows", "hhl"), (Bt, "cols", "lhh")])
    for name, x, y in (("a3 b3", a3, b3), ("at3^T bt3^T", at3.t(), bt3.t()), ("a3 bt3^T", a3, bt3.t())):
        r = FU._mm3(x, y)
        print(f"_mm3 {name:12s} max rel err {float((r.double() - ref).abs().max() / ref.abs().max()):.3e}", flush=True)
    o = torch.empty(M, N, device="cuda")
    FU._mm3(a3, b3, out=o)
    print(f"_mm3 out=      max rel err {float((o.double() - ref).abs().max() / ref.abs().max()):.3e}", flush=True)


if __name__ == "__main__":
    main()

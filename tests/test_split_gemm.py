"""The float32 actor's building blocks (rl/fused_update.py, models/fused.py):
three-term bf16 splits (trx_bf16_round modes 1 / 3 with a destination row
stride), the tripled-contraction GEMM and its split-K weight-gradient form,
against float64; and trx_partial_sum_multi against trx_partial_sum (same
summation order: bit-identical) with a column-block destination."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_split3_pieces_exact():
    from trafficrl.models import fused
    torch.manual_seed(0)
    x = torch.randn(96, 64, device="cuda") * 3.0
    c, r = fused.split3([(x, "cols", "hhl"), (x, "rows", "lhh")])
    hi = x.bfloat16()
    lo = (x - hi.float()).bfloat16()
    assert torch.equal(c[:, :64], hi) and torch.equal(c[:, 64:128], hi) and torch.equal(c[:, 128:], lo)
    assert torch.equal(r[:96], lo) and torch.equal(r[96:192], hi) and torch.equal(r[192:], hi)
    # hi + lo carries 16 mantissa bits
    rel = float(((hi.double() + lo.double()) - x.double()).abs().max() / x.abs().max())
    assert rel < 2 ** -15


@pytest.mark.parametrize("cols", [64, 63])
def test_split3_every_order_and_layout(cols):
    """Mode 16 + bits (ABI 12): every piece order, both layouts, the vector
    path (cols % 4 == 0) and the scalar one, from a row-strided view."""
    from trafficrl.models import fused
    torch.manual_seed(3)
    base = torch.randn(50, 80, device="cuda") * 7.0
    x = base[:, 3:3 + cols] if cols % 4 else base[:, 8:8 + cols]
    hi = x.bfloat16()
    lo = (x - hi.float()).bfloat16()
    orders = ["hhh", "hhl", "hlh", "lhh", "llh", "lhl", "hll", "lll"]
    specs = [(x, lay, o) for o in orders for lay in ("cols", "rows")]
    outs = fused.split3(specs)
    for (_, lay, o), out in zip(specs, outs):
        for p, ch in enumerate(o):
            piece = out[:, p * cols:(p + 1) * cols] if lay == "cols" else out[p * 50:(p + 1) * 50]
            assert torch.equal(piece, lo if ch == "l" else hi), (lay, o, p)


def test_tripled_contraction_gemm_and_split_k():
    from trafficrl.models import fused
    from trafficrl.rl import fused_update as FU
    torch.manual_seed(1)
    x = torch.randn(6144, 256, device="cuda")
    w = torch.randn(512, 256, device="cuda") * 0.05
    x_c, x_r = fused.split3([(x, "cols", "hhl"), (x, "rows", "lhh")])
    w_c, = fused.split3([(w, "cols", "lhh")])
    y = FU._mm3(x_c, w_c.t())                       # x @ w^T
    ref = x.double() @ w.double().t()
    assert float((y.double() - ref).abs().max() / ref.abs().max()) < 2e-5
    g = torch.randn(6144, 512, device="cuda")
    g_r, = fused.split3([(g, "rows", "hhl")])
    out = torch.empty(512, 256, device="cuda")
    FU._wgrad3(g_r, x_r, out)                        # g^T x, split-K
    ref = g.double().t() @ x.double()
    assert float((out.double() - ref).abs().max() / ref.abs().max()) < 2e-5


def test_inplace_residual_addmm_bit_identical():
    """The backward's g_xh W + g_res accumulated in place (out = the addend)
    equals the copying addmm bit for bit, at the update's actor shapes."""
    from trafficrl.rl import fused_update as FU
    torch.manual_seed(4)
    FU.probe_mm32(torch.device("cuda"))
    for (n, k, m) in ((6144, 3072, 1024), (6144, 1024, 1024), (500, 96, 40)):
        a = torch.randn(n, k, device="cuda").bfloat16()
        b = torch.randn(k, m, device="cuda").bfloat16()
        add = torch.randn(n, m, device="cuda")
        ref = FU._mm32(a, b, add)
        acc = add.clone()
        got = FU._mm3(a, b, acc, out=acc)
        assert got.data_ptr() == acc.data_ptr() and torch.equal(acc, ref), (n, k, m)


def test_partial_sum_multi_matches_single():
    from trafficrl import _lib
    from trafficrl.rl.fused_update import PartialSums
    L = _lib.load()
    torch.manual_seed(2)
    B = 256
    parts = [torch.randn(B, w, device="cuda") for w in (1, 77, 256, 1030)]
    want = []
    for p in parts:
        o = torch.empty(p.shape[1], device="cuda")
        _lib.check(L.trx_partial_sum(_lib.ptr(p), B, p.shape[1], p.shape[1], _lib.ptr(o), _lib.stream_ptr()),
                   "trx_partial_sum")
        want.append(o)
    sums = PartialSums(B)
    got = [torch.empty(p.shape[1], device="cuda") for p in parts]
    for p, o in zip(parts, got):
        sums.add(p, p.shape[1], p.shape[1], o)
    # a column block of a [16, 40] matrix: 16 x 6 sums into columns 20..25
    blk = torch.randn(B, 96, device="cuda")
    mat = torch.zeros(16, 40, device="cuda")
    sums.add(blk, 96, 96, mat[:, 20:], out_cols=6, out_ld=40)
    sums.flush(_lib.stream_ptr())
    torch.cuda.synchronize()
    for a, b in zip(got, want):
        assert torch.equal(a, b)
    ref = blk.sum(0).view(16, 6)
    torch.testing.assert_close(mat[:, 20:26], ref, rtol=1e-5, atol=1e-4)
    assert float(mat[:, :20].abs().sum()) == 0 and float(mat[:, 26:].abs().sum()) == 0

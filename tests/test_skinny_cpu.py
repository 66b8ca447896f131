"""CPU checks of the update's custom autograd helpers (trafficrl/models/skinny.py):
forward values and gradients equal the plain torch ops they replace."""
import torch
import torch.nn.functional as F

from trafficrl.models.skinny import perm_gather, regular_gather, skinny_linear


def test_skinny_linear_matches_linear():
    g = torch.Generator().manual_seed(0)
    for K, i, o, bias in ((25600, 6, 4, False), (6144, 4, 64, True), (1000, 256, 1, True), (512, 6, 3, False)):
        x = torch.randn(K, i, generator=g, dtype=torch.float64, requires_grad=True)
        w = torch.randn(o, i, generator=g, dtype=torch.float64, requires_grad=True)
        b = torch.randn(o, generator=g, dtype=torch.float64, requires_grad=True) if bias else None
        dy = torch.randn(K, o, generator=g, dtype=torch.float64)
        y = skinny_linear(x, w, b)
        y.backward(dy)
        gx, gw = x.grad.clone(), w.grad.clone()
        gb = b.grad.clone() if bias else None
        x.grad = w.grad = None
        if bias:
            b.grad = None
        y2 = F.linear(x, w, b)
        y2.backward(dy)
        torch.testing.assert_close(y, y2)
        torch.testing.assert_close(gx, x.grad)
        # split-K accumulates in float32 (like the GEMM it replaces under autocast)
        torch.testing.assert_close(gw, w.grad, rtol=1e-5, atol=1e-4)
        if bias:
            torch.testing.assert_close(gb, b.grad)


def test_regular_gather_matches_index():
    g = torch.Generator().manual_seed(1)
    B, n, m, Fd = 5, 24, 76, 7
    idx = torch.randint(0, n, (m,), generator=g)
    x = torch.randn(B * n, Fd, generator=g, dtype=torch.float64, requires_grad=True)
    glob = (torch.arange(B) * n).repeat_interleave(m) + idx.repeat(B)
    dy = torch.randn(B * m, Fd, generator=g, dtype=torch.float64)
    y = regular_gather(x, idx, B)
    y.backward(dy)
    gx = x.grad.clone()
    x.grad = None
    y2 = x[glob]
    y2.backward(dy)
    torch.testing.assert_close(y, y2)
    torch.testing.assert_close(gx, x.grad)


def test_perm_gather_matches_index():
    g = torch.Generator().manual_seed(2)
    perm = torch.randperm(100, generator=g)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(100)
    x = torch.randn(100, 4, generator=g, dtype=torch.float64, requires_grad=True)
    dy = torch.randn(100, 4, generator=g, dtype=torch.float64)
    perm_gather(x, perm, inv).backward(dy)
    gx = x.grad.clone()
    x.grad = None
    x[perm].backward(dy)
    torch.testing.assert_close(gx, x.grad)

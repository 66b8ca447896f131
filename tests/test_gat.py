"""GAT path (src/models/gat_encoder.py + PyG GATConv) on the HIP kernels vs a
plain-torch restatement of torch_geometric GATConv semantics (PyG 2.5:
remove/add self loops with fill_value='mean', leaky_relu 0.2, softmax over
destination in-edges with +1e-16, concat / head mean, bias).

torch_geometric is absent from this environment, so this restatement is the
checker ("parity unpinned" w.r.t. the reference's own outputs); parameter
layout is pinned by the reference's checkpoints (test_reference_checkpoint_
layout).  Tolerance: fp32 kernels vs fp32 torch, rtol 2e-5 / atol 2e-5
(forward) and 1e-4 relative on gradients (different summation orders).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT


def ref_gatconv(conv, x, edge_index, edge_attr):
    H, C = conv.heads, conv.out_channels
    N = x.size(0)
    xh = (x @ conv.lin.weight.t()).view(N, H, C)
    a_s = (xh * conv.att_src).sum(-1)
    a_d = (xh * conv.att_dst).sum(-1)
    keep = edge_index[0] != edge_index[1]
    ei = edge_index[:, keep]
    ea = edge_attr[keep]
    cnt = torch.zeros(N, device=x.device).index_add_(0, ei[1], torch.ones(ei.size(1), device=x.device))
    loop_attr = torch.zeros(N, ea.size(1), device=x.device).index_add_(0, ei[1], ea) / cnt.clamp(min=1).unsqueeze(1)
    loops = torch.arange(N, device=x.device)
    ei = torch.cat([ei, torch.stack([loops, loops])], 1)
    ea = torch.cat([ea, loop_attr], 0)
    e = (ea @ conv.lin_edge.weight.t()).view(-1, H, C)
    a_e = (e * conv.att_edge).sum(-1)
    logit = F.leaky_relu(a_s[ei[0]] + a_d[ei[1]] + a_e, conv.negative_slope)
    amax = torch.full((N, H), float("-inf"), device=x.device).scatter_reduce(
        0, ei[1].unsqueeze(1).expand(-1, H), logit, reduce="amax", include_self=True)
    ex = torch.exp(logit - amax[ei[1]])
    ssum = torch.zeros(N, H, device=x.device).index_add_(0, ei[1], ex)
    alpha = ex / (ssum[ei[1]] + 1e-16)
    out = torch.zeros(N, H, C, device=x.device).index_add_(0, ei[1], alpha.unsqueeze(-1) * xh[ei[0]])
    out = out.reshape(N, H * C) if conv.concat else out.mean(1)
    return out + conv.bias, alpha


def batched_graph(B, device):
    z = np.load(os.path.join(ROOT, "tests", "golden", "sf_graph.npz"))
    src = torch.as_tensor(z["src"], dtype=torch.long)
    dst = torch.as_tensor(z["dst"], dtype=torch.long)
    N, E = int(z["num_nodes"]), len(src)
    off = (torch.arange(B) * N).repeat_interleave(E)
    ei = torch.stack([src.repeat(B) + off, dst.repeat(B) + off]).to(device)
    batch = torch.arange(B).repeat_interleave(N).to(device)
    return ei, batch, N, E


def test_reference_checkpoint_layout():
    """The reference's saved actor (history-data/outputs1/model_best.pt: node_in 3,
    hidden 64, embed 64, older code without LayerNorms) loads into our Actor:
    every saved key exists here with the same shape."""
    path = "/root/reference/history-data/outputs1/model_best.pt"
    if not os.path.exists(path):
        pytest.skip("reference checkpoint not present (GPU box)")
    from trafficrl.rl.sac import Actor
    sd = torch.load(path, map_location="cpu", weights_only=True)
    actor = Actor(3, 6, 64, 64, num_layers=3)
    missing, unexpected = actor.load_state_dict(sd["actor"], strict=False)
    assert unexpected == []
    assert all(k.startswith(("node_norm", "edge_norm", "encoder.norms")) for k in missing), missing
    mine = actor.state_dict()
    for k, v in sd["actor"].items():
        assert mine[k].shape == v.shape, k


@pytest.mark.gpu
@pytest.mark.parametrize("heads,out_ch,concat,in_ch", [(4, 256, True, 1024), (1, 256, False, 1024), (4, 64, True, 4),
                                                       (4, 256, True, 4)])
def test_gatconv_matches_pyg_restatement(heads, out_ch, concat, in_ch):
    from trafficrl.models import GATConv
    torch.manual_seed(0)
    dev = "cuda"
    B = 16
    ei, batch, N, E = batched_graph(B, dev)
    conv = GATConv(in_ch, out_ch, heads=heads, concat=concat, edge_dim=6).to(dev)
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    x = torch.randn(B * N, in_ch, device=dev, requires_grad=True)
    ea = torch.randn(B * E, 6, device=dev, requires_grad=True)
    out, (ei_full, alpha) = conv(x, ei, ea, return_attention_weights=True)
    ref, ref_alpha = ref_gatconv(conv, x, ei, ea)
    torch.testing.assert_close(out, ref, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(alpha, ref_alpha, rtol=2e-5, atol=1e-6)
    # gradients of a random projection of the output
    w = torch.randn_like(out)
    params = [x, ea] + list(conv.parameters())
    g1 = torch.autograd.grad((out * w).sum(), params)
    g2 = torch.autograd.grad((ref * w).sum(), params)
    for a, b in zip(g1, g2):
        scale = b.abs().max().clamp(min=1e-6)
        assert (a - b).abs().max() / scale < 1e-4


@pytest.mark.gpu
def test_gatconv_bf16_input():
    from trafficrl.models import GATConv
    torch.manual_seed(1)
    ei, batch, N, E = batched_graph(8, "cuda")
    conv = GATConv(1024, 256, heads=4, edge_dim=6).cuda()
    x = torch.randn(8 * N, 1024, device="cuda")
    ea = torch.randn(8 * E, 6, device="cuda")
    ref = conv(x, ei, ea)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = conv(x, ei, ea)
    assert out.dtype == torch.float32
    torch.testing.assert_close(out, ref, rtol=5e-2, atol=5e-2)


@pytest.mark.gpu
def test_encoder_forward_backward_shapes():
    from trafficrl.models import GATEncoder
    torch.manual_seed(2)
    B = 32
    ei, batch, N, E = batched_graph(B, "cuda")
    enc = GATEncoder(4, 256, 256, edge_dim=6, heads=4, num_layers=3).cuda()
    x = torch.randn(B * N, 4, device="cuda")
    ea = torch.randn(B * E, 6, device="cuda")
    h, ctx, attn = enc(x, ei, ea, batch, return_attention=True)
    assert h.shape == (B * N, 256) and ctx.shape == (B, 512) and attn.shape == (B * (E + N), 1)
    (h.sum() + ctx.sum()).backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in enc.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize("act,res_dtype,F", [(0, torch.float32, 1024), (0, torch.bfloat16, 1024), (1, None, 256),
                                             (0, torch.float32, 12)])
def test_layer_tail_matches_torch_ops(act, res_dtype, F):
    """csrc/layer_tail.hip forward and backward against the torch ops of
    GATEncoder's layer tail (bias add, LayerNorm, residual, ReLU / ELU):
    values and all five gradients to fp32 reduction-order tolerance; two
    backward runs agree bit for bit (fixed-order column sums)."""
    from trafficrl.models.gat_encoder import layer_tail
    g = torch.Generator(device="cuda").manual_seed(F + act)
    N = 6144 if F > 12 else 37
    out = torch.randn(N, F, device="cuda", generator=g, requires_grad=True)
    norm = torch.nn.LayerNorm(F).cuda()
    with torch.no_grad():
        norm.weight.copy_(1 + 0.1 * torch.randn(F, device="cuda", generator=g))
        norm.bias.copy_(0.1 * torch.randn(F, device="cuda", generator=g))
    bias = (0.1 * torch.randn(F, device="cuda", generator=g)).requires_grad_()
    res = None
    if act == 0:
        res = torch.randn(N, F, device="cuda", generator=g).to(res_dtype).requires_grad_()
    gy = torch.randn(N, F, device="cuda", generator=g)

    def run(fused):
        for t in [out, bias, norm.weight, norm.bias] + ([res] if res is not None else []):
            t.grad = None
        if fused:
            y = layer_tail(out, bias, norm, res)
        else:
            h = F_.layer_norm(out + bias, (F,), norm.weight, norm.bias, norm.eps)
            y = torch.relu(h + res) if res is not None else F_.elu(h)
        y.backward(gy)
        grads = [t.grad.clone() for t in [out, bias, norm.weight, norm.bias] + ([res] if res is not None else [])]
        return y.detach(), grads

    F_ = torch.nn.functional
    y_ref, g_ref = run(False)
    y_got, g_got = run(True)
    _, g_again = run(True)
    torch.testing.assert_close(y_got, y_ref, atol=2e-5, rtol=2e-5)
    for a, b in zip(g_got, g_ref):
        assert a.dtype == b.dtype
        tol = 2e-2 if a.dtype == torch.bfloat16 else 1e-4 * max(1.0, b.abs().max().item())
        torch.testing.assert_close(a.float(), b.float(), atol=tol, rtol=1e-3)
    for a, b in zip(g_got, g_again):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("H,C,dt", [(4, 256, torch.bfloat16), (1, 256, torch.bfloat16), (4, 64, torch.float32),
                                    (3, 12, torch.float32)])
def test_att_dots_matches_torch_ops(H, C, dt):
    """csrc/att_dots.hip against (xh.view(N,H,C).float() * att).sum(-1) and
    its autograd gradients (xh in its own dtype, att float32); backward runs
    agree bit for bit (fixed-order column sums)."""
    from trafficrl.models.gat_encoder import att_dots
    g = torch.Generator(device="cuda").manual_seed(H * C)
    N = 6144 if C >= 64 else 50
    xh = torch.randn(N, H * C, device="cuda", generator=g).to(dt).requires_grad_()
    a_s = torch.randn(1, H, C, device="cuda", generator=g).requires_grad_()
    a_d = torch.randn(1, H, C, device="cuda", generator=g).requires_grad_()
    gs, gd = torch.randn(N, H, device="cuda", generator=g), torch.randn(N, H, device="cuda", generator=g)

    def run(fused):
        for t in (xh, a_s, a_d):
            t.grad = None
        if fused:
            s, d = att_dots(xh, a_s, a_d, H, C)
        else:
            x3 = xh.float().view(N, H, C)
            s, d = (x3 * a_s).sum(-1), (x3 * a_d).sum(-1)
        (s * gs + d * gd).sum().backward()
        return s.detach(), d.detach(), xh.grad.clone(), a_s.grad.clone(), a_d.grad.clone()

    ref = run(False)
    got = run(True)
    again = run(True)
    torch.testing.assert_close(got[0], ref[0], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(got[1], ref[1], atol=1e-4, rtol=1e-4)
    assert got[2].dtype == dt
    torch.testing.assert_close(got[2].float(), ref[2].float(), atol=1e-2 if dt == torch.bfloat16 else 1e-5,
                               rtol=1e-2 if dt == torch.bfloat16 else 1e-5)
    for k in (3, 4):
        torch.testing.assert_close(got[k], ref[k], atol=2e-3 * N ** 0.5 / 10, rtol=1e-4)
    for a, b in zip(got[2:], again[2:]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("N,d", [(19456, 6), (6144, 4), (300, 8)])
def test_small_layer_norm_matches_torch(N, d):
    """csrc/small_ln.hip (input_layer_norm on the GPU) against
    torch.nn.functional.layer_norm: output and the x / weight / bias
    gradients to fp32 reduction-order tolerance; deterministic backward."""
    from trafficrl.rl.sac import input_layer_norm
    g = torch.Generator(device="cuda").manual_seed(N + d)
    x = (3 * torch.randn(N, d, device="cuda", generator=g) + 1).requires_grad_()
    ln = torch.nn.LayerNorm(d).cuda()
    with torch.no_grad():
        ln.weight.copy_(1 + 0.2 * torch.randn(d, device="cuda", generator=g))
        ln.bias.copy_(0.2 * torch.randn(d, device="cuda", generator=g))
    gy = torch.randn(N, d, device="cuda", generator=g)

    def run(fused):
        for t in (x, ln.weight, ln.bias):
            t.grad = None
        y = input_layer_norm(ln, x) if fused else F.layer_norm(x, (d,), ln.weight, ln.bias, ln.eps)
        y.backward(gy)
        return y.detach(), x.grad.clone(), ln.weight.grad.clone(), ln.bias.grad.clone()

    ref, got, again = run(False), run(True), run(True)
    torch.testing.assert_close(got[0], ref[0], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(got[1], ref[1], atol=1e-4, rtol=1e-4)
    for k in (2, 3):
        torch.testing.assert_close(got[k], ref[k], atol=1e-3 * N ** 0.5 / 10, rtol=1e-4)
    for a, b in zip(got, again):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_graph_pool_matches_torch_ops():
    """csrc/graph_pool.hip: mean | max readout and its gradient against
    view().mean / amax (ties included: ReLU outputs are often exactly 0, and
    amax's backward spreads the gradient over ties)."""
    from trafficrl.models.gat_encoder import _GraphPool
    g = torch.Generator(device="cuda").manual_seed(11)
    B, n, F_ = 256, 24, 256
    x = torch.relu(torch.randn(B * n, F_, device="cuda", generator=g)).requires_grad_()
    x.data[:n, :8] = 0.0                      # an all-zero column block: n-way ties
    gy = torch.randn(B, 2 * F_, device="cuda", generator=g)
    out = _GraphPool.apply(x, B)
    out.backward(gy)
    gx = x.grad.clone()
    x.grad = None
    xv = x.view(B, n, F_)
    ref = torch.cat([xv.mean(1), xv.amax(1)], 1)
    ref.backward(gy)
    torch.testing.assert_close(out, ref, atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(gx, x.grad, atol=1e-6, rtol=1e-6)

"""Fused SAC update (src/rl/sac.py:157-243) for the trainer's regular batches.

The general update (DiscreteSAC.compute_gradients) runs the three training
forwards through torch autograd: ~700 kernels per update at batch 256, most of
them casts, elementwise glue and small reductions of a few microseconds each.
Here every network is evaluated by the fused inference kernels
(models/fused.py, csrc/gat_infer.hip) with their save_* outputs, the three
losses and their gradients come from one kernel (trx_sac_loss), and each
network's backward is explicit: the edge scorer's backward kernel, one
trx_gat_layer_backward launch per GAT layer, one prologue backward, the
bf16 GEMMs of the lin / edge-head weights (split-K float32 weight gradients),
and trx_partial_sum for the per-column parameter gradients.  About 230
launches per update, all graph-capturable (no host synchronisation).

Numerics: the forward is the fused inference path's (bf16 roundings where
torch autocast rounds, fp32 reductions in its own order); the backward is its
exact derivative with autocast's dtype rules (gradients of bf16 tensors rounded
to bf16 once, parameter gradients float32).  tests/test_fused_update.py checks
it against the autograd path and the fp32 restatement.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from .. import _lib
from ..models import fused
from ..models.fused import Topology
from ..models.skinny import _splitk_wgrad


def exact_nets(agent) -> dict:
    """Which networks' passes run in the exact (float32) mode: every one when
    the agent trains in float32 (amp off: the reference's precision), the
    actor's two (next-state probabilities and its training pass) under bf16
    autocast with agent.fp32_actor, the actor's training pass and its backward
    (its gradient is the softmax-centred logit difference, which bf16 operands
    blur: tests/test_fused_update.py, tools/precision_sites.py)."""
    full = agent.amp_dtype is None
    actor = full or bool(getattr(agent, "fp32_actor", False))
    return {"actor": actor, "critic": full}


def supported(agent, topo: Optional[Topology]) -> bool:
    """The fused update takes regular batches of <= 32-node graphs on the GPU,
    under bf16 autocast or in float32, with the reference's network shapes."""
    if topo is None or agent.amp_dtype not in (torch.bfloat16, None) or not agent.log_alpha.is_cuda:
        return False
    ex = exact_nets(agent)
    for net in (agent.actor, agent.critic1, agent.critic2, agent.target1, agent.target2):
        enc = net.encoder
        if not (fused.encoder_supported(enc) and fused.head_supported(net) and fused.prologue_supported(net)):
            return False
        if ex["actor" if net is agent.actor else "critic"] and not fused.exact_supported(net):
            return False
        layers = list(enc.layers)
        if len(layers) != 3 or net.edge_mlp[0].weight.shape[0] > 256:
            return False
    return topo.e <= 256 and topo.n <= 32


@dataclass
class NetCtx:
    """What one network's training forward keeps for its backward."""
    x0: torch.Tensor
    ea: torch.Tensor
    a_all: torch.Tensor
    m_work: torch.Tensor
    node_x: torch.Tensor
    edge_x: torch.Tensor
    layers: List[Dict]
    emb: torch.Tensor
    ctx: torch.Tensor
    p: torch.Tensor
    c: torch.Tensor
    head_w: tuple
    grp: Optional["NetGroup"] = None   # net_forward_multi: the stacked tensors of the group
    j: int = 0                         # this network's index in the group


@dataclass
class NetGroup:
    """The stacked ([k, ...], network-major) tensors of one net_forward_multi
    call that the GEMMs of net_backward_multi read."""
    x_in: List[torch.Tensor]   # per layer >= 1: its GEMM input [k, N, in] bf16
    W: List[torch.Tensor]      # per layer >= 1: its lin weights [k, out, in] bf16
    emb: torch.Tensor          # [k, N, embed] bf16
    ctx: torch.Tensor          # [k, B, 2 embed] float32
    WN: torch.Tensor           # [k, 2 hidden, embed] bf16 edge-MLP node blocks
    WC: torch.Tensor           # [k, hidden, 2 embed] bf16 edge-MLP context block


_MM32 = [None]   # torch.mm(..., out_dtype=torch.float32) available on this build (probe_mm32)


def probe_mm32(device) -> bool:
    """Probe torch.mm(bf16, bf16, out_dtype=float32) once, eagerly (DiscreteSAC
    construction): the first update may run inside a graph capture, where a
    failing probe call cannot be made."""
    if _MM32[0] is None:
        try:
            a = torch.zeros(2, 2, device=device, dtype=torch.bfloat16)
            _MM32[0] = torch.mm(a, a, out_dtype=torch.float32).dtype == torch.float32
        except (RuntimeError, TypeError):
            _MM32[0] = False
    return _MM32[0]


def _mm32(a: torch.Tensor, b: torch.Tensor, add: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a @ b (+ add) from bf16 operands with the float32 accumulator as the
    result (no bf16 rounding of the product: the update's gradients flow in
    fp32 between the layer kernels, and no cast kernel runs).  Without
    out_dtype support: a float32 GEMM of the same bf16 values (exact products,
    float32 sums) -- never a bf16-rounded product."""
    if _MM32[0] is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("fused_update.probe_mm32 must run before the update is captured")
        probe_mm32(a.device)
    if _MM32[0]:
        if add is None:
            return torch.mm(a, b, out_dtype=torch.float32)
        return torch.addmm(add, a, b, out_dtype=torch.float32)
    r = torch.mm(a.float(), b.float())
    return r if add is None else r + add


def _mm3(a3: torch.Tensor, b3: torch.Tensor, add: Optional[torch.Tensor] = None,
         out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a @ b (+ add) to ~float32 accuracy as ONE bf16 GEMM over a tripled
    contraction: a3 holds a's three-term pieces in order "hhl", b3 b's in
    order "lhh" (models/fused.py split3), so a3 @ b3 = a_hi b_lo + a_hi b_hi +
    a_lo b_hi with float32 accumulation (the dropped a_lo b_lo and the splits'
    rounding are ~2^-16 relative; tools/addmm_out_probe.py).  gfx950 has no
    xf32 and float32 matrix throughput is 1/16 of bf16's: three bf16 products
    in one launch cost a fraction of one float32 GEMM."""
    if out is None:
        return _mm32(a3, b3, add)
    if _MM32[0] is None:
        probe_mm32(a3.device)
    if _MM32[0]:
        if add is None:
            return torch.mm(a3, b3, out_dtype=torch.float32, out=out)
        return torch.addmm(add, a3, b3, out_dtype=torch.float32, out=out)
    return out.copy_(_mm32(a3, b3, add))


def _wgrad3(g_rows: torch.Tensor, x_rows: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out = g^T x to ~float32 accuracy from the row-stacked three-term pieces
    (g_rows [3K, M] in order "hhl", x_rows [3K, N] in order "lhh"; K = the
    batch's node / graph rows): split-K over the tripled contraction -- S
    float32 partial products in one batched bf16 GEMM, summed in order -- so
    the small [M, N] output still fills the chip (one plain GEMM of K = 18432
    ran at ~10 % of the bf16 peak)."""
    K3, M = g_rows.shape
    N = x_rows.shape[1]
    S = next((s for s in (12, 8, 6, 4, 3, 2) if K3 % s == 0 and K3 // s >= 512), 1)
    if S == 1 or not _MM32[0]:
        return _mm3(g_rows.t(), x_rows, out=out)
    part = torch.bmm(g_rows.view(S, K3 // S, M).transpose(1, 2), x_rows.view(S, K3 // S, N), out_dtype=torch.float32)
    return torch.sum(part, 0, out=out)


def _layer_args(l, norm, topo, a_all, off, stride, i, last):
    args = _lib.TrxGatLayerArgs()
    args.num_graphs, args.nodes_per_graph, args.heads, args.channels = topo.B, topo.n, l.heads, l.out_channels
    args.concat, args.max_graph_edges = int(l.concat), topo.max_graph_edges
    args.rowptr, args.col = topo.g.rowptr.data_ptr(), topo.g.col.data_ptr()
    args.a_edge, args.a_edge_stride, args.a_edge_offset = a_all.data_ptr(), stride, off
    args.negative_slope = float(l.negative_slope)
    args.ln_eps = float(norm.eps)
    args.activation = 1 if last else 0
    return args


def net_forward(net, node_x: torch.Tensor, edge_x: torch.Tensor, topo: Topology, save: bool,
                mask: Optional[torch.Tensor] = None, exact: bool = False):
    """Actor/Critic raw edge logits [B*e] (fp32) through the fused kernels, or
    with `mask` the Actor's masked softmax probabilities (sac.py:45-46).
    save=True also returns the NetCtx the backward needs.  exact=True: the
    float32 mode -- float32 GEMMs, activations and weights, no bf16 rounding
    (the reference's own precision)."""
    L = _lib.load()
    dev = node_x.device
    stream = _lib.stream_ptr(dev)
    enc = net.encoder
    layers = list(enc.layers)
    x0, ea, a_all = fused.prologue(net, node_x, edge_x, topo, keep_m=save, exact=exact)
    m_work = None
    if save:
        x0, ea, a_all, m_work = x0
    N = x0.shape[0]
    stride = a_all.shape[1]
    if exact:
        # float32 weights as they are; the lin / edge-head GEMM operands as
        # two-term bf16 splits (one launch for the four weight blocks)
        ip = enc.input_proj
        wts = [(layers[0].lin.weight.detach(), ip.weight.detach(), ip.bias.detach())] + \
              [l.lin.weight.detach() for l in layers[1:]]
        head_w = fused._head_weights_exact(net)
        wn_, wc_ = head_w[0], head_w[1].t()                    # [2H, d], [H, 2d] contiguous
        lin_w = [l.lin.weight for l in layers[1:]]
        ws = fused.split3([(w, "cols", "lhh") for w in lin_w] + [(w, "rows", "lhh") for w in lin_w] +
                          [(wn_, "cols", "lhh"), (wn_, "rows", "lhh"), (wc_, "cols", "lhh"), (wc_, "rows", "lhh")])
        nl = len(lin_w)
        w_cols, w_rows, (wn_c, wn_r, wc_c, wc_r) = ws[:nl], ws[nl:2 * nl], ws[2 * nl:]
    else:
        wts = fused._encoder_weights(enc, layers) if save else fused.prepared_encoder(enc, layers)
    # the linear-form layer 0 pays for its per-update weight preparation
    # (trx_gat_layer0_prepare, ~40 us on H + 1 workgroups) only at acting sizes
    lin0 = (not save and not exact and topo.B >= 1024 and fused.LAYER0_LINEAR and fused.layer0_supported(enc))
    mid = lin0 and fused.MID_REGEN and fused.mid_supported(enc)
    keep = []
    recs = []
    prev_f32 = prev_bf16 = None
    ctx = None
    off = 0
    for i, l in enumerate(layers):
        last = i == len(layers) - 1
        HC = l.heads * l.out_channels
        norm = enc.norms[i]
        args = _layer_args(l, norm, topo, a_all, off, stride, i, last)
        rec = {"off": off, "heads": l.heads, "channels": l.out_channels}
        args.exact = int(exact)
        if i == 0 and lin0:
            # no-grad passes: the linear-form layer 0 (csrc/gat_layer0.hip)
            out_bf16 = torch.empty(N, HC, device=dev, dtype=torch.bfloat16)
            out_f32 = torch.empty(N, HC, device=dev, dtype=torch.float32) if len(layers) > 2 and not mid else None
            desc = torch.empty(N, 4 * l.heads + 8, device=dev, dtype=torch.float32) if mid else None
            fused.layer0_infer(enc, x0, topo, a_all, off, out_f32, out_bf16, desc)
            recs.append(rec)
            prev_f32, prev_bf16 = out_f32, out_bf16
            off += l.heads
            continue
        if i == 1 and mid:   # layer 1 with the regenerated residual
            xh = F.linear(prev_bf16, wts[i])
            out_bf16 = torch.empty(N, HC, device=dev, dtype=torch.bfloat16)
            out_f32 = torch.empty(N, HC, device=dev, dtype=torch.float32) if i + 1 < len(layers) - 1 else None
            fused.mid_infer(enc, xh, desc, topo, a_all, off, out_f32, out_bf16)
            recs.append(rec)
            prev_f32, prev_bf16 = out_f32, out_bf16
            off += l.heads
            continue
        if i == 0:
            w0, wp, bp = wts[0]
            args.in_dim, args.x0, args.w0 = x0.shape[1], x0.data_ptr(), w0.data_ptr()
            args.residual, args.wp, args.bp = 2, wp.data_ptr(), bp.data_ptr()
            rec.update(w0=w0, wp=wp)
        else:
            if exact:
                x_c, x_r = fused.split3([(prev_f32, "cols", "hhl"), (prev_f32, "rows", "lhh")])
                xh = _mm3(x_c, w_cols[i - 1].t())                  # x_in @ W^T, ~float32
                rec.update(xh=xh, x_in=x_r, w=w_rows[i - 1])       # the backward's operands
            else:
                xh = F.linear(prev_bf16, wts[i])
                rec.update(xh=xh, x_in=prev_bf16, w=wts[i])
            args.in_dim, args.xh = 0, xh.data_ptr()
            if last:
                args.residual = 0
            else:
                args.residual, args.res = 1, prev_f32.data_ptr()
        att_s = l.att_src.detach().reshape(-1)
        att_d = l.att_dst.detach().reshape(-1)
        bias = l.bias.detach()
        lw, lb = norm.weight.detach(), norm.bias.detach()
        keep += [att_s, att_d, bias, lw, lb]
        args.att_src, args.att_dst, args.bias = att_s.data_ptr(), att_d.data_ptr(), bias.data_ptr()
        args.ln_weight, args.ln_bias = lw.data_ptr(), lb.data_ptr()
        out_bf16 = None if exact else torch.empty(N, HC, device=dev, dtype=torch.bfloat16)
        args.out_bf16 = 0 if exact else out_bf16.data_ptr()
        out_f32 = None
        if save or exact or (i + 1 < len(layers) - 1):
            out_f32 = torch.empty(N, HC, device=dev, dtype=torch.float32)
            args.out_f32 = out_f32.data_ptr()
        if last:
            ctx = torch.empty(topo.B, 2 * HC, device=dev, dtype=torch.float32)
            args.pool = ctx.data_ptr()
        if save:
            Et = topo.g.col.numel()
            rec.update(alpha=torch.empty(Et, l.heads, device=dev), asd=torch.empty(N, 2 * l.heads, device=dev),
                       v=torch.empty(N, HC, device=dev), stats=torch.empty(N, 2, device=dev), y=out_f32)
            args.save_alpha, args.save_asd = rec["alpha"].data_ptr(), rec["asd"].data_ptr()
            args.save_v, args.save_stats = rec["v"].data_ptr(), rec["stats"].data_ptr()
        _lib.check(L.trx_gat_layer_infer(args, stream), "trx_gat_layer_infer")
        recs.append(rec)
        prev_f32, prev_bf16 = out_f32, out_bf16
        off += l.heads
    b1 = net.edge_mlp[0].bias.detach()
    if exact:
        emb = prev_f32
        wn, wc, we, w2, b2 = head_w
        emb_c, emb_r, ctx_c, ctx_r = fused.split3([(emb, "cols", "hhl"), (emb, "rows", "lhh"),
                                                   (ctx, "cols", "hhl"), (ctx, "rows", "lhh")])
        p = _mm3(emb_c, wn_c.t())                               # ~float32 [N, 2H]
        c = _mm3(ctx_c, wc_c.t(), b1)
        head_w = (wn, wc, we, w2, b2, emb_r, ctx_r, wn_r, wc_r)
    else:
        emb = prev_bf16
        head_w = fused._head_weights(net) if save else fused.prepared_head(net)
        wn, wc, we, w2, b2 = head_w
        p = F.linear(emb, wn)                                   # bf16 [N, 2H] per-node projections
        c = _mm32(ctx.to(torch.bfloat16), wc, b1)               # bf16 operands, fp32 product + fp32 bias
    logits = torch.empty(topo.B * topo.e, device=dev, dtype=torch.float32)
    a = fused._edge_args(p, c, ea, we, w2, b2, topo.src32, topo.dst32, topo.B, topo.n, topo.e)
    a.exact = int(exact)
    a.out = logits.data_ptr()
    if mask is not None:
        m = mask.float().contiguous()
        a.mask, a.softmax = m.data_ptr(), 1
        keep.append(m)
    _lib.check(L.trx_edge_head_infer(a, stream), "trx_edge_head_infer")
    del keep
    if not save:
        return logits, None
    return logits, NetCtx(x0, ea, a_all, m_work, node_x, edge_x, recs, emb, ctx, p, c, head_w)


# grouped launches in the update: 0 = six branches, one network each (the default: the
# fastest replay, 2.01 ms per update); 1 = the five bf16 passes in one group beside the
# float32 actor (two branches, 2.21 ms); 2 = the critics' training passes and the three
# next-state passes as two groups (three branches, 2.13 ms).  Bit-identical results
# (tests/test_fused_update.py test_grouped_update_bit_identical); DESIGN §5
MULTI = int(os.environ.get("TRX_UPD_MULTI", "0"))


def _stack_weights(nets):
    """Every network's weight blocks for the bf16 (non-exact) passes, stacked
    network-major: layer 0's w0 / wp / bp bf16-rounded float32 [k, ...], the
    lin weights of layers >= 1 as bf16 [k, out, in], the edge MLP's node and
    context blocks as bf16 WN [k, 2H, d] / WC [k, H, 2d], its link-feature
    block, output weight and bias float32 (models/fused.py _encoder_weights
    and _head_weights, for k networks in trx_bf16_round launches of 48)."""
    k, dev = len(nets), nets[0].edge_mlp[0].weight.device
    enc0, head0 = nets[0].encoder, nets[0]
    l0 = list(enc0.layers)
    W1 = head0.edge_mlp[0].weight
    d, K, hid = head0.embed, head0.edge_in, W1.shape[0]
    bf = torch.bfloat16
    w0 = torch.empty((k,) + tuple(l0[0].lin.weight.shape), device=dev)
    wp = torch.empty((k,) + tuple(enc0.input_proj.weight.shape), device=dev)
    bp = torch.empty((k,) + tuple(enc0.input_proj.bias.shape), device=dev)
    W = [torch.empty((k,) + tuple(l.lin.weight.shape), device=dev, dtype=bf) for l in l0[1:]]
    WN = torch.empty(k, 2 * hid, d, device=dev, dtype=bf)
    WC = torch.empty(k, hid, W1.shape[1] - 2 * d - K, device=dev, dtype=bf)
    WE = torch.empty(k, hid, K, device=dev)
    W2 = torch.empty(k, hid, device=dev)
    B2 = torch.empty(k, 1, device=dev)
    pairs = []
    for j, net in enumerate(nets):
        enc = net.encoder
        ls = list(enc.layers)
        pairs += [(ls[0].lin.weight, w0[j]), (enc.input_proj.weight, wp[j]), (enc.input_proj.bias, bp[j])]
        pairs += [(l.lin.weight, Wl[j]) for l, Wl in zip(ls[1:], W)]
        W1 = net.edge_mlp[0].weight
        pairs += [(W1[:, :d], WN[j, :hid]), (W1[:, d:2 * d], WN[j, hid:]), (W1[:, 2 * d + K:], WC[j]),
                  (W1[:, 2 * d:2 * d + K], WE[j], True), (net.edge_mlp[2].weight.reshape(-1), W2[j], True),
                  (net.edge_mlp[2].bias.reshape(-1), B2[j], True)]
    fused._round_into(pairs)
    return w0, wp, bp, W, WN, WC, WE, W2, B2


def multi_supported(nets) -> bool:
    """Networks whose passes can share launches: identical layer / head shapes."""
    def sig(net):
        return ([(l.heads, l.out_channels, l.concat, tuple(l.lin.weight.shape)) for l in net.encoder.layers],
                tuple(net.edge_mlp[0].weight.shape), net.embed, net.edge_in)
    return len(nets) <= _lib.MAX_NETS and all(sig(n) == sig(nets[0]) for n in nets)


def net_forward_multi(specs, topo: Topology):
    """net_forward (bf16 mode) for several networks of the same shapes in
    shared launches: specs = [(net, node_x, edge_x, save, mask)], each with its
    own inputs, weights and outputs.  One trx_*_multi launch per kernel (the
    network index in blockIdx.y), the lin / edge-head GEMMs per network as
    net_forward issues them, the edge scorer once per softmax kind.  Same kernels,
    arithmetic and rounding points per network as net_forward; returns
    [(logits, NetCtx | None)] in spec order (the contexts share one NetGroup)."""
    L = _lib.load()
    k = len(specs)
    nets = [sp[0] for sp in specs]
    dev = specs[0][1].device
    stream = _lib.stream_ptr(dev)
    layers = list(nets[0].encoder.layers)
    B, n, e = topo.B, topo.n, topo.e
    N = B * n
    pro = [fused.prologue_args(net, nx, ex, topo) for net, nx, ex, _, _ in specs]
    _lib.check(L.trx_gat_prologue_infer_multi(_lib.multi(_lib.TrxGatPrologueArgs, [p[0] for p in pro]), k, stream),
               "trx_gat_prologue_infer_multi")
    keep = [p[2] for p in pro]
    x0s, eas, a_alls, m_works = zip(*[p[1] for p in pro])
    stride = a_alls[0].shape[1]
    w0, wp, bp, W, WN, WC, WE, W2, B2 = _stack_weights(nets)
    recs = [[] for _ in range(k)]
    prev_f32 = [None] * k
    prev_b = None
    x_in = []
    ctx = None
    off = 0
    for i, l in enumerate(layers):
        last = i == len(layers) - 1
        HC = l.heads * l.out_channels
        xh = None
        if i > 0:
            # per network, the single pass's GEMM (a batched bf16 GEMM over the networks faulted
            # in hipBLASLt on this image at [5, 6144, 1024] x [5, 1024, 1024]^T)
            xh = [F.linear(prev_b[j], W[i - 1][j]) for j in range(k)]   # [N, HC] bf16 each
            x_in.append(prev_b)
        out_b = torch.empty(k, N, HC, device=dev, dtype=torch.bfloat16)
        if last:
            ctx = torch.empty(k, B, 2 * HC, device=dev)
        arglist = []
        for j, (net, _, _, save, _) in enumerate(specs):
            enc = net.encoder
            lj, norm = enc.layers[i], enc.norms[i]
            args = _layer_args(lj, norm, topo, a_alls[j], off, stride, i, last)
            args.exact = 0
            rec = {"off": off, "heads": lj.heads, "channels": lj.out_channels}
            if i == 0:
                args.in_dim, args.x0, args.w0 = x0s[j].shape[1], x0s[j].data_ptr(), w0[j].data_ptr()
                args.residual, args.wp, args.bp = 2, wp[j].data_ptr(), bp[j].data_ptr()
                rec.update(w0=w0[j], wp=wp[j])
            else:
                args.in_dim, args.xh = 0, xh[j].data_ptr()
                rec.update(xh=xh[j], x_in=prev_b[j], w=W[i - 1][j])
                if last:
                    args.residual = 0
                else:
                    args.residual, args.res = 1, prev_f32[j].data_ptr()
            att_s, att_d = lj.att_src.detach().reshape(-1), lj.att_dst.detach().reshape(-1)
            args.att_src, args.att_dst, args.bias = att_s.data_ptr(), att_d.data_ptr(), lj.bias.detach().data_ptr()
            args.ln_weight, args.ln_bias = norm.weight.detach().data_ptr(), norm.bias.detach().data_ptr()
            args.out_bf16 = out_b[j].data_ptr()
            out_f32 = None
            if save or (i + 1 < len(layers) - 1):
                out_f32 = torch.empty(N, HC, device=dev)
                args.out_f32 = out_f32.data_ptr()
            if last:
                args.pool = ctx[j].data_ptr()
            if save:
                Et = topo.g.col.numel()
                rec.update(alpha=torch.empty(Et, lj.heads, device=dev), asd=torch.empty(N, 2 * lj.heads, device=dev),
                           v=torch.empty(N, HC, device=dev), stats=torch.empty(N, 2, device=dev), y=out_f32)
                args.save_alpha, args.save_asd = rec["alpha"].data_ptr(), rec["asd"].data_ptr()
                args.save_v, args.save_stats = rec["v"].data_ptr(), rec["stats"].data_ptr()
            arglist.append(args)
            recs[j].append(rec)
            prev_f32[j] = out_f32
        _lib.check(L.trx_gat_layer_infer_multi(_lib.multi(_lib.TrxGatLayerArgs, arglist), k, stream),
                   "trx_gat_layer_infer_multi")
        prev_b = out_b
        off += l.heads
    emb = prev_b                                                        # [k, N, d] bf16
    p = [F.linear(emb[j], WN[j]) for j in range(k)]                     # bf16 [N, 2H] per-node projections
    ctx_b = ctx.to(torch.bfloat16)
    c = [_mm32(ctx_b[j], WC[j].t(), net.edge_mlp[0].bias.detach())      # bf16 operands, fp32 product + bias
         for j, net in enumerate(nets)]
    grp = NetGroup(x_in, W, emb, ctx, WN, WC)
    logits = [torch.empty(B * e, device=dev) for _ in range(k)]
    heads = {0: [], 1: []}
    for j, (net, _, _, _, mask) in enumerate(specs):
        a = fused._edge_args(p[j], c[j], eas[j], WE[j], W2[j], B2[j], topo.src32, topo.dst32, B, n, e)
        a.exact = 0
        a.out = logits[j].data_ptr()
        if mask is not None:
            m = mask.float().contiguous()
            keep.append(m)
            a.mask, a.softmax = m.data_ptr(), 1
        heads[a.softmax].append(a)
    for grp_args in heads.values():
        if grp_args:
            _lib.check(L.trx_edge_head_infer_multi(_lib.multi(_lib.TrxEdgeHeadArgs, grp_args), len(grp_args), stream),
                       "trx_edge_head_infer_multi")
    del keep
    out = []
    for j, (net, nx, ex, save, _) in enumerate(specs):
        if not save:
            out.append((logits[j], None))
            continue
        head_w = (WN[j], WC[j].t(), WE[j], W2[j], B2[j])
        out.append((logits[j], NetCtx(x0s[j], eas[j], a_alls[j], m_works[j], nx, ex, recs[j], emb[j], ctx[j], p[j],
                                      c[j], head_w, grp, j)))
    return out


def net_backward_multi(nets, cxs: List[NetCtx], g_logits: List[torch.Tensor], topo: Topology,
                       sinks: List["GradFlat"], sums: "PartialSums"):
    """net_backward (bf16 mode) for networks of one net_forward_multi group in
    shared launches: the edge-scorer, layer and prologue backward kernels once
    per kind (trx_*_backward_multi), the weight-gradient and input-gradient
    GEMMs per network as net_backward issues them.  Each network's gradients go into its own
    sink in net_backward's order; the column sums are left to `sums`."""
    L = _lib.load()
    k = len(nets)
    grp = cxs[0].grp
    assert grp is not None and all(cx.grp is grp for cx in cxs) and [cx.j for cx in cxs] == list(range(k))
    dev = g_logits[0].device
    stream = _lib.stream_ptr(dev)
    layers = list(nets[0].encoder.layers)
    B, n, e = topo.B, topo.n, topo.e
    N = B * n
    WN, WC = grp.WN[:k], grp.WC[:k]   # the group's first k networks (the trained ones)
    Hd = WN.shape[1] // 2
    K = cxs[0].head_w[2].shape[1]
    # ---- edge scorer
    g_p = torch.empty(k, N, 2 * Hd, device=dev, dtype=torch.bfloat16)
    g_c = torch.empty(k, B, Hd, device=dev)
    gw2p = torch.empty(k, B, Hd, device=dev)
    gwep = torch.empty(k, B, Hd * K, device=dev)
    g_ea_head = torch.empty(k, B * e, K, device=dev)
    gl = [g.contiguous() for g in g_logits]
    args, ios = [], []
    for j, cx in enumerate(cxs):
        wn, wc, we, w2, b2 = cx.head_w[:5]
        a = fused._edge_args(cx.p, cx.c, cx.ea, we, w2, b2, topo.src32, topo.dst32, B, n, e)
        a.exact = 0
        args.append(a)
        ios.append(_lib.TrxEdgeHeadBwdIO(gl[j].data_ptr(), g_p[j].data_ptr(), g_c[j].data_ptr(), None,
                                         gw2p[j].data_ptr(), gwep[j].data_ptr(), g_ea_head[j].data_ptr()))
    _lib.check(L.trx_edge_head_backward_multi(_lib.multi(_lib.TrxEdgeHeadArgs, args),
                                              _lib.multi(_lib.TrxEdgeHeadBwdIO, ios), k, stream),
               "trx_edge_head_backward_multi")
    g_we = torch.empty(k, Hd, K, device=dev)
    for j in range(k):
        sums.add(gwep[j], Hd * K, Hd * K, g_we[j])
    # the GEMMs per network, as net_backward issues them
    g_wn = [_splitk_wgrad(g_p[j], grp.emb[j]) for j in range(k)]              # [2H, embed] fp32
    g_emb = [_mm32(g_p[j], WN[j]) for j in range(k)]                           # [N, embed] fp32
    g_cb = g_c.to(torch.bfloat16)
    ctx_b = grp.ctx[:k].to(torch.bfloat16)
    g_wc = [_mm32(g_cb[j].t(), ctx_b[j]) for j in range(k)]                    # [H, 2 embed]
    g_ctx = [_mm32(g_cb[j], WC[j]) for j in range(k)]                          # [B, 2 embed]
    for j, net in enumerate(nets):
        W1 = net.edge_mlp[0].weight
        gW1 = sinks[j].take(W1.numel()).view_as(W1)
        sums.after.append(lambda j=j, gW1=gW1: torch.cat([g_wn[j][:Hd], g_wn[j][Hd:], g_we[j], g_wc[j]], 1, out=gW1))
        sums.used += [gW1]
        _grad(W1, gW1)
        for prm, src in ((net.edge_mlp[0].bias, g_c[j]), (net.edge_mlp[2].weight, gw2p[j])):
            dst = sinks[j].take(prm.numel())
            sums.add(src, Hd, Hd, dst)
            _grad(prm, dst)
        gb2 = sinks[j].take(1)
        torch.sum(gl[j], 0, keepdim=True, out=gb2)
        _grad(net.edge_mlp[2].bias, gb2)
    sums.used += g_wn + g_wc + [g_we]
    # ---- GAT layers, last to first
    g_a_all = [torch.empty_like(cx.a_all) for cx in cxs]
    g_x0 = [torch.empty_like(cx.x0) for cx in cxs]
    gy, g_pool = g_emb, g_ctx
    for i in range(len(layers) - 1, -1, -1):
        l = layers[i]
        last = i == len(layers) - 1
        HC = l.heads * l.out_channels
        g_xh = torch.empty(k, N, HC, device=dev, dtype=torch.bfloat16)
        g_res = torch.empty(k, N, HC, device=dev)
        PW = int(L.trx_gat_layer_backward_part_floats(l.heads, l.out_channels, 4 if i == 0 else 0))
        part = torch.empty(k, B, PW, device=dev)
        bargs = []
        for j, (net, cx) in enumerate(zip(nets, cxs)):
            lj, norm, rec = net.encoder.layers[i], net.encoder.norms[i], cx.layers[i]
            ba = _lib.TrxGatLayerBwdArgs()
            ba.num_graphs, ba.nodes_per_graph, ba.heads, ba.channels = B, n, lj.heads, lj.out_channels
            ba.max_graph_edges, ba.in_dim = topo.max_graph_edges, 4 if i == 0 else 0
            g = topo.g
            ba.rowptr, ba.col, ba.sptr, ba.spos = g.rowptr.data_ptr(), g.col.data_ptr(), g.sptr.data_ptr(), g.spos.data_ptr()
            ba.att_src = lj.att_src.detach().reshape(-1).data_ptr()
            ba.att_dst = lj.att_dst.detach().reshape(-1).data_ptr()
            ba.ln_weight = norm.weight.detach().data_ptr()
            ba.a_edge, ba.a_edge_stride, ba.a_edge_offset = cx.a_all.data_ptr(), cx.a_all.shape[1], rec["off"]
            ba.negative_slope = float(lj.negative_slope)
            ba.exact = 0
            ba.activation = 1 if last else 0
            ba.residual = 0 if last else (2 if i == 0 else 1)
            if i == 0:
                ba.x0, ba.w0, ba.wp, ba.g_x0 = (cx.x0.data_ptr(), rec["w0"].data_ptr(), rec["wp"].data_ptr(),
                                                g_x0[j].data_ptr())
            else:
                ba.xh = rec["xh"].data_ptr()
            ba.alpha, ba.asd, ba.v, ba.stats, ba.y = (rec["alpha"].data_ptr(), rec["asd"].data_ptr(),
                                                       rec["v"].data_ptr(), rec["stats"].data_ptr(), rec["y"].data_ptr())
            ba.gy = gy[j].data_ptr()
            ba.g_pool = 0 if g_pool is None else g_pool[j].data_ptr()
            ba.g_xh, ba.g_res, ba.g_a_edge, ba.part = (g_xh[j].data_ptr(), g_res[j].data_ptr(), g_a_all[j].data_ptr(),
                                                       part[j].data_ptr())
            bargs.append(ba)
        _lib.check(L.trx_gat_layer_backward_multi(_lib.multi(_lib.TrxGatLayerBwdArgs, bargs), k, stream),
                   "trx_gat_layer_backward_multi")
        for j, net in enumerate(nets):
            lj, norm = net.encoder.layers[i], net.encoder.norms[i]
            pg = sinks[j].take(PW)
            sums.add(part[j], PW, PW, pg)
            _grad(lj.bias, pg[:HC])
            _grad(norm.weight, pg[HC:2 * HC])
            _grad(norm.bias, pg[2 * HC:3 * HC])
            _grad(lj.att_src, pg[3 * HC:4 * HC])
            _grad(lj.att_dst, pg[4 * HC:5 * HC])
            if i == 0:
                _grad(lj.lin.weight, pg[5 * HC:9 * HC])
                _grad(net.encoder.input_proj.weight, pg[9 * HC:13 * HC])
                _grad(net.encoder.input_proj.bias, pg[13 * HC:14 * HC])
        sums.used += [part]
        if i > 0:
            # lin: xh = x_in @ w^T (bf16): split-K fp32 weight gradients, then the previous layer's output gradient (bf16 through lin + fp32 residual)
            x_in = grp.x_in[i - 1]
            S = 4 if N % 4 == 0 else 1
            gy = []
            for j, net in enumerate(nets):
                lw = net.encoder.layers[i].lin.weight
                gw = sinks[j].take(lw.numel()).view_as(lw)
                part_w = torch.bmm(g_xh[j].view(S, N // S, -1).transpose(1, 2), x_in[j].view(S, N // S, -1))
                torch.sum(part_w, 0, dtype=torch.float32, out=gw)
                _grad(lw, gw)
                # a middle layer's input also reaches it as the float32 residual
                gy.append(_mm32(g_xh[j], grp.W[i - 1][j]) if last else
                          _mm3(g_xh[j], grp.W[i - 1][j], g_res[j], out=g_res[j]))   # in place: no addend copy
            g_pool = None
    # ---- prologue (input LayerNorms, loop attrs, edge-logit projections)
    A = cxs[0].a_all.shape[1]
    PP = 8 * A + 32
    ppart = torch.empty(k, B, PP, device=dev)
    pargs = []
    for j, (net, cx) in enumerate(zip(nets, cxs)):
        pa = _lib.TrxGatPrologueBwdArgs()
        pa.num_graphs, pa.nodes_per_graph, pa.edges_per_graph = B, n, e
        pa.node_dim, pa.edge_dim, pa.A = cx.node_x.shape[1], cx.edge_x.shape[1], A
        pa.node_x, pa.edge_x = cx.node_x.data_ptr(), cx.edge_x.data_ptr()
        nw, nb = net.node_norm.weight.detach(), net.node_norm.bias.detach()
        ew, eb = net.edge_norm.weight.detach(), net.edge_norm.bias.detach()
        pa.node_ln_w, pa.node_ln_b, pa.node_ln_eps = nw.data_ptr(), nb.data_ptr(), float(net.node_norm.eps)
        pa.edge_ln_w, pa.edge_ln_b, pa.edge_ln_eps = ew.data_ptr(), eb.data_ptr(), float(net.edge_norm.eps)
        pa.src, pa.dst, pa.rowptr, pa.pos_src = (topo.src32.data_ptr(), topo.dst32.data_ptr(),
                                                 topo.g.rowptr.data_ptr(), topo.pos_src.data_ptr())
        pa.m_work, pa.g_a_edge, pa.g_x0, pa.g_ea_head = (cx.m_work.data_ptr(), g_a_all[j].data_ptr(),
                                                         g_x0[j].data_ptr(), g_ea_head[j].data_ptr())
        pa.part = ppart[j].data_ptr()
        pa.exact = 0
        pargs.append(pa)
    _lib.check(L.trx_gat_prologue_backward_multi(_lib.multi(_lib.TrxGatPrologueBwdArgs, pargs), k, stream),
               "trx_gat_prologue_backward_multi")
    sums.used += [ppart] + g_a_all + g_x0 + [g_ea_head]
    for j, (net, cx) in enumerate(zip(nets, cxs)):
        _prologue_grads(net, cx, ppart[j], sinks[j], sums, PP, A, dev)


def _prologue_grads(net, cx: NetCtx, ppart: torch.Tensor, sink: "GradFlat", sums: "PartialSums", PP: int, A: int,
                    dev):
    """The prologue's parameter gradients from its per-graph partials: the
    input LayerNorms (column sums) and every layer's lin_edge / att_edge
    (trx_edge_att_weights_backward after the sums), into `sink`."""
    L = _lib.load()
    layers = list(net.encoder.layers)
    pp = sink.take(PP)
    sums.add(ppart, PP, PP, pp)
    ed, nd = cx.edge_x.shape[1], cx.node_x.shape[1]
    _grad(net.edge_norm.weight, pp[8 * A:8 * A + ed])
    _grad(net.edge_norm.bias, pp[8 * A + 8:8 * A + 8 + ed])
    _grad(net.node_norm.weight, pp[8 * A + 16:8 * A + 16 + nd])
    _grad(net.node_norm.bias, pp[8 * A + 24:8 * A + 24 + nd])
    # M[h, j] = sum_c W[h*C + c, j] * att[h, c] (fp32, then bf16-rounded in the forward):
    # every layer's lin_edge / att_edge gradient from the summed M-row gradients, one launch
    ea_args = _lib.TrxGatPrologueArgs()
    ea_args.num_layers, ea_args.edge_dim = len(layers), ed
    keep = []
    for i, l in enumerate(layers):
        w, at = l.lin_edge.weight.detach().contiguous(), l.att_edge.detach().contiguous()
        keep += [w, at]
        ea_args.heads[i], ea_args.channels[i] = l.heads, l.out_channels
        ea_args.lin_edge_w[i], ea_args.att_edge[i] = w.data_ptr(), at.data_ptr()
    tot = sum(l.heads * l.out_channels * (ed + 1) for l in layers)
    gout = sink.take(tot)

    def att_weights():   # needs the summed prologue partials (pp)
        _lib.check(L.trx_edge_att_weights_backward(ea_args, _lib.ptr(pp), 8, _lib.ptr(gout),
                                                   _lib.stream_ptr(dev)), "trx_edge_att_weights_backward")
    sums.after.append(att_weights)
    sums.used += [gout] + keep
    off = 0
    for l in layers:
        HC = l.heads * l.out_channels
        _grad(l.lin_edge.weight, gout[off:off + HC * ed].view(HC, ed))
        _grad(l.att_edge, gout[off + HC * ed:off + HC * (ed + 1)])
        off += HC * (ed + 1)


class GradFlat:
    """Every gradient of one fused update as a view into ONE float32 buffer,
    carved in the order the backward produces them, so each producer (GEMM,
    partial-sum kernel, loss kernel) writes its parameters' gradients in place:
    the data-parallel all-reduce (train.GradAllReduce) then reduces this
    buffer directly -- no concatenation and no copy back."""

    def __init__(self, total: int, device):
        self.buf = torch.empty(total, device=device, dtype=torch.float32)
        self.off = 0

    def take(self, n: int) -> torch.Tensor:
        t = self.buf[self.off:self.off + n]
        self.off += n
        assert self.off <= self.buf.numel(), "GradFlat layout overflow"
        return t


def flat_size(net) -> int:
    """GradFlat floats one network's backward takes: its parameters plus the
    prologue partial sums' padding (M-row gradients, 8-wide LayerNorm rows)."""
    A = sum(l.heads for l in net.encoder.layers)
    ed, nd = net.edge_norm.weight.numel(), net.node_norm.weight.numel()
    return sum(p.numel() for p in net.parameters()) + 8 * A + 32 - 2 * ed - 2 * nd


def _grad(param, g):
    """param.grad = g (set_to_none semantics of the reference's zero_grad():
    the gradient tensor is handed over, not accumulated)."""
    param.grad = g.view_as(param) if g.shape != param.shape else g


class PartialSums:
    """The per-graph parameter partials of one update's backwards, column-summed
    by ONE trx_partial_sum_multi launch at the end (each sum in the fixed order of
    trx_partial_sum; 21 launches -> 1), and the work that needs the sums."""

    def __init__(self, rows: int):
        self.rows, self.entries, self.after, self.used = rows, [], [], []

    def add(self, part: torch.Tensor, width: int, stride: int, out: torch.Tensor, out_cols: int = 0,
            out_ld: int = 0):
        self.entries.append((part, width, stride, out, out_cols, out_ld))

    def flush(self, stream):
        """Run on the stream that joined the backwards: every buffer a side stream
        allocated is recorded as used here before its last reference drops."""
        L = _lib.load()
        cur = torch.cuda.current_stream()
        for t in [x for e in self.entries for x in (e[0], e[3])] + self.used:
            t.record_stream(cur)
        for b0 in range(0, len(self.entries), _lib.MAX_PSUM):
            lst = _lib.TrxPsumList()
            chunk = self.entries[b0:b0 + _lib.MAX_PSUM]
            lst.count, lst.rows = len(chunk), self.rows
            for e, (part, width, stride, out, oc, ld) in enumerate(chunk):
                lst.part[e], lst.width[e], lst.stride[e] = part.data_ptr(), width, stride
                lst.out[e], lst.out_cols[e], lst.out_ld[e] = out.data_ptr(), oc, ld
            _lib.check(L.trx_partial_sum_multi(ctypes.byref(lst), stream), "trx_partial_sum_multi")
        for fn in self.after:
            fn()
        self.entries, self.after, self.used = [], [], []


def net_backward(net, cx: NetCtx, g_logits: torch.Tensor, topo: Topology, sink: GradFlat, exact: bool = False,
                 sums: Optional[PartialSums] = None):
    """Gradients of every parameter of `net` from dL/dlogits [B*e] fp32,
    written into `sink` and handed to the parameters as views (exact: the
    backward of net_forward(..., exact=True), float32 throughout).  With
    `sums` the column sums of the per-graph partials are left to sums.flush()
    (after every network's backward); without, they run here."""
    own = sums is None
    if own:
        sums = PartialSums(topo.B)
    L = _lib.load()
    dev = g_logits.device
    stream = _lib.stream_ptr(dev)
    enc = net.encoder
    layers = list(enc.layers)
    B, n, e = topo.B, topo.n, topo.e
    N = B * n
    wn, wc, we, w2, b2 = cx.head_w[:5]
    Hd = wn.shape[0] // 2
    # ---- edge scorer (sac.py:42-44 factored): kernel + link-feature / weight products
    a = fused._edge_args(cx.p, cx.c, cx.ea, we, w2, b2, topo.src32, topo.dst32, B, n, e)
    a.exact = int(exact)
    k = we.shape[1]
    g_p = torch.empty_like(cx.p)
    g_c = torch.empty(B, Hd, device=dev, dtype=torch.float32)
    gw2p = torch.empty(B, Hd, device=dev, dtype=torch.float32)
    gwep = torch.empty(B, Hd * k, device=dev, dtype=torch.float32)      # per-graph link-feature weight partials
    g_ea_head = torch.empty(B * e, k, device=dev, dtype=torch.float32)   # link features' gradient (fp32)
    gl = g_logits.contiguous()
    _lib.check(L.trx_edge_head_backward(a, _lib.ptr(gl), _lib.ptr(g_p), _lib.ptr(g_c), None, _lib.ptr(gw2p),
                                        _lib.ptr(gwep), _lib.ptr(g_ea_head), stream), "trx_edge_head_backward")
    g_we = torch.empty(Hd, k, device=dev, dtype=torch.float32)
    sums.add(gwep, Hd * k, Hd * k, g_we)
    if exact:
        emb_r, ctx_r, wn_r, wc_r = cx.head_w[5:]
        gp_c, gp_r, gc_c, gc_r = fused.split3([(g_p, "cols", "hhl"), (g_p, "rows", "hhl"),
                                               (g_c, "cols", "hhl"), (g_c, "rows", "hhl")])
        g_wn = _wgrad3(gp_r, emb_r, torch.empty(gp_r.shape[1], emb_r.shape[1], device=dev))   # [2H, embed]
        g_emb = _mm3(gp_c, wn_r)                                        # [N, embed]
        g_wc = _mm3(gc_r.t(), ctx_r)                                    # [H, 2*embed]
        g_ctx = _mm3(gc_c, wc_r)                                        # [B, 2*embed]
    else:
        g_wn = _splitk_wgrad(g_p, cx.emb)                               # [2H, embed] fp32
        g_emb = _mm32(g_p, wn)                                          # fp32 [N, embed]
        g_cb = g_c.to(torch.bfloat16)
        ctx_b = cx.ctx.to(torch.bfloat16)
        g_wc = _mm32(g_cb.t(), ctx_b)                                   # [H, 2*embed]
        g_ctx = _mm32(g_cb, wc.t())                                     # [B, 2*embed]
    W1 = net.edge_mlp[0].weight
    gW1 = sink.take(W1.numel()).view_as(W1)
    sums.after.append(lambda: torch.cat([g_wn[:Hd], g_wn[Hd:], g_we, g_wc], 1, out=gW1))
    sums.used += [g_wn, g_wc, gW1]
    _grad(W1, gW1)
    for prm, src in ((net.edge_mlp[0].bias, g_c), (net.edge_mlp[2].weight, gw2p)):
        dst = sink.take(prm.numel())      # column sums over the graphs, fixed order
        sums.add(src, Hd, Hd, dst)
        _grad(prm, dst)
    gb2 = sink.take(1)
    torch.sum(gl, 0, keepdim=True, out=gb2)
    _grad(net.edge_mlp[2].bias, gb2)
    # ---- GAT layers, last to first
    a_all = cx.a_all
    g_a_all = torch.empty_like(a_all)
    g_x0 = torch.empty_like(cx.x0)
    gy_f32, gy_b16, g_pool = g_emb, None, g_ctx
    for i in range(len(layers) - 1, -1, -1):
        l, rec = layers[i], cx.layers[i]
        last = i == len(layers) - 1
        norm = enc.norms[i]
        HC = l.heads * l.out_channels
        ba = _lib.TrxGatLayerBwdArgs()
        ba.num_graphs, ba.nodes_per_graph, ba.heads, ba.channels = B, n, l.heads, l.out_channels
        ba.max_graph_edges, ba.in_dim = topo.max_graph_edges, 4 if i == 0 else 0
        g = topo.g
        ba.rowptr, ba.col, ba.sptr, ba.spos = g.rowptr.data_ptr(), g.col.data_ptr(), g.sptr.data_ptr(), g.spos.data_ptr()
        att_s, att_d = l.att_src.detach().reshape(-1), l.att_dst.detach().reshape(-1)
        lw = norm.weight.detach()
        ba.att_src, ba.att_dst, ba.ln_weight = att_s.data_ptr(), att_d.data_ptr(), lw.data_ptr()
        ba.a_edge, ba.a_edge_stride, ba.a_edge_offset = a_all.data_ptr(), a_all.shape[1], rec["off"]
        ba.negative_slope = float(l.negative_slope)
        ba.exact = int(exact)
        ba.activation = 1 if last else 0
        ba.residual = 0 if last else (2 if i == 0 else 1)
        if i == 0:
            ba.x0, ba.w0, ba.wp, ba.g_x0 = cx.x0.data_ptr(), rec["w0"].data_ptr(), rec["wp"].data_ptr(), g_x0.data_ptr()
        else:
            ba.xh = rec["xh"].data_ptr()
        ba.alpha, ba.asd, ba.v, ba.stats, ba.y = (rec["alpha"].data_ptr(), rec["asd"].data_ptr(), rec["v"].data_ptr(),
                                                   rec["stats"].data_ptr(), rec["y"].data_ptr())
        ba.gy = 0 if gy_f32 is None else gy_f32.data_ptr()
        ba.gy_bf16 = 0 if gy_b16 is None else gy_b16.data_ptr()
        ba.g_pool = 0 if g_pool is None else g_pool.data_ptr()
        g_xh = torch.empty(N, HC, device=dev, dtype=torch.float32 if exact else torch.bfloat16)
        g_res = torch.empty(N, HC, device=dev, dtype=torch.float32)
        PW = int(L.trx_gat_layer_backward_part_floats(l.heads, l.out_channels, ba.in_dim))
        part = torch.empty(B, PW, device=dev, dtype=torch.float32)
        ba.g_xh, ba.g_res, ba.g_a_edge, ba.part = g_xh.data_ptr(), g_res.data_ptr(), g_a_all.data_ptr(), part.data_ptr()
        _lib.check(L.trx_gat_layer_backward(ba, stream), "trx_gat_layer_backward")
        pg = sink.take(PW)
        sums.add(part, PW, PW, pg)
        _grad(l.bias, pg[:HC])
        _grad(norm.weight, pg[HC:2 * HC])
        _grad(norm.bias, pg[2 * HC:3 * HC])
        _grad(l.att_src, pg[3 * HC:4 * HC])
        _grad(l.att_dst, pg[4 * HC:5 * HC])
        if i == 0:
            _grad(l.lin.weight, pg[5 * HC:9 * HC])
            _grad(enc.input_proj.weight, pg[9 * HC:13 * HC])
            _grad(enc.input_proj.bias, pg[13 * HC:14 * HC])
        else:
            # lin: xh = x_in @ w^T (bf16): split-K fp32 weight gradient, bf16 input gradient
            x_in = rec["x_in"]
            S = 4 if N % 4 == 0 else 1
            gw = sink.take(l.lin.weight.numel()).view_as(l.lin.weight)
            if exact:
                gx_c, gx_r = fused.split3([(g_xh, "cols", "hhl"), (g_xh, "rows", "hhl")])
                _wgrad3(gx_r, x_in, gw)                                 # g_xh^T x_in
            else:
                part_w = torch.bmm(g_xh.view(S, N // S, -1).transpose(1, 2), x_in.view(S, N // S, -1))
                torch.sum(part_w, 0, dtype=torch.float32, out=gw)
            _grad(l.lin.weight, gw)
            # the previous layer's output reaches this layer twice: bf16 through lin,
            # fp32 as the residual of a middle layer (gat_encoder.py:44-46)
            # (+ residual): accumulated in place into g_res -- addmm into a fresh
            # output first copies the [N, HC] float32 addend (a 25 MB device copy)
            a3 = gx_c if exact else g_xh
            gy_f32 = _mm3(a3, rec["w"], g_res, out=g_res) if ba.residual == 1 else _mm3(a3, rec["w"])   # g_xh W
            gy_b16 = None
            g_pool = None
    # ---- prologue: input LayerNorms, loop attrs, edge-logit projections
    A = a_all.shape[1]
    pa = _lib.TrxGatPrologueBwdArgs()
    pa.num_graphs, pa.nodes_per_graph, pa.edges_per_graph = B, n, e
    pa.node_dim, pa.edge_dim, pa.A = cx.node_x.shape[1], cx.edge_x.shape[1], A
    nx, ex = cx.node_x, cx.edge_x
    pa.node_x, pa.edge_x = nx.data_ptr(), ex.data_ptr()
    nw, nb = net.node_norm.weight.detach(), net.node_norm.bias.detach()
    ew, eb = net.edge_norm.weight.detach(), net.edge_norm.bias.detach()
    pa.node_ln_w, pa.node_ln_b, pa.node_ln_eps = nw.data_ptr(), nb.data_ptr(), float(net.node_norm.eps)
    pa.edge_ln_w, pa.edge_ln_b, pa.edge_ln_eps = ew.data_ptr(), eb.data_ptr(), float(net.edge_norm.eps)
    pa.src, pa.dst, pa.rowptr, pa.pos_src = (topo.src32.data_ptr(), topo.dst32.data_ptr(), topo.g.rowptr.data_ptr(),
                                             topo.pos_src.data_ptr())
    pa.m_work, pa.g_a_edge, pa.g_x0, pa.g_ea_head = (cx.m_work.data_ptr(), g_a_all.data_ptr(), g_x0.data_ptr(),
                                                     g_ea_head.data_ptr())
    PP = 8 * A + 32
    ppart = torch.empty(B, PP, device=dev, dtype=torch.float32)
    pa.part = ppart.data_ptr()
    pa.exact = int(exact)
    _lib.check(L.trx_gat_prologue_backward(pa, stream), "trx_gat_prologue_backward")
    pp = sink.take(PP)
    sums.add(ppart, PP, PP, pp)
    ed, nd = cx.edge_x.shape[1], cx.node_x.shape[1]
    _grad(net.edge_norm.weight, pp[8 * A:8 * A + ed])
    _grad(net.edge_norm.bias, pp[8 * A + 8:8 * A + 8 + ed])
    _grad(net.node_norm.weight, pp[8 * A + 16:8 * A + 16 + nd])
    _grad(net.node_norm.bias, pp[8 * A + 24:8 * A + 24 + nd])
    # M[h, j] = sum_c W[h*C + c, j] * att[h, c] (fp32, then bf16-rounded in the forward):
    # every layer's lin_edge / att_edge gradient from the summed M-row gradients, one launch
    ea_args = _lib.TrxGatPrologueArgs()
    ea_args.num_layers, ea_args.edge_dim = len(layers), ed
    keep = []
    for i, l in enumerate(layers):
        w, at = l.lin_edge.weight.detach().contiguous(), l.att_edge.detach().contiguous()
        keep += [w, at]
        ea_args.heads[i], ea_args.channels[i] = l.heads, l.out_channels
        ea_args.lin_edge_w[i], ea_args.att_edge[i] = w.data_ptr(), at.data_ptr()
    tot = sum(l.heads * l.out_channels * (ed + 1) for l in layers)
    gout = sink.take(tot)

    def att_weights():   # needs the summed prologue partials (pp)
        _lib.check(L.trx_edge_att_weights_backward(ea_args, _lib.ptr(pp), 8, _lib.ptr(gout),
                                                   _lib.stream_ptr(dev)), "trx_edge_att_weights_backward")
    sums.after.append(att_weights)
    sums.used += [gout] + keep
    off = 0
    for l in layers:
        HC = l.heads * l.out_channels
        _grad(l.lin_edge.weight, gout[off:off + HC * ed].view(HC, ed))
        _grad(l.att_edge, gout[off + HC * ed:off + HC * (ed + 1)])
        off += HC * (ed + 1)
    if own:
        sums.flush(stream)


def compute_gradients_fused(agent, batch, weights, topo: Topology, on_td=None):
    """DiscreteSAC.compute_gradients (sac.py:157-243) on the fused path: the
    same returned metrics (device tensors), every gradient set.  on_td(td):
    work that needs only the TD errors (the trainer's priority write-back),
    run as one more branch beside the backwards."""
    (node_x, edge_index, edge_attr, action_mask, batch_vec, action, reward, next_node_x, next_edge_attr,
     next_action_mask, next_batch_vec, done) = batch
    B = reward.shape[0]
    E = topo.e
    dev = reward.device
    nx, ex = node_x.float().contiguous(), edge_attr.float().contiguous()
    nnx, nex = next_node_x.float().contiguous(), next_edge_attr.float().contiguous()
    # the training forwards of the actor and the two critics (raw logits, with
    # saves) and the no-grad next-state passes (sac.py:184-191: next actor probs,
    # two target critics) are independent: six branches on the side streams
    # (each network's kernels fill a fraction of the GPU at batch 256).  The
    # actor's training pass is issued first on every stream: its float32
    # forward + backward is the update's longest chain, and a replayed graph
    # starts its branches in issue order, ~0.2 ms apart
    xa, xc = (exact_nets(agent)[k] for k in ("actor", "critic"))
    # grouped (MULTI 1 / 2): the five bf16 passes -- the critics' training forwards and
    # the next-state actor / target passes -- share their launches (net_forward_multi),
    # beside the actor's float32 training pass: two or three branches instead of six
    grouped = MULTI in (1, 2) and not xc and multi_supported([agent.critic1, agent.critic2, agent.actor, agent.target1,
                                                     agent.target2])
    with torch.no_grad():
        if grouped:
            specs = [(agent.critic1, nx, ex, True, None), (agent.critic2, nx, ex, True, None),
                     (agent.actor, nnx, nex, False, next_action_mask), (agent.target1, nnx, nex, False, None),
                     (agent.target2, nnx, nex, False, None)]
            if MULTI == 2:
                (lg, ca), crit, nxt = agent._concurrent(
                    [lambda: net_forward(agent.actor, nx, ex, topo, save=True, exact=xa),
                     lambda: net_forward_multi(specs[:2], topo), lambda: net_forward_multi(specs[2:], topo)])
                group = crit + nxt
            else:
                (lg, ca), group = agent._concurrent(
                    [lambda: net_forward(agent.actor, nx, ex, topo, save=True, exact=xa),
                     lambda: net_forward_multi(specs, topo)])
            (q1, c1), (q2, c2), (nprobs, _), (qt1, _), (qt2, _) = group
        else:
            outs = agent._concurrent(
                [lambda net=net, x=x: net_forward(net, nx, ex, topo, save=True, exact=x)
                 for net, x in ((agent.actor, xa), (agent.critic1, xc), (agent.critic2, xc))] + [
                    # the next-state probabilities only enter the critics' target: the
                    # critics' precision (bf16 unless the agent trains in float32)
                    lambda: net_forward(agent.actor, nnx, nex, topo, save=False, mask=next_action_mask, exact=xc)[0],
                    lambda: net_forward(agent.target1, nnx, nex, topo, save=False, exact=xc)[0],
                    lambda: net_forward(agent.target2, nnx, nex, topo, save=False, exact=xc)[0]])
            (lg, ca), (q1, c1), (q2, c2) = outs[:3]
            nprobs, qt1, qt2 = outs[3:]
    L = _lib.load()
    la = agent.log_alpha.detach().reshape(1)
    act_local = action % E      # the batch tuple carries graph offsets (arange(B) * E + action)
    g_q1, g_q2, g_lg = torch.empty_like(q1), torch.empty_like(q2), torch.empty_like(lg)
    td = torch.empty(B, device=dev, dtype=torch.float32)
    part = torch.empty(B, 8, device=dev, dtype=torch.float32)
    out = torch.empty(8, device=dev, dtype=torch.float32)
    nets = (agent.critic1, agent.critic2, agent.actor)
    sizes = [flat_size(net) for net in nets]
    flat = torch.empty(sum(sizes) + 1, device=dev, dtype=torch.float32)
    sinks = []
    o = 0
    for sz in sizes:   # one GradFlat window per network (their backwards run on three streams)
        gf = GradFlat.__new__(GradFlat)
        gf.buf, gf.off = flat[o:o + sz], 0
        sinks.append(gf)
        o += sz
    g_la = flat[o:o + 1]
    if weights is None:
        w = torch.ones(B, device=dev)
    else:   # a 0-dim weight applies to every sample, as in sac.py:180-181
        w = torch.as_tensor(weights, device=dev).float()
        w = (w.expand(B) if w.dim() == 0 else w.reshape(B)).contiguous()
    sa = _lib.TrxSacLossArgs()
    sa.num_graphs, sa.edges_per_graph = B, E
    npf = nprobs.contiguous()
    r32, d32 = reward.float().contiguous(), done.float().contiguous()
    mk = action_mask.float().contiguous()
    act = act_local.to(torch.int64).contiguous()
    keep = [npf, r32, d32, mk, act, w, la]
    for name, t in (("next_probs", npf), ("qt1", qt1), ("qt2", qt2), ("reward", r32), ("done", d32), ("q1", q1),
                    ("q2", q2), ("logits", lg), ("mask", mk), ("action", act), ("weights", w), ("log_alpha", la),
                    ("g_q1", g_q1), ("g_q2", g_q2), ("g_logits", g_lg), ("td_error", td), ("part", part),
                    ("out", out), ("g_log_alpha", g_la)):
        setattr(sa, name, t.data_ptr())
    sa.gamma = float(agent.gamma)
    if agent.target_entropy is None:
        sa.target_entropy_given, sa.target_entropy_ratio = 0, float(agent.target_entropy_ratio)
    else:
        sa.target_entropy_given, sa.target_entropy = 1, float(agent.target_entropy)
    _lib.check(L.trx_sac_loss(sa, _lib.stream_ptr(dev)), "trx_sac_loss")
    del keep
    agent.critic_opt.zero_grad(set_to_none=True)
    agent.actor_opt.zero_grad(set_to_none=True)
    agent.alpha_opt.zero_grad(set_to_none=True)
    # each network's backward on the stream its training forward ran on: the
    # saved tensors are read on the stream that allocated them
    sums = PartialSums(B)
    if grouped:
        fns = [lambda: net_backward(agent.actor, ca, g_lg, topo, sinks[2], exact=xa, sums=sums),
               lambda: net_backward_multi([agent.critic1, agent.critic2], [c1, c2], [g_q1, g_q2], topo, sinks[:2],
                                          sums)]
    else:
        # each backward column-sums its own partials at the end of its branch (sums=None):
        # one launch per network, but off the joined tail -- 1.857 -> 1.81 ms per update
        # against one launch for all three after the join
        fns = [lambda: net_backward(agent.actor, ca, g_lg, topo, sinks[2], exact=xa),
               lambda: net_backward(agent.critic1, c1, g_q1, topo, sinks[0], exact=xc),
               lambda: net_backward(agent.critic2, c2, g_q2, topo, sinks[1], exact=xc)]
    streams = list(range(len(fns)))
    if on_td is not None:   # behind the last critic backward: off the actor's (longest) chain
        fns.append(lambda: on_td(td))
        streams.append(streams[-1])   # (its own fourth stream measured 20-40 us slower)
    agent._concurrent(fns, streams)
    sums.flush(_lib.stream_ptr(dev))   # the grouped backward's column sums, on the joined stream
    agent.log_alpha.grad = g_la.view_as(agent.log_alpha)
    agent.grad_flat = flat        # every gradient of this update is a view of it (GradAllReduce)
    agent._warm = True
    return {"critic_loss": out[0], "actor_loss": out[1], "alpha": out[7], "alpha_loss": out[2],
            "policy_entropy": out[3], "q_taken": out[4], "q_mean": out[5], "logp_mean": out[6], "td_errors": td}

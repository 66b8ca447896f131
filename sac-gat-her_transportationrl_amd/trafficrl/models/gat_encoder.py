"""GAT encoder (src/models/gat_encoder.py:9-53) on gfx950 kernels.

`GATConv` keeps torch_geometric's GATConv parameter layout and state_dict keys
(lin.weight [H*C,in], lin_edge.weight [H*C,edge_dim], att_src/att_dst/att_edge
[1,H,C], bias) and its forward semantics (PyG 2.5 defaults used by the
reference: add_self_loops=True with fill_value='mean' edge attributes,
negative_slope=0.2, softmax over each destination's in-edges with a +1e-16
denominator, concat or head-mean, bias).  The reference's checkpoints
(history-data/outputs1/*.pt) load into these modules.

Split of work:
  * dense projections (lin, the per-head attention dot products, the edge
    logits) -- torch GEMMs (hipBLASLt, bf16 MFMA under autocast);
  * edge softmax + neighbour aggregation (+ bias), forward and backward --
    trx_gat_forward / trx_gat_backward HIP kernels (csrc/gat_kernel.hip) over a
    cached CSR-by-destination of the batch graph.
The edge logits use a_edge = edge_attr @ M^T with M[h] = sum_c W_edge[h,c,:] *
att_edge[h,c] -- algebraically PyG's (lin_edge(edge_attr) * att_edge).sum(-1)
without materialising the [E, H*C] edge embedding.

torch_geometric is not importable in this environment, so GAT numerics are
pinned only against tests/test_gat.py's plain-torch restatement of PyG
semantics ("parity unpinned" w.r.t. the reference's own outputs).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch
from torch import nn
import torch.nn.functional as F

from .. import _lib
from .skinny import perm_gather, skinny_linear, splitk_linear
from .tensor_cache import TensorKeyed

# in-feature widths up to which a projection's weight gradient takes the
# split-K path (trafficrl/models/skinny.py)
_SKINNY_IN = 8


# --------------------------------------------------------------- graph CSR
@dataclass
class GraphCSR:
    num_nodes: int
    keep: torch.Tensor      # [E0] bool: non-self-loop input edges (PyG remove_self_loops)
    src_all: torch.Tensor   # [Et] source of each edge in PyG order (kept edges, then loops)
    dst_all: torch.Tensor   # [Et]
    perm: torch.Tensor      # [Et] CSR position -> PyG-order edge id
    rowptr: torch.Tensor    # [N+1] int32 CSR by destination
    col: torch.Tensor       # [Et]  int32 source per CSR position
    sptr: torch.Tensor      # [N+1] int32 CSR by source
    spos: torch.Tensor      # [Et]  int32 dst-CSR position per source-CSR entry
    sdst: torch.Tensor      # [Et]  int32 destination per source-CSR entry
    deg_in: torch.Tensor    # [N] float in-degree of kept edges (for the mean loop attr)
    kept_idx: Optional[torch.Tensor]  # [E_kept] int64 kept input edges, None when no input self loops
    in_pad: torch.Tensor    # [N, D] int64 kept-edge ids entering each node, padded with E_kept (zero row)
    dst_kept: torch.Tensor  # [E_kept] int64 destination of each kept edge
    inv_perm: torch.Tensor  # [Et] int64 inverse of perm (PyG-order edge id -> CSR position)


_csr_cache = TensorKeyed()


def build_csr(edge_index: torch.Tensor, num_nodes: int) -> GraphCSR:
    key = (edge_index.data_ptr(), edge_index.shape[1], edge_index._version, num_nodes, edge_index.device)
    g = _csr_cache.get(key)
    if g is not None:
        return g
    dev = edge_index.device
    src0, dst0 = edge_index[0].long(), edge_index[1].long()
    keep = src0 != dst0
    loops = torch.arange(num_nodes, device=dev)
    src_all = torch.cat([src0[keep], loops])
    dst_all = torch.cat([dst0[keep], loops])
    Et = src_all.numel()
    # stable sort by destination -> CSR by destination
    perm = torch.argsort(dst_all * (Et + 1) + torch.arange(Et, device=dev))
    counts = torch.bincount(dst_all, minlength=num_nodes)
    rowptr = torch.zeros(num_nodes + 1, dtype=torch.int64, device=dev)
    rowptr[1:] = torch.cumsum(counts, 0)
    col = src_all[perm]
    # CSR by source over dst-CSR positions
    sperm = torch.argsort(col * (Et + 1) + torch.arange(Et, device=dev))
    scounts = torch.bincount(col, minlength=num_nodes)
    sptr = torch.zeros(num_nodes + 1, dtype=torch.int64, device=dev)
    sptr[1:] = torch.cumsum(scounts, 0)
    sdst = dst_all[perm][sperm]
    deg_cnt = torch.bincount(dst0[keep], minlength=num_nodes)
    deg_in = deg_cnt.to(torch.float32)
    # padded in-edge table: deterministic (gather + sum) replacement of the
    # scatter-mean PyG uses for the 'mean' self-loop edge attributes
    kept_idx = None if bool(keep.all()) else torch.nonzero(keep).squeeze(1)
    dk = dst0[keep]
    Ek = dk.numel()
    D = max(1, int(deg_cnt.max()) if num_nodes else 1)
    order = torch.argsort(dk * (Ek + 1) + torch.arange(Ek, device=dev))
    kstart = torch.zeros(num_nodes + 1, dtype=torch.int64, device=dev)
    kstart[1:] = torch.cumsum(deg_cnt, 0)
    slot = torch.arange(Ek, device=dev) - kstart[dk[order]]
    in_pad = torch.full((num_nodes, D), Ek, dtype=torch.int64, device=dev)
    in_pad[dk[order], slot] = order
    inv_perm = torch.empty_like(perm)
    inv_perm[perm] = torch.arange(Et, device=dev)
    g = GraphCSR(num_nodes, keep, src_all, dst_all, perm, rowptr.to(torch.int32), col.to(torch.int32),
                 sptr.to(torch.int32), sperm.to(torch.int32), sdst.to(torch.int32), deg_in, kept_idx, in_pad, dk,
                 inv_perm)
    _csr_cache.put(key, (edge_index,), g)
    return g


# ---------------------------------------------------- HIP aggregation op
class _GATAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xh, a_src, a_dst, a_edge, g: GraphCSR, heads: int, channels: int, slope: float):
        L = _lib.load()
        N = g.num_nodes
        xh = xh.contiguous()
        bf16 = 1 if xh.dtype == torch.bfloat16 else 0
        if not bf16 and xh.dtype != torch.float32:
            xh = xh.float()
        a_src = a_src.float().contiguous()
        a_dst = a_dst.float().contiguous()
        a_edge = a_edge.float().contiguous()
        out = torch.empty(N, heads * channels, device=xh.device, dtype=torch.float32)
        alpha = torch.empty(a_edge.shape[0], heads, device=xh.device, dtype=torch.float32)
        _lib.check(L.trx_gat_forward(N, heads, channels, _lib.ptr(g.rowptr), _lib.ptr(g.col), _lib.ptr(xh), bf16,
                                     _lib.ptr(a_src), _lib.ptr(a_dst), _lib.ptr(a_edge), float(slope), None,
                                     _lib.ptr(out), _lib.ptr(alpha), _lib.stream_ptr(xh.device)), "trx_gat_forward")
        ctx.save_for_backward(xh, a_src, a_dst, a_edge, alpha)
        ctx.g, ctx.heads, ctx.channels, ctx.slope, ctx.bf16 = g, heads, channels, slope, bf16
        ctx.xh_dtype = xh.dtype
        ctx.mark_non_differentiable(alpha)
        return out, alpha

    @staticmethod
    def backward(ctx, gout, _galpha):
        L = _lib.load()
        xh, a_src, a_dst, a_edge, alpha = ctx.saved_tensors
        g = ctx.g
        N = g.num_nodes
        gout = gout.float().contiguous()
        gxh = torch.empty(N, ctx.heads * ctx.channels, device=gout.device, dtype=xh.dtype)  # written in xh's dtype
        ga_src = torch.empty_like(a_src)
        ga_dst = torch.empty_like(a_dst)
        ga_edge = torch.empty_like(a_edge)
        _lib.check(L.trx_gat_backward(N, ctx.heads, ctx.channels, _lib.ptr(g.rowptr), _lib.ptr(g.col),
                                      _lib.ptr(g.sptr), _lib.ptr(g.spos), _lib.ptr(g.sdst), _lib.ptr(xh), ctx.bf16,
                                      _lib.ptr(a_src), _lib.ptr(a_dst), _lib.ptr(a_edge), float(ctx.slope),
                                      _lib.ptr(alpha), _lib.ptr(gout), _lib.ptr(gxh), _lib.ptr(ga_src),
                                      _lib.ptr(ga_dst), _lib.ptr(ga_edge), _lib.stream_ptr(gout.device)),
                   "trx_gat_backward")
        return gxh.to(ctx.xh_dtype), ga_src, ga_dst, ga_edge, None, None, None, None  # no-op cast unless xh was promoted


def gat_aggregate(xh, a_src, a_dst, a_edge_csr, g: GraphCSR, heads, channels, slope=0.2):
    return _GATAggregate.apply(xh, a_src, a_dst, a_edge_csr, g, heads, channels, slope)


class _AttDots(torch.autograd.Function):
    """a_src[i,h] = <xh[i,h,:], att_src[h,:]>, a_dst likewise, float32 --
    GATConv's attention dot products as one kernel each way
    (csrc/att_dots.hip) instead of a cast + block-diagonal GEMM."""

    @staticmethod
    def forward(ctx, xh, att_src, att_dst, heads: int, channels: int):
        L = _lib.load()
        if xh.dtype not in (torch.float32, torch.bfloat16):
            xh = xh.float()
        xh = xh.contiguous()
        N = xh.shape[0]
        s_, d_ = att_src.detach().float().reshape(-1).contiguous(), att_dst.detach().float().reshape(-1).contiguous()
        a_src = torch.empty(N, heads, device=xh.device, dtype=torch.float32)
        a_dst = torch.empty_like(a_src)
        dt = 1 if xh.dtype == torch.bfloat16 else 0
        _lib.check(L.trx_att_dots_forward(N, heads, channels, _lib.ptr(xh), dt, _lib.ptr(s_), _lib.ptr(d_),
                                          _lib.ptr(a_src), _lib.ptr(a_dst), _lib.stream_ptr(xh.device)),
                   "trx_att_dots_forward")
        ctx.save_for_backward(xh, s_, d_)
        ctx.dims, ctx.dt, ctx.att_shape = (heads, channels), dt, att_src.shape
        return a_src, a_dst

    @staticmethod
    def backward(ctx, g_src, g_dst):
        L = _lib.load()
        xh, s_, d_ = ctx.saved_tensors
        H, C = ctx.dims
        N = xh.shape[0]
        g_src = torch.zeros(N, H, device=xh.device) if g_src is None else g_src.float().contiguous()
        g_dst = torch.zeros(N, H, device=xh.device) if g_dst is None else g_dst.float().contiguous()
        gxh = torch.empty_like(xh)
        gatt = torch.empty(2, H * C, device=xh.device, dtype=torch.float32)
        ws = torch.empty(max(1, int(L.trx_att_dots_workspace_floats(N, H, C))), device=xh.device,
                         dtype=torch.float32)
        _lib.check(L.trx_att_dots_backward(N, H, C, _lib.ptr(xh), ctx.dt, _lib.ptr(s_), _lib.ptr(d_), _lib.ptr(g_src),
                                           _lib.ptr(g_dst), _lib.ptr(gxh), _lib.ptr(gatt), _lib.ptr(ws),
                                           _lib.stream_ptr(xh.device)), "trx_att_dots_backward")
        return gxh, gatt[0].view(ctx.att_shape), gatt[1].view(ctx.att_shape), None, None


def att_dots(xh, att_src, att_dst, heads: int, channels: int):
    return _AttDots.apply(xh, att_src, att_dst, heads, channels)


class _LayerTail(torch.autograd.Function):
    """GATEncoder's per-layer tail (gat_encoder.py:40-49 of the reference):
    y = relu(LayerNorm(out + bias) + res) (act 0) or elu(LayerNorm(out +
    bias)) (act 1), forward and backward as single kernels
    (csrc/layer_tail.hip); same math as the torch ops it replaces, fp32."""

    @staticmethod
    def forward(ctx, out, bias, w, b, eps: float, res, act: int):
        L = _lib.load()
        out = out.float().contiguous()
        N, F = out.shape
        y = torch.empty_like(out)
        stats = torch.empty(N, 2, device=out.device, dtype=torch.float32)
        rdt = 0
        if res is not None:
            if res.dtype != torch.bfloat16:
                res = res.float()
            res = res.contiguous()
            rdt = 1 if res.dtype == torch.bfloat16 else 0
        bias_c, w_c, b_c = bias.float().contiguous(), w.float().contiguous(), b.float().contiguous()
        _lib.check(L.trx_layer_tail_forward(N, F, act, rdt, _lib.ptr(out), _lib.ptr(bias_c), _lib.ptr(w_c),
                                            _lib.ptr(b_c), float(eps), _lib.ptr(res), _lib.ptr(y), _lib.ptr(stats),
                                            _lib.stream_ptr(out.device)), "trx_layer_tail_forward")
        ctx.save_for_backward(out, bias_c, w_c, y, stats)
        ctx.act, ctx.rdt = act, rdt
        ctx.res_dtype = None if res is None else res.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        L = _lib.load()
        out, bias, w, y, stats = ctx.saved_tensors
        N, F = out.shape
        gy = gy.float().contiguous()
        gout = torch.empty_like(out)
        gres = torch.empty(N, F, device=out.device, dtype=ctx.res_dtype) if ctx.act == 0 else None
        grads = torch.empty(3, F, device=out.device, dtype=torch.float32)
        ws = torch.empty(max(1, int(L.trx_layer_tail_workspace_floats(N, F))), device=out.device,
                         dtype=torch.float32)
        _lib.check(L.trx_layer_tail_backward(N, F, ctx.act, ctx.rdt, _lib.ptr(gy), _lib.ptr(out), _lib.ptr(bias),
                                             _lib.ptr(w), _lib.ptr(y), _lib.ptr(stats), _lib.ptr(gout),
                                             _lib.ptr(gres), _lib.ptr(grads), _lib.ptr(ws),
                                             _lib.stream_ptr(out.device)), "trx_layer_tail_backward")
        return gout, grads[0], grads[1], grads[2], None, gres, None


def layer_tail(out, bias, norm: nn.LayerNorm, res=None):
    """relu(norm(out + bias) + res) when res is given, else elu(norm(out + bias))."""
    return _LayerTail.apply(out, bias, norm.weight, norm.bias, norm.eps, res, 0 if res is not None else 1)


class _GraphPool(torch.autograd.Function):
    """cat([global_mean_pool, global_max_pool], 1) for a regular batch as one
    kernel each way (csrc/graph_pool.hip)."""

    @staticmethod
    def forward(ctx, x, B: int):
        L = _lib.load()
        x = x.float().contiguous()
        N, F_ = x.shape
        out = torch.empty(B, 2 * F_, device=x.device, dtype=torch.float32)
        ties = torch.empty(B, F_, device=x.device, dtype=torch.float32)
        _lib.check(L.trx_graph_pool_forward(B, N // B, F_, _lib.ptr(x), _lib.ptr(out), _lib.ptr(ties),
                                            _lib.stream_ptr(x.device)), "trx_graph_pool_forward")
        ctx.save_for_backward(x, out, ties)
        ctx.B = B
        return out

    @staticmethod
    def backward(ctx, g):
        L = _lib.load()
        x, out, ties = ctx.saved_tensors
        N, F_ = x.shape
        gx = torch.empty_like(x)
        _lib.check(L.trx_graph_pool_backward(ctx.B, N // ctx.B, F_, _lib.ptr(x), _lib.ptr(out), _lib.ptr(ties),
                                             _lib.ptr(g.float().contiguous()), _lib.ptr(gx),
                                             _lib.stream_ptr(x.device)), "trx_graph_pool_backward")
        return gx, None


class _LoopMean(torch.autograd.Function):
    """PyG add_remaining_self_loops(fill_value='mean'): loop_attr[i] = sum of
    the kept in-edge attrs of i / max(count, 1).  Forward gathers through the
    padded in-edge table (fixed order, deterministic); backward is a plain
    gather, grad_ea[e] = grad[dst[e]] / deg[dst[e]], because every kept edge
    has exactly one destination -- autograd's default (an accumulating
    index_put through the pad row) serialises on the duplicated pad index."""

    @staticmethod
    def forward(ctx, ea, g: GraphCSR):
        ea_pad = torch.cat([ea, ea.new_zeros(1, ea.size(1))], 0)
        deg = g.deg_in.clamp(min=1.0).unsqueeze(1)
        ctx.g = g
        return ea_pad[g.in_pad].sum(1) / deg

    @staticmethod
    def backward(ctx, grad):
        g = ctx.g
        return (grad / g.deg_in.clamp(min=1.0).unsqueeze(1)).index_select(0, g.dst_kept), None


# ------------------------------------------------------------- modules
def _glorot_(t: torch.Tensor):
    # PyG inits.glorot on a [1,H,C] attention vector / [out,in] weight
    fan = t.size(-2) + t.size(-1)
    a = math.sqrt(6.0 / fan)
    with torch.no_grad():
        t.uniform_(-a, a)


class _Lin(nn.Module):
    """PyG Linear without bias: state_dict key `weight` [out, in]."""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(out_ch, in_ch))
        _glorot_(self.weight)

    def forward(self, x):
        return splitk_linear(x, self.weight)


def _f32up(t: torch.Tensor) -> torch.Tensor:
    """At least float32 (half types up, float64 kept)."""
    return t.float() if t.dtype in (torch.bfloat16, torch.float16) else t


class GATConv(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 negative_slope: float = 0.2, dropout: float = 0.0, add_self_loops: bool = True,
                 edge_dim: Optional[int] = None, fill_value: str = "mean", bias: bool = True):
        super().__init__()
        if not add_self_loops or fill_value != "mean" or dropout != 0.0:
            raise NotImplementedError("only the reference's GATConv configuration is ported "
                                      "(add_self_loops=True, fill_value='mean', dropout=0)")
        self.in_channels, self.out_channels, self.heads, self.concat = in_channels, out_channels, heads, concat
        self.negative_slope = negative_slope
        self.edge_dim = edge_dim
        self.lin = _Lin(in_channels, heads * out_channels)
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        if edge_dim is not None:
            self.lin_edge = _Lin(edge_dim, heads * out_channels)
            self.att_edge = nn.Parameter(torch.empty(1, heads, out_channels))
        else:
            self.lin_edge = None
            self.register_parameter("att_edge", None)
        self.bias = nn.Parameter(torch.zeros(heads * out_channels if concat else out_channels)) if bias else None
        _glorot_(self.att_src)
        _glorot_(self.att_dst)
        if self.att_edge is not None:
            _glorot_(self.att_edge)

    def forward(self, x, edge_index, edge_attr=None, return_attention_weights=None, a_edge_csr=None,
                skip_bias: bool = False):
        """a_edge_csr: this layer's edge logits [Et, H] already in CSR order
        (GATEncoder computes every layer's in one product); else computed here.
        skip_bias: return the output before `+ bias` (GATEncoder fuses the add
        into the layer tail kernel)."""
        H, C = self.heads, self.out_channels
        N = x.size(0)
        g = build_csr(edge_index, N)
        if self.in_channels <= _SKINNY_IN:
            # 4 input features: kept in fp32 under autocast (the reference's precision;
            # the fused inference kernel's linear form, csrc/gat_layer0.hip, does the same)
            with torch.autocast("cuda", enabled=False):
                xh = skinny_linear(_f32up(x), self.lin.weight)   # [N, H*C]
        else:
            xh = self.lin(x)                               # [N, H*C]  (MFMA GEMM)
        # per-head attention dot products <xh_h, att_h> for src and dst: one
        # kernel each way on the GPU; elsewhere ONE float32 product with a
        # block-diagonal [H*C, 2H] matrix; same fp32 values as (xh3 * att).sum(-1)
        if xh.is_cuda and H <= 8 and C % 4 == 0 and H * C <= 1024:
            a_src, a_dst = att_dots(xh, self.att_src, self.att_dst, H, C)   # csrc/att_dots.hip
        else:
            eye = torch.eye(H, device=xh.device, dtype=torch.float32)
            A = torch.cat([(self.att_src.view(H, C, 1).float() * eye.view(H, 1, H)).reshape(H * C, H),
                           (self.att_dst.view(H, C, 1).float() * eye.view(H, 1, H)).reshape(H * C, H)], 1)
            with torch.autocast("cuda", enabled=False):
                a_sd = skinny_linear(xh.float(), A.t())        # [N, 2H]
            a_src, a_dst = a_sd[:, :H], a_sd[:, H:]
        if a_edge_csr is not None:
            a_edge = None
        elif self.lin_edge is not None and edge_attr is not None:
            ea = (edge_attr if g.kept_idx is None else edge_attr.index_select(0, g.kept_idx)).float()
            # fill_value='mean': loop attr = mean of the node's incoming edge attrs
            loop = _LoopMean.apply(ea, g)
            full = torch.cat([ea, loop], 0)
            M = (self.lin_edge.weight.view(H, C, -1).float() * self.att_edge.view(H, C, 1).float()).sum(1)
            a_edge = skinny_linear(full, M)                # [Et, H]
        else:
            a_edge = torch.zeros(g.src_all.numel(), H, device=x.device)
        if a_edge_csr is None:
            a_edge_csr = perm_gather(a_edge, g.perm, g.inv_perm)
        out, alpha = gat_aggregate(xh, a_src, a_dst, a_edge_csr, g, H, C, self.negative_slope)
        if not self.concat:
            out = out.view(N, H, C).mean(1) if H > 1 else out.view(N, C)
        if self.bias is not None and not skip_bias:
            out = out + self.bias
        if return_attention_weights:
            a_pyg = torch.empty_like(alpha)
            a_pyg[g.perm] = alpha
            ei = torch.stack([g.src_all, g.dst_all])
            return out, (ei, a_pyg)
        return out


_layout_cache = TensorKeyed()


def is_regular_batch(batch: torch.Tensor, num_graphs: int) -> bool:
    """True when `batch` is arange(B).repeat_interleave(n) (the trainer's
    fixed-topology batches): pooling then reduces a [B, n, F] view without
    atomics.  One host check per distinct batch tensor, cached."""
    n_tot = batch.numel()
    if num_graphs <= 0 or n_tot % num_graphs:
        return False
    key = (batch.data_ptr(), n_tot, batch._version, num_graphs, batch.device)
    r = _layout_cache.get(key)
    if r is None:
        ref = torch.arange(num_graphs, device=batch.device).repeat_interleave(n_tot // num_graphs)
        r = bool(torch.equal(batch.long(), ref))
        _layout_cache.put(key, (batch,), r)
    return r


def global_mean_pool(x, batch, num_graphs: Optional[int] = None):
    B = int(batch.max()) + 1 if num_graphs is None else num_graphs
    if is_regular_batch(batch, B):
        return x.view(B, -1, x.size(1)).sum(1) / float(x.size(0) // B)
    out = torch.zeros(B, x.size(1), device=x.device, dtype=x.dtype)
    out.index_add_(0, batch, x)
    cnt = torch.bincount(batch, minlength=B).clamp(min=1).to(x.dtype).unsqueeze(1)
    return out / cnt


def global_max_pool(x, batch, num_graphs: Optional[int] = None):
    B = int(batch.max()) + 1 if num_graphs is None else num_graphs
    if is_regular_batch(batch, B):
        return x.view(B, -1, x.size(1)).amax(1)
    out = torch.full((B, x.size(1)), float("-inf"), device=x.device, dtype=x.dtype)
    return out.scatter_reduce(0, batch.unsqueeze(1).expand_as(x), x, reduce="amax", include_self=True)


class GATEncoder(nn.Module):
    """src/models/gat_encoder.py:9-53, same submodule names and forward."""

    def __init__(self, in_dim: int, hidden_dim: int, out_dim: int, edge_dim: int, heads: int = 4,
                 num_layers: int = 3):
        super().__init__()
        self.num_layers = max(2, num_layers)
        self.layers = nn.ModuleList()
        self.layers.append(GATConv(in_dim, hidden_dim, heads=heads, concat=True, edge_dim=edge_dim))
        for _ in range(self.num_layers - 2):
            self.layers.append(GATConv(hidden_dim * heads, hidden_dim, heads=heads, concat=True, edge_dim=edge_dim))
        self.layers.append(GATConv(hidden_dim * heads, out_dim, heads=1, concat=False, edge_dim=edge_dim))
        self.input_proj = nn.Linear(in_dim, hidden_dim * heads)
        self.norms = nn.ModuleList()
        for i in range(self.num_layers):
            self.norms.append(nn.LayerNorm(out_dim if i == self.num_layers - 1 else hidden_dim * heads))

    def edge_logits(self, edge_index, edge_attr, num_nodes: int):
        """Every layer's a_edge in CSR order, as one product: the self-loop
        mean attrs, the cast and the skinny GEMM happen once per forward
        instead of once per layer.  Column block l holds layer l's heads."""
        g = build_csr(edge_index, num_nodes)
        ea = (edge_attr if g.kept_idx is None else edge_attr.index_select(0, g.kept_idx)).float()
        full = torch.cat([ea, _LoopMean.apply(ea, g)], 0)
        M = torch.cat([(l.lin_edge.weight.view(l.heads, l.out_channels, -1).float()
                        * l.att_edge.view(l.heads, l.out_channels, 1).float()).sum(1) for l in self.layers], 0)
        return perm_gather(skinny_linear(full, M), g.perm, g.inv_perm)

    def forward(self, x, edge_index, edge_attr, batch, return_attention: bool = False,
                num_graphs: Optional[int] = None):
        attn = None
        shared = edge_attr is not None and all(l.lin_edge is not None for l in self.layers)
        a_all = self.edge_logits(edge_index, edge_attr, x.size(0)) if shared else None
        # torch.split: one cat in the backward instead of a zero-fill + copy per slice
        a_layers = torch.split(a_all, [l.heads for l in self.layers], dim=1) if shared else None
        for i, layer in enumerate(self.layers):
            last = i == len(self.layers) - 1
            ae = a_layers[i] if shared else None
            norm = self.norms[i]
            F_out = layer.heads * layer.out_channels if layer.concat else layer.out_channels
            tail = (x.is_cuda and layer.bias is not None and norm.elementwise_affine and F_out % 4 == 0
                    and F_out <= 1024 and not (last and return_attention))
            if last and return_attention:
                x, attn_info = layer(x, edge_index, edge_attr=edge_attr, return_attention_weights=True, a_edge_csr=ae)
                attn = attn_info[1]
            elif last:
                x = layer(x, edge_index, edge_attr=edge_attr, a_edge_csr=ae, skip_bias=tail)
                if tail:
                    x = layer_tail(x, layer.bias, norm)
                    continue
            else:
                x_in = x
                x = layer(x, edge_index, edge_attr=edge_attr, a_edge_csr=ae, skip_bias=tail)
                if i == 0:
                    ip = self.input_proj
                    if ip.in_features <= _SKINNY_IN:   # fp32, like layer 0's projection
                        with torch.autocast("cuda", enabled=False):
                            x_in = skinny_linear(_f32up(x_in), ip.weight, ip.bias)
                    else:
                        x_in = ip(x_in)
                if tail:
                    x = layer_tail(x, layer.bias, norm, x_in)
                    continue
                x = norm(x)
                x = torch.relu(x + x_in)
                continue
            x = norm(x)
            x = F.elu(x)
        B = int(batch.max()) + 1 if num_graphs is None else num_graphs
        if x.is_cuda and x.dtype == torch.float32 and B > 0 and is_regular_batch(batch, B):
            return x, _GraphPool.apply(x, B), attn                       # csrc/graph_pool.hip
        g_mean = global_mean_pool(x, batch, num_graphs)
        g_max = global_max_pool(x, batch, num_graphs)
        return x, torch.cat([g_mean, g_max], dim=1), attn

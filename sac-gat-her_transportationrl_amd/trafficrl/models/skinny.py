"""Autograd helpers for the GAT-SAC update's odd-shaped products.

Profiling one SAC update (round 2; DESIGN.md §6, profiles/r02_update_kernel_stats.csv)
showed two kinds of ops
costing far more than their FLOPs:

* weight gradients of "skinny" products -- a 4-, 6- or 1-wide side against a
  long K of 6 144-25 600 batch rows (edge-attention projections, the 4-feature
  input layer, the edge MLP's link-feature block and its 256->1 output):
  hipBLASLt runs them as one output tile walking all of K (~155 us each).
  `skinny_linear` computes them as a split-K batched product over 256-row
  chunks plus a sum, in float32.
* backward passes of gathers -- `p[src]`, `ctx[edge_batch]`, `a_edge[perm]` --
  which autograd turns into sorting, deterministic `index_put_` scatters.
  For the trainer's fixed-topology batches (every graph the same, edges in
  contiguous per-graph blocks) `regular_gather` scatters back with a batched
  [nodes x links] incidence product, and `perm_gather` inverts a permutation
  with a gather.

Forward values are unchanged (same products, same dtypes under autocast).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

from .tensor_cache import TensorKeyed

_SPLIT = 256


def _splitk_wgrad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW[o, i] = sum_k dy[k, o] x[k, i] in (at least) float32, split-K when K allows.
    bf16 operands (autocast): the 256-row partial products run in bf16 on the
    MFMA path (float32 accumulation, one bf16 rounding per partial) and are
    summed in float32 -- no float32 copies of dy and x."""
    K = dy.shape[0]
    acc = torch.float64 if dy.dtype == torch.float64 else torch.float32
    split = K % _SPLIT == 0 and K >= 4 * _SPLIT
    if split and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16:
        S = K // _SPLIT
        part = torch.bmm(dy.reshape(S, _SPLIT, -1).transpose(1, 2), x.reshape(S, _SPLIT, -1))
        return part.sum(0, dtype=torch.float32)
    dy32, x32 = dy.to(acc), x.to(acc)
    if not split:
        return dy32.t() @ x32
    S = K // _SPLIT
    part = torch.bmm(dy32.view(S, _SPLIT, -1).transpose(1, 2), x32.view(S, _SPLIT, -1))
    return part.sum(0)


class _SkinnyMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        # bias in the GEMM epilogue: one rounding of the output, like F.linear
        return x @ w.t() if b is None else torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy @ w.to(dy.dtype) if ctx.needs_input_grad[0] else None
        dw = _splitk_wgrad(dy, x).to(w.dtype) if ctx.needs_input_grad[1] else None
        acc = torch.float64 if dy.dtype == torch.float64 else torch.float32
        db = dy.sum(0, dtype=acc).to(dy.dtype) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


class _SplitKLinear(torch.autograd.Function):
    """y = bf16(x) @ bf16(w)^T (autocast's product, bf16 output) whose weight
    gradient is `splits` bf16 partial products over K/splits batch rows summed
    in float32 and returned as the float32 master weight's gradient: no
    bf16 -> float32 cast of dW, and hipBLASLt's single-tile walk over K = 6144
    (~11 % of the MFMA peak) becomes a batched product (44 -> 29 us for
    6144 x 1024 x 1024 in round 2's probe)."""

    @staticmethod
    def forward(ctx, x, w, splits: int):
        xb, wb = x.to(torch.bfloat16), w.to(torch.bfloat16)
        ctx.save_for_backward(xb, wb)
        ctx.splits = splits
        return xb @ wb.t()

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        dy = dy.to(torch.bfloat16)
        dx = dy @ wb if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            S = ctx.splits
            K = dy.shape[0]
            part = torch.bmm(dy.reshape(S, K // S, -1).transpose(1, 2), xb.reshape(S, K // S, -1))
            dw = part.sum(0, dtype=torch.float32)
        return dx, dw, None


def splitk_linear(x: torch.Tensor, w: torch.Tensor, splits: int = 4) -> torch.Tensor:
    """F.linear(x, w) under bf16 autocast with a split-K float32 weight
    gradient (large square products of the SAC update); plain F.linear
    otherwise (other dtypes, no autograd, batch rows not divisible)."""
    if (torch.is_grad_enabled() and w.requires_grad and w.dtype == torch.float32 and x.dim() == 2
            and x.shape[0] % splits == 0 and x.shape[0] >= 1024 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        with torch.autocast("cuda", enabled=False):
            return _SplitKLinear.apply(x, w, splits)
    return torch.nn.functional.linear(x, w)


def skinny_linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor = None) -> torch.Tensor:
    """F.linear(x, w, b) (autocast-aware) whose weight gradient is a split-K
    float32 reduction; for products with a tiny in- or out-feature side."""
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        x, w = x.to(dt), w.to(dt)
        b = None if b is None else b.to(dt)
    with torch.autocast("cuda", enabled=False):
        return _SkinnyMM.apply(x, w, b)


class _RegularGather(torch.autograd.Function):
    """x [B*n, F] -> x.view(B, n, F)[:, idx].reshape(B*m, F) for a graph-local
    index idx [m]; backward = incidence [n, m] @ grad.view(B, m, F)."""

    @staticmethod
    def forward(ctx, x, idx, inc, B):
        n = x.shape[0] // B
        ctx.inc, ctx.B, ctx.n = inc, B, n
        return x.view(B, n, -1).index_select(1, idx).reshape(B * idx.numel(), -1)

    @staticmethod
    def backward(ctx, grad):
        B, n = ctx.B, ctx.n
        g = grad.reshape(B, -1, grad.shape[-1])
        return torch.matmul(ctx.inc.to(g.dtype), g).reshape(B * n, -1), None, None, None


_inc_cache = TensorKeyed()


def regular_gather(x: torch.Tensor, idx_local: torch.Tensor, B: int) -> torch.Tensor:
    n = x.shape[0] // B
    key = (idx_local.data_ptr(), idx_local._version, n, idx_local.device)
    inc = _inc_cache.get(key)
    if inc is None:
        inc = torch.zeros(n, idx_local.numel(), device=x.device)
        inc[idx_local, torch.arange(idx_local.numel(), device=x.device)] = 1.0
        _inc_cache.put(key, (idx_local,), inc)
    return _RegularGather.apply(x, idx_local, inc, B)


class _PermGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, perm, inv):
        ctx.inv = inv
        return x.index_select(0, perm)

    @staticmethod
    def backward(ctx, grad):
        return grad.index_select(0, ctx.inv), None, None


def perm_gather(x: torch.Tensor, perm: torch.Tensor, inv: torch.Tensor) -> torch.Tensor:
    """x[perm] for a permutation perm (inverse inv); backward is a gather."""
    return _PermGather.apply(x, perm, inv)

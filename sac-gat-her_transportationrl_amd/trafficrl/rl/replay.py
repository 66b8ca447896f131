"""Device-resident prioritized replay + HER relabelling (src/train.py:27-91,
125-135, 805-823).

Transitions of fixed-topology graphs are stored as dense device tensors
(structure of arrays, [capacity, ...]); the PER sum tree runs on the GPU
(trx_per_update / trx_per_sample, csrc/replay_kernel.hip).  Semantics kept
from the reference ReplayBuffer:
  * add(): priority = max_priority, then abs()+eps, max_priority updated,
    leaf = priority**alpha -- so a batch of k adds gets max_p+eps, max_p+2eps,
    ... exactly like k sequential reference adds;
  * sample(): r = u * total, descend `r <= tree[left]`; probs = leaf/total,
    weights = (size * probs)^-beta / max;
  * update_priorities(): abs(err)+eps, max_priority, **alpha; for duplicate
    indices the last one wins (sequential semantics).
tree_dtype="float32" is the reference's own tree bit for bit (float32 nodes,
float32 deltas added down each leaf's ancestor chain in update order, the
float32 NEP 50 descent; trx_per32_*); "float64" recomputes ancestors as sums of
their children (no drift; trx_per_*).
HER (train.py:805-823) reproduces the reference's behaviour including two
quirks, flagged here: apply_goal writes the goal into edge-feature column -1
(edge_id_norm; get_state's goal column is 4, repair_env.py:799-808), and the
relabelled `done` = is_goal_complete(1 - mask', mask') is always 1.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass
from typing import Optional

import torch

from .. import _lib


@dataclass
class Sample:
    idx: torch.Tensor          # [bs] int64 slots
    weights: torch.Tensor      # [bs] float32 importance weights
    node_x: torch.Tensor       # [bs, N, 4]
    edge_x: torch.Tensor       # [bs, E, 6]
    mask: torch.Tensor         # [bs, E]
    action: torch.Tensor       # [bs] int64 (local link id)
    reward: torch.Tensor       # [bs] float32 (scaled)
    next_node_x: torch.Tensor
    next_edge_x: torch.Tensor
    next_mask: torch.Tensor
    done: torch.Tensor         # [bs] float32
    goal: torch.Tensor         # [bs, E]
    prev_tstt: torch.Tensor    # [bs] float64
    next_tstt: torch.Tensor
    init_tstt: torch.Tensor
    pri: Optional[torch.Tensor] = None  # [bs] float64 sampled leaf priorities


def _last_wins(idx: torch.Tensor, val: torch.Tensor) -> torch.Tensor:
    """Give every duplicate of an index the value of its LAST occurrence, so
    concurrent leaf writes all store the same number (the reference's
    sequential update order) -- without a data-dependent shape, hence without
    a host synchronisation (HIP-graph capturable)."""
    n = idx.numel()
    pos = torch.arange(n, device=idx.device)
    order = torch.argsort(idx * (n + 1) + pos)          # stable: by index, then position
    s = idx[order]
    is_last = torch.ones(n, dtype=torch.bool, device=idx.device)
    is_last[:-1] = s[1:] != s[:-1]
    # run end for each sorted position: smallest q >= p with is_last[q]
    cand = torch.where(is_last, pos, torch.full_like(pos, n))
    run_end = torch.flip(torch.cummin(torch.flip(cand, [0]), 0).values, [0])
    out = torch.empty_like(val)
    out[order] = val[order[run_end]]
    return out


class DeviceReplay:
    def __init__(self, capacity: int, num_nodes: int, num_edges: int, node_dim: int = 4, edge_dim: int = 6,
                 alpha: float = 0.6, beta: float = 0.4, eps: float = 1e-6, device="cuda",
                 tree_dtype: str = "float64"):
        if tree_dtype not in ("float32", "float64"):
            raise ValueError(f"tree_dtype must be 'float32' (reference) or 'float64', got {tree_dtype!r}")
        self.tree_dtype = tree_dtype
        self.capacity = int(capacity)
        self.alpha, self.beta, self.eps = alpha, beta, eps
        dev = self.device = torch.device(device)
        C, N, E = self.capacity, num_nodes, num_edges
        f32 = dict(device=dev, dtype=torch.float32)
        self.node_x = torch.zeros(C, N, node_dim, **f32)
        self.edge_x = torch.zeros(C, E, edge_dim, **f32)
        self.mask = torch.zeros(C, E, **f32)
        self.next_node_x = torch.zeros(C, N, node_dim, **f32)
        self.next_edge_x = torch.zeros(C, E, edge_dim, **f32)
        self.next_mask = torch.zeros(C, E, **f32)
        self.goal = torch.zeros(C, E, **f32)
        self.action = torch.zeros(C, dtype=torch.int64, device=dev)
        self.reward = torch.zeros(C, **f32)
        self.done = torch.zeros(C, **f32)
        self.prev_tstt = torch.zeros(C, dtype=torch.float64, device=dev)
        self.next_tstt = torch.zeros(C, dtype=torch.float64, device=dev)
        self.init_tstt = torch.zeros(C, dtype=torch.float64, device=dev)
        self.tree = torch.zeros(2 * C, dtype=getattr(torch, tree_dtype), device=dev)
        self.max_priority = torch.ones((), dtype=torch.float64, device=dev)
        self.ptr = 0
        self.size = 0
        self.size_t = torch.zeros((), dtype=torch.float64, device=dev)  # device copy for graph-captured sampling
        # overlap_adds (the trainer sets it): the float32 tree's ring adds run on a side
        # stream of their own, beside the next acting pass (they read only the tree and
        # max_priority); sync_adds() joins them before anything reads those again
        self.overlap_adds = False
        self._add_stream = None
        self._adds_pending = False
        self._size_dirty = False

    def sync_adds(self):
        """Make the current stream wait for the side-stream tree adds and refresh
        the device copy of the fill level (no-op when nothing is pending).  Call
        outside graph capture, before sample / update_priorities / reading the
        tree or size_t."""
        if self._adds_pending:
            torch.cuda.current_stream(self.device).wait_stream(self._add_stream)
            self._adds_pending = False
        if self._size_dirty:
            self.size_t.fill_(float(self.size))
            self._size_dirty = False

    def _ring_idx(self, B: int) -> torch.Tensor:
        return (self.ptr + torch.arange(B, device=self.device)) % self.capacity

    def _set(self, idx: torch.Tensor, leaf: torch.Tensor, distinct: bool = False):
        """distinct: the caller guarantees no repeated index (ring-buffer adds of
        at most `capacity` entries), so no last-wins resolution is needed."""
        idx = idx.contiguous()
        leaf = leaf.to(torch.float64)
        leaf = (leaf if distinct else _last_wins(idx, leaf)).contiguous()
        L = _lib.load()
        _lib.check(L.trx_per_update(_lib.ptr(self.tree), self.capacity, _lib.ptr(idx), _lib.ptr(leaf), idx.numel(),
                                    _lib.stream_ptr(self.device)), "trx_per_update")

    def _write(self, idx, pairs, B: int):
        """Rows [ptr, ptr + B) of each (buffer, values) pair: one trx_multi_copy
        launch when the slots are contiguous, index_copy otherwise."""
        if self.ptr + B <= self.capacity and self.device.type == "cuda":
            _lib.multi_copy([(dst[self.ptr:self.ptr + B],
                              src.reshape((B,) + dst.shape[1:]).to(dst.dtype).contiguous()) for dst, src in pairs],
                            self.device)
        else:
            idx = self._ring_idx(B) if idx is None else idx
            for dst, src in pairs:
                dst.index_copy_(0, idx, src.reshape((B,) + dst.shape[1:]).to(dst.dtype))

    def stage_prev(self, node_x, edge_x, mask, goal, prev_tstt) -> bool:
        """Write the pre-step fields of the next B transitions into their ring
        slots now -- before env.step overwrites the observation buffers, so no
        clones are needed.  add_staged() completes them; False (nothing
        written) when the slots would wrap: use add_batch then."""
        B = node_x.shape[0]
        if self.ptr + B > self.capacity or self.device.type != "cuda":
            return False
        self._write(None, ((self.node_x, node_x), (self.edge_x, edge_x), (self.mask, mask), (self.goal, goal),
                           (self.prev_tstt, prev_tstt)), B)
        self._staged = B
        return True

    def add_staged(self, action, reward, next_node_x, next_edge_x, next_mask, done, next_tstt, init_tstt):
        B = action.shape[0]
        assert getattr(self, "_staged", None) == B, "stage_prev() first"
        self._staged = None
        idx = None   # staged slots are contiguous: no index tensor needed (see _ring_idx)
        self._write(idx, ((self.action, action), (self.reward, reward), (self.next_node_x, next_node_x),
                          (self.next_edge_x, next_edge_x), (self.next_mask, next_mask), (self.done, done),
                          (self.next_tstt, next_tstt), (self.init_tstt, init_tstt)), B)
        self._priorities_for_new(idx, B)

    def _priorities_for_new(self, idx, B: int):
        # k sequential reference adds: priority_k = max_p + (k+1)*eps (train.py:50-58)
        if self.tree_dtype == "float32":
            L, lo, left = _lib.load(), self.ptr, B
            side = self.overlap_adds and self.device.type == "cuda" and not torch.cuda.is_current_stream_capturing()
            if side:
                if self._add_stream is None:
                    self._add_stream = torch.cuda.Stream(self.device)
                self._add_stream.wait_stream(torch.cuda.current_stream(self.device))   # after every earlier write
                self._adds_pending = True
            with torch.cuda.stream(self._add_stream) if side else contextlib.nullcontext():
                while left > 0:          # ring order: [ptr, capacity) then from 0 (each piece one launch)
                    n = min(left, self.capacity - lo)
                    _lib.check(L.trx_per32_add_range(_lib.ptr(self.tree), self.capacity, lo, n,
                                                     _lib.ptr(self.max_priority), float(self.eps), float(self.alpha),
                                                     _lib.stream_ptr(self.device)), "trx_per32_add_range")
                    lo, left = (lo + n) % self.capacity, left - n
        elif self.ptr + B <= self.capacity and self.device.type == "cuda":
            L = _lib.load()     # one launch: leaves, ancestors and max_priority (updated in place)
            _lib.check(L.trx_per_add_range(_lib.ptr(self.tree), self.capacity, self.ptr, B, _lib.ptr(self.max_priority),
                                           float(self.eps), float(self.alpha), _lib.stream_ptr(self.device)),
                       "trx_per_add_range")
        else:
            idx = self._ring_idx(B) if idx is None else idx
            pr = self.max_priority + self.eps * torch.arange(1, B + 1, device=self.device, dtype=torch.float64)
            self.max_priority.copy_(pr[-1])   # in place: graph-captured updates read this tensor
            self._set(idx, pr ** self.alpha, distinct=B <= self.capacity)
        self.ptr = (self.ptr + B) % self.capacity
        self.size = min(self.size + B, self.capacity)
        if self.overlap_adds:
            self._size_dirty = True   # refreshed by sync_adds(), before any sample
        else:
            self.size_t.fill_(float(self.size))

    @property
    def total(self) -> torch.Tensor:
        """The sum tree's root; joins pending side-stream adds first (outside a
        capture).  Direct reads of `tree` / `max_priority` / `size_t` need
        sync_adds() the same way when overlap_adds is on."""
        if not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
            self.sync_adds()
        return self.tree[1]

    def add_batch(self, node_x, edge_x, mask, action, reward, next_node_x, next_edge_x, next_mask, done, goal,
                  prev_tstt, next_tstt, init_tstt):
        B = action.shape[0]
        idx = (self.ptr + torch.arange(B, device=self.device)) % self.capacity
        pairs = ((self.node_x, node_x), (self.edge_x, edge_x), (self.mask, mask), (self.next_node_x, next_node_x),
                 (self.next_edge_x, next_edge_x), (self.next_mask, next_mask), (self.goal, goal),
                 (self.action, action), (self.reward, reward), (self.done, done), (self.prev_tstt, prev_tstt),
                 (self.next_tstt, next_tstt), (self.init_tstt, init_tstt))
        self._write(idx, pairs, B)
        self._priorities_for_new(idx, B)

    def sample(self, batch_size: int, generator: Optional[torch.Generator] = None,
               u: Optional[torch.Tensor] = None) -> Sample:
        """`u` (float64 [batch_size] in [0,1)) replaces the internal draw; the
        HIP-graph trainer fills it outside the captured region."""
        if self.size == 0:
            raise ValueError("Cannot sample from an empty replay buffer.")
        if not torch.cuda.is_available() or not torch.cuda.is_current_stream_capturing():
            self.sync_adds()
        if u is None:
            u = torch.rand(batch_size, dtype=torch.float64, device=self.device, generator=generator)
        idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        pri = torch.empty(batch_size, dtype=self.tree.dtype, device=self.device)
        L = _lib.load()
        if self.tree_dtype == "float32":
            # train.py:80-82 in float32: probs = pri / total, (size * probs) ** -beta, / max,
            # in the descent's launch (one workgroup; size_t read on the device)
            w = torch.empty(batch_size, dtype=torch.float32, device=self.device)
            _lib.check(L.trx_per32_sample_weighted(_lib.ptr(self.tree), self.capacity, _lib.ptr(u.contiguous()),
                                                   batch_size, _lib.ptr(self.size_t), float(self.beta), _lib.ptr(idx),
                                                   _lib.ptr(pri), _lib.ptr(w), _lib.stream_ptr(self.device)),
                       "trx_per32_sample_weighted")
        else:
            _lib.check(L.trx_per_sample(_lib.ptr(self.tree), self.capacity, _lib.ptr(u), batch_size, _lib.ptr(idx),
                                        _lib.ptr(pri), _lib.stream_ptr(self.device)), "trx_per_sample")
            probs = pri / self.total
            w = (self.size_t * probs) ** (-self.beta)
            w = w / torch.clamp(w.max(), min=1e-300)
        fields = (self.node_x, self.edge_x, self.mask, self.action, self.reward, self.next_node_x, self.next_edge_x,
                  self.next_mask, self.done, self.goal, self.prev_tstt, self.next_tstt, self.init_tstt)
        if self.device.type == "cuda":   # every field's rows in one trx_multi_gather launch
            rows = [torch.empty((batch_size,) + f.shape[1:], dtype=f.dtype, device=self.device) for f in fields]
            _lib.multi_gather(list(zip(rows, fields)), idx, self.device)
        else:
            rows = [f[idx] for f in fields]
        return Sample(idx, w.float(), *rows, pri)

    def update_priorities(self, idx: torch.Tensor, td_errors: torch.Tensor):
        if not torch.cuda.is_available() or not torch.cuda.is_current_stream_capturing():
            self.sync_adds()
        if self.tree_dtype == "float32":
            err = td_errors.detach().to(torch.float64).contiguous()
            idx = idx.contiguous()
            L = _lib.load()
            _lib.check(L.trx_per32_update(_lib.ptr(self.tree), self.capacity, _lib.ptr(idx), _lib.ptr(err), idx.numel(),
                                          _lib.ptr(self.max_priority), float(self.eps), float(self.alpha),
                                          _lib.stream_ptr(self.device)), "trx_per32_update")
            return
        pr = td_errors.detach().to(torch.float64).abs() + self.eps
        self.max_priority.copy_(torch.maximum(self.max_priority, pr.max()))
        self._set(idx, pr ** self.alpha)


def reward_with_goal(mode, prev, curr, init, complete, alpha=1.0, beta=10.0, gamma=0.1, clip=0.0):
    """Vectorised RepairEnv.compute_reward_with_goal (repair_env.py:244-291), float64."""
    bonus = torch.where(complete, torch.full_like(prev, beta), torch.zeros_like(prev))
    if mode in ("minimize_tstt", "rel_improve"):
        bb = torch.clamp(init, min=1.0)
        if mode == "minimize_tstt":
            r = -alpha * (curr / bb)
        else:
            r = alpha * (((prev - curr) / bb) * 100.0) - 1.0 * (curr / bb)
        r = r + bonus
    else:
        if mode == "neg_tstt":
            delta = -curr
        elif mode == "log_delta":
            delta = torch.log10(torch.clamp(prev, min=1.0)) - torch.log10(torch.clamp(curr, min=1.0))
        else:
            delta = prev - curr
        r = alpha * delta + bonus - gamma
    if clip and clip > 0:
        r = torch.clamp(r, -clip, clip)
    return r


def her_relabel(s: Sample, her_ratio: float, reward_mode: str, reward_scale: float, alpha: float, beta: float,
                gamma: float, clip: float, generator: Optional[torch.Generator] = None, goal_column: int = -1,
                u: Optional[torch.Tensor] = None):
    """train.py:805-823 on a sampled batch (in place).  goal_column=-1
    reproduces apply_goal (train.py:127); 4 would write the real goal column.
    `u` (float32 [bs]) replaces the internal draw (graph capture)."""
    if her_ratio <= 0:
        return s
    bs = s.action.shape[0]
    if u is None:
        u = torch.rand(bs, device=s.action.device, generator=generator)
    pick = u < her_ratio
    goal = 1.0 - s.next_mask
    complete = ((goal * s.next_mask).sum(dim=1) == 0)
    r = reward_with_goal(reward_mode, s.prev_tstt, s.next_tstt, s.init_tstt, complete, alpha, beta, gamma, clip)
    r = (r * reward_scale).float()
    s.reward = torch.where(pick, r, s.reward)
    s.done = torch.where(pick, complete.float(), s.done)
    s.goal = torch.where(pick[:, None], goal, s.goal)
    s.edge_x = s.edge_x.clone()
    s.next_edge_x = s.next_edge_x.clone()
    # masked column write without boolean indexing (no host sync)
    s.edge_x[:, :, goal_column] = torch.where(pick[:, None], goal, s.edge_x[:, :, goal_column])
    s.next_edge_x[:, :, goal_column] = torch.where(pick[:, None], goal, s.next_edge_x[:, :, goal_column])
    return s

"""VecRepairEnv: B Sioux-Falls-sized repair envs stepping in lockstep on one
MI355X.  The batched form of RepairEnv (src/env/repair_env.py:22-819).

State lives in device tensors (structure of arrays, [B, E] row-major, float32
per link, float64 per env), every hot operation is one gfx950 kernel launch
through libtrafficrl.so:

  reset   -> trx_reset    (repair_env.py:167-205, damage draw on the host RNG)
  step    -> trx_step     (repair_env.py:207-237, assignment fused in)
  observe -> trx_observe  (repair_env.py:751-819)
  assign  -> trx_assign   (repair_env.py:299-345, what-if batches)

Nothing here falls back to the CPU: without libtrafficrl.so or a HIP device
the constructor raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from .. import _lib
from ..graph import DamageSampler, TrafficGraph, damage_sample_batch, pcg_states, set_generator_state


def resolve_sp_rule(sp_backend: Optional[str], num_nodes: int, force_gpu_sp: bool = False) -> int:
    """RepairEnv(sp_backend=...) -> the all-or-nothing shortest-path rule
    (repair_env.py:111-161 backend resolution, 421-573 dispatch).

    "torch": the reference's GPU backend _all_or_nothing_torch (float32
      Floyd-Warshall, strict <, next_hop walk) -- what configs/sioux_falls.yaml
      (sp_backend: torch, force_gpu_sp: true) and run_greedy.py select on a GPU;
      here it runs as TRX_SP_TORCH inside the fused env kernel (N <= 32).
    "scipy", "auto" and anything else: scipy's dijkstra semantics (float64
      labels, heap order on ties) -- what "auto" resolves to where cupy and
      cugraph are absent, as in the reference's own CPU runs.
    "cupy" / "cugraph": their Dijkstra variants are not importable here, so
      their tie order cannot be pinned; they get the scipy rule (a Dijkstra).
    Every rule runs on the GPU, so force_gpu_sp never falls back; a rule this
    build cannot run raises RuntimeError (never a silent substitution)."""
    b = (sp_backend or "auto").lower()
    if b == "torch":
        if num_nodes > 32:
            raise RuntimeError(f"sp_backend='torch' (all-pairs Floyd-Warshall rule) supports <= 32 nodes on this "
                               f"build (got {num_nodes}); use sp_backend='scipy'")
        return _lib.SP_TORCH
    return _lib.SP_SCIPY


@dataclass
class VecObs:
    """A step's observation as VIEWS of the env's persistent buffers: valid
    until the next step / reset / observe overwrites them (clone to keep)."""
    node_x: torch.Tensor     # [B, N, 4]
    edge_x: torch.Tensor     # [B, E, 6]
    action_mask: torch.Tensor  # [B, E]
    tstt: torch.Tensor       # [B] float64, the env's TSTT buffer (valid until the next step, like the rest)

    @property
    def log_tstt(self) -> torch.Tensor:   # [B] float64, evaluated on access (no per-step launch)
        return torch.log10(torch.clamp(self.tstt, min=1.0))


class VecRepairEnv:
    def __init__(
        self,
        graph_data,
        num_envs: int,
        device="cuda",
        damaged_ratio: float = 0.3,
        bpr_alpha: float = 0.15,
        bpr_beta: float = 4.0,
        assignment_iters: int = 20,
        assignment_method: str = "msa",
        reward_mode: str = "log_delta",
        reward_alpha: float = 1.0,
        reward_beta: float = 10.0,
        reward_gamma: float = 0.1,
        reward_clip: float = 0.0,
        capacity_damage: float = 1e-3,
        unassigned_penalty: float = 2e7,
        gp_step: float = 1.0,
        gp_keep_paths: int = 3,
        fixed_damage: bool = False,
        fixed_damage_seed: Optional[int] = None,
        seed: int = 0,
        seeds: Optional[Sequence[int]] = None,
        graph: Optional[TrafficGraph] = None,
        reset: bool = True,
        sp_backend: str = "auto",
        force_gpu_sp: bool = False,
    ):
        if assignment_method.lower() not in _lib.METHODS:
            raise ValueError(f"assignment_method {assignment_method!r} not supported (msa, fw, cfw, gp)")
        if int(assignment_iters) <= 0:
            raise ValueError("assignment_iters must be > 0 to update TSTT.")
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("VecRepairEnv runs on a HIP device only (device='cuda[:i]')")
        if not torch.cuda.is_available():
            raise RuntimeError("VecRepairEnv needs a HIP device (MI355X); there is no CPU fallback")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        torch.cuda.set_device(self.device)
        self.graph = graph if graph is not None else TrafficGraph(graph_data, self.device)
        self.graph_data = self.graph.graph_data
        self.num_envs = B = int(num_envs)
        self.num_nodes = N = self.graph.num_nodes
        self.num_edges = E = self.graph.num_edges
        self.damaged_ratio = damaged_ratio
        self.assignment_method = assignment_method.lower()
        self.assignment_iters = int(assignment_iters)
        self.reward_mode = reward_mode
        self.params = _lib.TrxParams(
            method=_lib.METHODS[self.assignment_method], iters=self.assignment_iters, bpr_alpha=bpr_alpha,
            bpr_beta=bpr_beta, capacity_damage=capacity_damage, unassigned_penalty=unassigned_penalty,
            reward_mode=_lib.REWARD_MODES[reward_mode], reward_alpha=reward_alpha, reward_beta=reward_beta,
            reward_gamma=reward_gamma, reward_clip=reward_clip, gp_step=float(gp_step),
            gp_keep_paths=int(gp_keep_paths), sp_rule=resolve_sp_rule(sp_backend, N, force_gpu_sp))
        self.sp_backend = (sp_backend or "auto").lower()
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        f64 = dict(dtype=torch.float64, device=dev)
        self.flow = torch.zeros(B, E, **f32)
        self.capacity = torch.zeros(B, E, **f32)
        self.damaged = torch.zeros(B, E, **f32)
        self.goal = torch.zeros(B, E, **f32)
        self.t = torch.zeros(B, E, **f32)
        self.tstt = torch.zeros(B, **f64)
        self.initial_tstt = torch.zeros(B, **f64)
        self.unassigned = torch.zeros(B, **f64)
        self.reward = torch.zeros(B, **f64)
        self.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.valid = torch.zeros(B, dtype=torch.uint8, device=dev)
        self._obs_bufs = None
        self.workspace = torch.empty(self.graph.workspace_bytes(B), dtype=torch.uint8, device=dev)
        # GP: per-env path sets (RepairEnv.od_paths / od_path_flows) live on the device
        self.gp_state = None
        if self.assignment_method == "gp":
            self.gp_state = torch.zeros(self.graph.gp_state_bytes(B, gp_keep_paths), dtype=torch.uint8, device=dev)
        self._state = _lib.TrxState(
            flow=self.flow.data_ptr(), capacity=self.capacity.data_ptr(), damaged=self.damaged.data_ptr(),
            goal=self.goal.data_ptr(), t=self.t.data_ptr(), tstt=self.tstt.data_ptr(),
            initial_tstt=self.initial_tstt.data_ptr(), unassigned=self.unassigned.data_ptr(),
            gp=0 if self.gp_state is None else self.gp_state.data_ptr())
        self.edge_index = torch.as_tensor(self.graph.edge_index, device=dev)
        self._seeds = list(seeds) if seeds is not None else [seed + i for i in range(B)]
        self._fixed = (fixed_damage, fixed_damage_seed)
        self._samplers = None
        self._rng_states = None   # PCG64 records of default_rng(seed_b), the non-fixed reset path
        self._prefetch = None     # DamagePrefetch (enable_damage_prefetch)
        if reset:
            self.reset()

    def enable_damage_prefetch(self, on: bool = True):
        """Draw every env's NEXT damage mask on a host thread while the device
        runs the current episode (native trx_damage_sample, GIL released),
        into pinned memory, so a whole-batch reset costs an asynchronous copy
        instead of a blocking host draw.  The masks and the generator states
        are exactly those of drawing at reset time: a prefetched draw is
        committed only when all envs reset together; any other reset discards
        it and draws synchronously from the envs' true states."""
        if self._prefetch is not None:
            self._prefetch.close()
            self._prefetch = None
        if on and not self._fixed[0] and self._samplers is None and self.num_edges <= 10000:
            if self._rng_states is None:
                self._rng_states = pcg_states(self._seeds)
            self._prefetch = DamagePrefetch(self)
        return self._prefetch is not None

    @property
    def samplers(self):
        """Per-env DamageSampler objects.  Built lazily; when native batch draws
        have already advanced the envs' generators (_rng_states), the samplers
        continue from those states and become the only RNG record, so no reset
        ever repeats a damage set already drawn."""
        if self._samplers is None:
            fd, fds = self._fixed
            self._samplers = [DamageSampler(self.graph, int(s), fd, fds) for s in self._seeds]
            if self._rng_states is not None:
                for smp, rec in zip(self._samplers, self._rng_states):
                    set_generator_state(smp.rng, rec)
                self._rng_states = None
        return self._samplers

    @property
    def kernel_name(self) -> str:
        """The env kernel trx_step / trx_reset / trx_assign launch for this
        graph and parameters (trx_env_kernel_name)."""
        return _lib.load().trx_env_kernel_name(self.graph.handle, ctypes.byref(self.params)).decode()

    def _obs_buffers(self):
        if self._obs_bufs is None:
            B, N, E = self.num_envs, self.num_nodes, self.num_edges
            f32 = dict(dtype=torch.float32, device=self.device)
            self._obs_bufs = (torch.zeros(B, N, 4, **f32), torch.zeros(B, E, 6, **f32), torch.zeros(B, E, **f32))
        return self._obs_bufs

    # ------------------------------------------------------------ kernels
    def _stream(self):
        return _lib.stream_ptr(self.device)

    def assign(self, env_mask: Optional[torch.Tensor] = None):
        """compute_flow_assignment for the envs in env_mask (uint8 [B]); warm
        start from self.flow with the current capacities/damage."""
        L = _lib.load()
        m = None if env_mask is None else env_mask.to(device=self.device, dtype=torch.uint8).contiguous()
        _lib.check(L.trx_assign(self.graph.handle, ctypes.byref(self.params), self.num_envs, ctypes.byref(self._state),
                                _lib.ptr(m), _lib.ptr(self.workspace), self._stream()), "trx_assign")

    def reset(self, env_ids=None, damaged: Optional[torch.Tensor] = None, damaged_ratio: Optional[float] = None,
              observe: bool = True):
        """Reset all envs (or env_ids).  Damage masks come from each env's
        host RNG unless `damaged` [B,E] (or [len(env_ids),E]) is given."""
        ratio = self.damaged_ratio if damaged_ratio is None else damaged_ratio
        B = self.num_envs
        ids = list(range(B)) if env_ids is None else [int(i) for i in (env_ids.tolist() if torch.is_tensor(env_ids)
                                                                       else env_ids)]
        if damaged is None:
            damaged = self._take_prefetched(ids, ratio)
            if damaged is None:
                damaged = self.draw_damage(ids, ratio)
        damaged = damaged.to(device=self.device, dtype=torch.float32)
        env_mask = None
        if env_ids is None:
            self.damaged.copy_(damaged)
        else:
            idx = torch.as_tensor(ids, device=self.device, dtype=torch.long)
            self.damaged.index_copy_(0, idx, damaged)
            env_mask = torch.zeros(B, dtype=torch.uint8, device=self.device)
            env_mask[idx] = 1
        L = _lib.load()
        _lib.check(L.trx_reset(self.graph.handle, ctypes.byref(self.params), B, ctypes.byref(self._state),
                               _lib.ptr(env_mask), _lib.ptr(self.workspace), self._stream()), "trx_reset")
        return self.observe() if observe else None

    def draw_damage(self, ids=None, damaged_ratio: Optional[float] = None) -> torch.Tensor:
        """The next damage masks (float32 [len(ids), E], host) of envs `ids`
        (default all) from their own RNG streams, as RepairEnv.reset draws them."""
        ratio = self.damaged_ratio if damaged_ratio is None else damaged_ratio
        ids = list(range(self.num_envs)) if ids is None else ids
        got = self._take_prefetched(ids, ratio)
        if got is not None:
            return got.cpu()
        # numpy's choice for E > 10000 links is not the Floyd draw the native sampler
        # restates (trx_damage_sample's limit): those graphs take the numpy samplers,
        # which continue the same per-env streams
        if self._fixed[0] or self._samplers is not None or self.num_edges > 10000:
            masks = np.stack([self.samplers[i].sample(ratio) for i in ids])
        else:   # every env's own default_rng(seed) stream, one native call for the batch
            if self._rng_states is None:
                self._rng_states = pcg_states(self._seeds)
            sel = np.asarray(ids, np.int64)
            st = np.ascontiguousarray(self._rng_states[sel])
            masks = damage_sample_batch(self.num_nodes, self.graph.src, self.graph.dst, st, ratio)
            self._rng_states[sel] = st
            if self._prefetch is not None:
                self._prefetch.restart(ratio)   # from the advanced states
        return torch.from_numpy(masks)

    def _take_prefetched(self, ids, ratio) -> Optional[torch.Tensor]:
        """The prefetched masks already on the device (an asynchronous copy
        from pinned memory) when every env resets at once; else None and the
        prefetch is dropped (the caller draws from the envs' true states)."""
        pf = self._prefetch
        if pf is None:
            return None
        if self._fixed[0] or self._samplers is not None:   # the RNG record moved to the samplers
            self.enable_damage_prefetch(False)
            return None
        return pf.take(ids, ratio)

    def close(self):
        if self._prefetch is not None:
            self._prefetch.close()
            self._prefetch = None

    def reset_where(self, env_mask: torch.Tensor, damaged: torch.Tensor, observe: bool = False):
        """Reset the envs where env_mask (bool/uint8 [B]) is set, with damage
        rows taken from `damaged` [B,E]; fully on device (no host sync)."""
        m = env_mask.to(device=self.device, dtype=torch.bool)
        self.damaged.copy_(torch.where(m[:, None], damaged.to(self.damaged.dtype), self.damaged))
        L = _lib.load()
        mu8 = m.to(torch.uint8).contiguous()
        _lib.check(L.trx_reset(self.graph.handle, ctypes.byref(self.params), self.num_envs, ctypes.byref(self._state),
                               _lib.ptr(mu8), _lib.ptr(self.workspace), self._stream()), "trx_reset")
        return self.observe() if observe else None

    def step(self, actions: torch.Tensor, observe: bool = True, check: bool = True):
        """Batched RepairEnv.step.  Returns (obs, reward[B] f64, done[B] bool, info).

        The returned tensors ALIAS the env's own buffers, overwritten by the next
        step: reward, done / info["valid"] (bool views of the byte buffers),
        info["tstt"] and the observation buffers (VecObs.log_tstt is computed
        from the live tstt on access).  Clone what must outlive the step."""
        a = actions.to(device=self.device, dtype=torch.int32).contiguous()
        if a.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {a.numel()}")
        if check:
            lo, hi = int(a.min()), int(a.max())
            if lo < 0 or hi >= self.num_edges:
                bad = lo if lo < 0 else hi
                raise ValueError(f"action_edge_id {bad} out of range (0..{self.num_edges - 1})")
        L = _lib.load()
        _lib.check(L.trx_step(self.graph.handle, ctypes.byref(self.params), self.num_envs, ctypes.byref(self._state),
                              _lib.ptr(a), _lib.ptr(self.reward), _lib.ptr(self.done), _lib.ptr(self.valid),
                              _lib.ptr(self.workspace), self._stream()), "trx_step")
        obs = self.observe() if observe else None
        # done / valid are 0/1 bytes: bool views of the env's buffers (no cast launch; valid
        # until the next step, like reward and the observation buffers)
        return obs, self.reward, self.done.view(torch.bool), {"tstt": self.tstt, "valid": self.valid.view(torch.bool)}

    def observe(self) -> VecObs:
        L = _lib.load()
        node_x, edge_x, mask = self._obs_buffers()
        _lib.check(L.trx_observe(self.graph.handle, self.num_envs, ctypes.byref(self._state), _lib.ptr(node_x),
                                 _lib.ptr(edge_x), _lib.ptr(mask), _lib.ptr(self.workspace), self._stream()),
                   "trx_observe")
        return VecObs(node_x, edge_x, mask, self.tstt)

    # ------------------------------------------------------ GP path sets
    def _gp_rows(self):
        if self.gp_state is None:
            raise ValueError("path sets exist only for assignment_method='gp'")
        P = len(self.graph.od_o)
        lay = _lib.gp_layout(P, int(self.params.gp_keep_paths))
        return self.gp_state.view(self.num_envs, lay["total"]), lay, P

    def gp_paths(self, b: int):
        """Env b's (od_paths, od_path_flows) as the reference's dicts
        (repair_env.py:374-404): 1-based (o, d) keys in insertion order, paths
        as link-id tuples in path order, float64 flows."""
        rows, lay, P = self._gp_rows()
        row = rows[b].cpu().numpy()
        KP = int(self.params.gp_keep_paths) + 1
        nkeys = int(row[lay["nkeys"]:lay["nkeys"] + 4].view(np.int32)[0])
        order = row[lay["ord"]:lay["ord"] + 2 * P].view(np.int16)[:nkeys]
        npath = row[lay["np"]:lay["np"] + P]
        flows = row[lay["flow"]:lay["flow"] + 8 * P * KP].view(np.float64).reshape(P, KP)
        lens = row[lay["len"]:lay["len"] + P * KP].reshape(P, KP)
        edges = row[lay["edges"]:lay["edges"] + P * KP * _lib.GP_MAX_HOPS].reshape(P, KP, _lib.GP_MAX_HOPS)
        key_of = self.graph.od_key_order()
        paths, pflows = {}, {}
        for q in order.tolist():
            key = key_of[q]
            n = int(npath[q])
            paths[key] = [tuple(int(e) for e in edges[q, i, :lens[q, i]]) for i in range(n)]
            pflows[key] = [float(flows[q, i]) for i in range(n)]
        return paths, pflows

    def set_gp_paths(self, b: int, paths: dict, pflows: dict):
        """Load env b's path sets from reference-style dicts (inverse of gp_paths)."""
        rows, lay, P = self._gp_rows()
        KP = int(self.params.gp_keep_paths) + 1
        row = np.zeros(lay["total"], np.uint8)
        q_of = {k: q for q, k in enumerate(self.graph.od_key_order())}
        order = np.zeros(P, np.int16)
        npath = np.zeros(P, np.uint8)
        flows = np.zeros((P, KP), np.float64)
        masks = np.zeros((P, KP, 4), np.uint32)
        lens = np.zeros((P, KP), np.uint8)
        edges = np.zeros((P, KP, _lib.GP_MAX_HOPS), np.uint8)
        for k, key in enumerate(paths):
            q = q_of[key]
            order[k] = q
            npath[q] = len(paths[key])
            for i, (pth, f) in enumerate(zip(paths[key], pflows[key])):
                flows[q, i] = f
                lens[q, i] = len(pth)
                edges[q, i, :len(pth)] = pth
                for e in pth:
                    masks[q, i, e // 32] |= np.uint32(1 << (e % 32))
        row[lay["nkeys"]:lay["nkeys"] + 4] = np.array([len(paths)], np.int32).view(np.uint8)
        row[lay["ord"]:lay["ord"] + 2 * P] = order.view(np.uint8)
        row[lay["np"]:lay["np"] + P] = npath
        row[lay["flow"]:lay["flow"] + 8 * P * KP] = flows.reshape(-1).view(np.uint8)
        row[lay["mask"]:lay["mask"] + 16 * P * KP] = masks.reshape(-1).view(np.uint8)
        row[lay["len"]:lay["len"] + P * KP] = lens.reshape(-1)
        row[lay["edges"]:lay["edges"] + P * KP * _lib.GP_MAX_HOPS] = edges.reshape(-1)
        rows[b].copy_(torch.from_numpy(row))

    def is_goal_complete(self) -> torch.Tensor:
        return (self.goal * self.damaged).sum(dim=1) == 0



class DamagePrefetch:
    """Background draw of every env's next damage mask (VecRepairEnv.
    enable_damage_prefetch): one host thread, two pinned buffers.  The draw
    for the next whole-batch reset runs while the current episode steps; a
    buffer is rewritten only after the device copy that read it completed
    (its HIP event, waited on by the worker thread)."""

    def __init__(self, env: "VecRepairEnv"):
        from concurrent.futures import ThreadPoolExecutor
        self.env = env
        B, E = env.num_envs, env.num_edges
        self.bufs = [torch.empty(B, E, dtype=torch.float32).pin_memory() for _ in range(2)]
        self.copied = [None, None]   # HIP event of the last device copy out of each buffer
        self.which = 0
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="trx-damage")
        self.job = None
        self.restart(env.damaged_ratio)

    def restart(self, ratio):
        """(Re)start the draw of the next masks from the envs' current states.
        Never blocks: a stale draw still running (a partial reset discarded it)
        is left to finish -- the pool's single worker runs draws in submission
        order, so two draws never write one buffer at the same time."""
        env, k = self.env, self.which
        states = np.ascontiguousarray(env._rng_states).copy()
        ev = self.copied[k]
        buf = self.bufs[k].numpy()

        def work():
            if ev is not None:
                ev.synchronize()     # the previous copy out of this buffer has finished
            damage_sample_batch(env.num_nodes, env.graph.src, env.graph.dst, states, ratio, out=buf)
            return states

        self.job = (k, ratio, self.pool.submit(work))

    def take(self, ids, ratio) -> Optional[torch.Tensor]:
        env = self.env
        k, r, fut = self.job
        if r != ratio or len(ids) != env.num_envs or list(ids) != list(range(env.num_envs)):
            # not committed, and not waited for: the caller draws synchronously from the
            # envs' true states and restarts us (the stale draw finishes on its own)
            return None
        states = fut.result()
        env._rng_states[:] = states
        dev = self.bufs[k].to(env.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.copied[k] = ev
        self.which = 1 - k
        self.job = None
        self.restart(ratio)
        return dev

    def close(self):
        if self.job is not None:
            self.job[2].result()
            self.job = None
        self.pool.shutdown(wait=True)

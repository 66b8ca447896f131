"""Baseline repair policies (src/baselines/__init__.py:11-113).

The greedy one-step policy (35-69) runs one warm-started assignment per
damaged candidate; here all candidates are ONE batched trx_assign launch
(candidate rows of a what-if batch) instead of 22 serial assignments.  The
choice rule is the reference's: first candidate (in link order) with the
strictly smallest TSTT.
"""
from __future__ import annotations

from typing import Callable, Dict, List

import numpy as np
import torch

from ..env.repair_env import EnvState, RepairEnv
from ..env.vec_env import VecRepairEnv


def _best_masked(score: np.ndarray, mask: np.ndarray) -> int:
    """Index of the largest score among masked-in links (score * mask, first
    maximum: np.argmax semantics of src/baselines/__init__.py:16-32)."""
    return int(np.argmax(score * mask))


def select_random(state: EnvState) -> int:
    """Uniform draw over the repairable links from numpy's global RNG (11-13)."""
    return int(np.random.choice(np.flatnonzero(state.action_mask > 0)))


def select_max_vc(state: EnvState) -> int:
    """Largest clipped log(1 + v/c) feature (edge feature 2; 16-19)."""
    return _best_masked(state.edge_features[:, 2], state.action_mask)


def select_max_flow(state: EnvState) -> int:
    """Largest v/c feature x normalised capacity feature (a flow proxy; 22-25)."""
    ef = state.edge_features
    return _best_masked(ef[:, 2] * ef[:, 1], state.action_mask)


def select_max_betweenness(state: EnvState, node_betweenness: np.ndarray, edge_index: np.ndarray) -> int:
    """Largest mean betweenness of the link's two end nodes (28-32)."""
    bw = 0.5 * (node_betweenness[edge_index[0]] + node_betweenness[edge_index[1]])
    return _best_masked(bw, state.action_mask)


class WhatIfBatch:
    """Reusable device batch of what-if rows sharing one graph."""

    def __init__(self, graph, params, device, rows: int):
        self.rows = 0
        self.graph, self.params, self.device = graph, params, device
        self._vec = None
        self.ensure(rows)

    def ensure(self, rows: int):
        if self._vec is not None and rows <= self.rows:
            return
        self.rows = max(rows, 1)
        # shares the graph handle and params; only state tensors are allocated
        v = VecRepairEnv(self.graph.graph_data, self.rows, device=self.device, graph=self.graph, reset=False,
                         assignment_iters=self.params.iters,
                         assignment_method={0: "msa", 1: "fw", 2: "cfw", 3: "gp"}[self.params.method],
                         gp_step=self.params.gp_step, gp_keep_paths=max(1, self.params.gp_keep_paths))
        v.params = self.params
        self._vec = v

    def tstt(self, cap: torch.Tensor, dmg: torch.Tensor, flow: torch.Tensor, gp_row=None) -> torch.Tensor:
        """Run warm-started assignments for rows [R,E]; return tstt[R] (f64).
        GP: every row starts from the path sets `gp_row` (one env's state row),
        like the reference's deepcopy/restore of od_paths (baselines 46-65)."""
        R = cap.shape[0]
        self.ensure(R)
        v = self._vec
        if v.gp_state is not None:
            v.gp_state.view(v.num_envs, -1)[:R].copy_(gp_row[None].expand(R, -1))
        v.capacity[:R].copy_(cap)
        v.damaged[:R].copy_(dmg)
        v.flow[:R].copy_(flow)
        mask = torch.zeros(v.num_envs, dtype=torch.uint8, device=v.device)
        mask[:R] = 1
        v.assign(mask)
        return v.tstt[:R]


_batches: Dict[int, WhatIfBatch] = {}


def select_greedy_one_step(env: RepairEnv, state: EnvState) -> int:
    candidates = np.where(state.action_mask > 0)[0]
    if candidates.size == 0:
        return int(np.argmax(state.action_mask))
    candidates = candidates[env.is_damaged[candidates] != 0]
    if candidates.size == 0:
        return int(np.where(state.action_mask > 0)[0][0])
    dev = env.device
    D = candidates.size
    cap = torch.from_numpy(np.repeat(env.capacities[None], D, 0)).to(dev)
    dmg = torch.from_numpy(np.repeat(env.is_damaged[None], D, 0)).to(dev)
    flow = torch.from_numpy(np.repeat(env.flow[None], D, 0)).to(dev)
    idx = torch.arange(D, device=dev)
    cand = torch.from_numpy(candidates).to(dev)
    cap[idx, cand] = torch.from_numpy(env.initial_capacities[candidates]).to(dev)
    dmg[idx, cand] = 0.0
    key = id(env)
    wb = _batches.get(key)
    if wb is None or wb.graph is not env.graph:
        wb = _batches[key] = WhatIfBatch(env.graph, env._vec.params, dev, max(D, 32))
    gp_row = None if env._vec.gp_state is None else env._vec.gp_state.view(1, -1)[0]
    if env._gp_dirty:
        env._push()
    ts = wb.tstt(cap, dmg, flow, gp_row).cpu().numpy()
    return int(candidates[int(np.argmin(ts))])  # first strict minimum, like `if env.tstt < best_tstt`


def greedy_actions(venv: VecRepairEnv, batch: WhatIfBatch | None = None) -> torch.Tensor:
    """Greedy one-step action for every env of a VecRepairEnv at once: B x E
    what-if rows (non-damaged links masked out) in one trx_assign launch."""
    B, E = venv.num_envs, venv.num_edges
    dev = venv.device
    rows = B * E
    if batch is None:
        batch = WhatIfBatch(venv.graph, venv.params, dev, rows)
    eye = torch.eye(E, device=dev, dtype=torch.bool)
    cap = venv.capacity[:, None, :].expand(B, E, E).clone()
    dmg = venv.damaged[:, None, :].expand(B, E, E).clone()
    cap0 = torch.as_tensor(venv.graph.cap0, device=dev)
    cap = torch.where(eye[None], cap0[None, None, :].expand(B, E, E), cap)
    dmg = torch.where(eye[None], torch.zeros((), device=dev), dmg)
    flow = venv.flow[:, None, :].expand(B, E, E).reshape(rows, E)
    cand = venv.damaged > 0  # [B,E]
    batch.ensure(rows)
    v = batch._vec
    v.capacity[:rows].copy_(cap.reshape(rows, E))
    v.damaged[:rows].copy_(dmg.reshape(rows, E))
    v.flow[:rows].copy_(flow)
    mask = torch.zeros(v.num_envs, dtype=torch.uint8, device=dev)
    mask[:rows] = cand.reshape(-1).to(torch.uint8)
    v.assign(mask)
    ts = torch.where(cand, v.tstt[:rows].view(B, E), torch.full((), float("inf"), dtype=torch.float64, device=dev))
    return torch.argmin(ts, dim=1).to(torch.int32)  # first minimum in link order


def run_episode(env: RepairEnv, policy: Callable[[EnvState], int], reward_scale: float = 1.0,
                max_steps: int = 0) -> Dict:
    """One episode of `policy` from env.reset() (src/baselines/__init__.py:72-101):
    the TSTT after every step, the scaled reward sum, and the curve's last /
    mean / trapezoid area (an empty episode reports the env's TSTT)."""
    state = env.reset()
    curve: List[float] = []
    reward_sum = 0.0
    done = False
    while not done and not (max_steps > 0 and len(curve) >= max_steps):
        state, reward, done, info = env.step(policy(state))
        reward_sum += reward * reward_scale
        curve.append(info.get("tstt", env.tstt))
    if curve:
        last, mean, auc = float(curve[-1]), float(np.mean(curve)), float(np.trapezoid(curve))
    else:
        last = mean = auc = env.tstt
    return {"tstt_curve": curve, "reward": reward_sum, "tstt_last": last, "tstt_mean": mean, "tstt_auc": auc,
            "auc": auc}


def get_baseline_policies(env: RepairEnv) -> Dict[str, Callable[[EnvState], int]]:
    """The reference's policy table (104-113); betweenness and links are read once."""
    bw, ei = env.betweenness_vec, env.edge_index
    table: Dict[str, Callable[[EnvState], int]] = dict(random=select_random, max_vc=select_max_vc,
                                                       max_flow=select_max_flow)
    table["max_betweenness"] = lambda st: select_max_betweenness(st, bw, ei)
    table["greedy"] = lambda st: select_greedy_one_step(env, st)
    return table

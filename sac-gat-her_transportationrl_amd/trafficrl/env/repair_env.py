"""Drop-in RepairEnv: the reference's single-env API (src/env/repair_env.py:22-819)
with every assignment, reward and observation computed by the gfx950 kernels.

Callers written against the reference (src/train.py:251-277, 916-927;
src/baselines/__init__.py:35-101) keep working: same constructor keywords,
same EnvState, same numpy attributes (is_damaged, capacities, flow,
goal_mask, tstt, initial_tstt, unassigned_demand, ...), and callers may still
mutate those attributes and call compute_flow_assignment() (the greedy
baseline does).  The numpy attributes are the source of truth between calls;
each device call uploads the 4 x E link arrays and downloads the result.

Backend keywords: everything runs on gfx950 and never falls back to the
CPU.  sp_backend selects the shortest-path RULE of the all-or-nothing step,
as in the reference: "torch" = _all_or_nothing_torch (float32 Floyd-Warshall,
strict <, next_hop walk, repair_env.py:520-573; configs/sioux_falls.yaml and
run_greedy.py), anything else = scipy dijkstra semantics (481-503; what "auto"
resolves to without cupy/cugraph) -- see vec_env.resolve_sp_rule.  use_torch
(torch BPR) and use_cugraph change no arithmetic here and are accepted as is.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Tuple

import numpy as np
import torch

from .. import _lib
from ..graph import DamageSampler, TrafficGraph
from .vec_env import VecRepairEnv


@dataclass
class EnvState:
    node_features: np.ndarray
    edge_features: np.ndarray
    edge_index: np.ndarray
    action_mask: np.ndarray
    log_tstt: float
    goal_mask: np.ndarray


_banner_done = False


class RepairEnv:
    def __init__(
        self,
        graph_data,
        damaged_ratio: float = 0.3,
        bpr_alpha: float = 0.15,
        bpr_beta: float = 4.0,
        assignment_iters: int = 20,
        assignment_method: str = "msa",
        use_cugraph: bool = False,
        use_torch: bool = False,
        device: str = "cuda",
        sp_backend: str = "auto",
        force_gpu_sp: bool = False,
        reward_mode: str = "log_delta",
        reward_alpha: float = 1.0,
        reward_beta: float = 10.0,
        reward_gamma: float = 0.1,
        reward_clip: float = 0.0,
        capacity_damage: float = 1e-3,
        unassigned_penalty: float = 2e7,
        gp_step: float = 1.0,
        gp_keep_paths: int = 3,
        debug_reward: bool = False,
        debug_reward_every: int = 0,
        fixed_damage: bool = False,
        fixed_damage_seed: int | None = None,
        seed: int = 0,
    ):
        global _banner_done
        self.graph_data = graph_data
        self.bpr_alpha = bpr_alpha
        self.bpr_beta = bpr_beta
        self.assignment_iters = assignment_iters
        self.assignment_method = assignment_method.lower()
        self.sp_backend = (sp_backend or "auto").lower()
        self.force_gpu_sp = bool(force_gpu_sp)
        self.use_cugraph = use_cugraph
        self.use_torch = use_torch
        dev = torch.device(device) if str(device).startswith("cuda") else torch.device("cuda")
        if not torch.cuda.is_available():
            raise RuntimeError("RepairEnv needs a HIP device (MI355X): there is no CPU backend")
        self.device = dev
        self.reward_mode = reward_mode
        self.reward_alpha = reward_alpha
        self.reward_beta = reward_beta
        self.reward_gamma = reward_gamma
        self.reward_clip = reward_clip
        self.capacity_damage = capacity_damage
        self.unassigned_penalty = unassigned_penalty
        self.gp_step = float(gp_step)
        self.gp_keep_paths = int(gp_keep_paths)
        self.debug_reward = debug_reward
        self.debug_reward_every = debug_reward_every
        self._debug_step = 0
        self.fixed_damage = bool(fixed_damage)
        self.fixed_damage_seed = fixed_damage_seed

        self._vec = VecRepairEnv(
            graph_data, 1, device=dev, damaged_ratio=damaged_ratio, bpr_alpha=bpr_alpha, bpr_beta=bpr_beta,
            assignment_iters=assignment_iters, assignment_method=self.assignment_method, reward_mode=reward_mode,
            reward_alpha=reward_alpha, reward_beta=reward_beta, reward_gamma=reward_gamma, reward_clip=reward_clip,
            capacity_damage=capacity_damage, unassigned_penalty=unassigned_penalty, gp_step=gp_step,
            gp_keep_paths=gp_keep_paths, seeds=[seed], reset=False, sp_backend=self.sp_backend,
            force_gpu_sp=self.force_gpu_sp)
        self._gp_cache = None    # GP path sets decoded from the device (od_paths, od_path_flows)
        self._gp_dirty = False   # set when a caller assigns od_paths / od_path_flows
        self._od_host = [{}, {}]
        self.graph: TrafficGraph = self._vec.graph
        self._sampler: DamageSampler = self._vec.samplers[0]
        self.rng = self._sampler.rng
        if fixed_damage:
            self._sampler.fixed_damage = True
            self._sampler._fixed_rng = (np.random.default_rng(fixed_damage_seed)
                                        if fixed_damage_seed is not None else None)

        g = self.graph
        self.num_nodes = g.num_nodes
        self.edges = graph_data.edges
        self.num_edges = g.num_edges
        self.edge_index = g.edge_index.copy()
        self.initial_capacities = g.cap0.copy()
        self.capacities = self.initial_capacities.copy()
        self.t0 = g.t0.copy()
        self.max_capacity = float(np.max(self.initial_capacities)) if self.num_edges > 0 else 1.0
        self.max_t0 = float(np.max(self.t0)) if self.num_edges > 0 else 1.0
        self.edge_id_map = dict(g.edge_id_map)
        self.initial_tstt = None
        self.total_demand = g.total_demand
        self.unassigned_demand = 0.0
        self.is_reset = True
        self.tstt = None
        self.is_damaged = np.zeros(self.num_edges, dtype=np.float32)
        self.goal_mask = np.zeros(self.num_edges, dtype=np.float32)
        self.flow = np.zeros(self.num_edges, dtype=np.float32)
        if not _banner_done:
            rule = "Floyd-Warshall (torch rule)" if self._vec.params.sp_rule == _lib.SP_TORCH else "Dijkstra (scipy rule)"
            print(f"[RepairEnv] backend=hip(gfx950) device={dev} method={self.assignment_method} "
                  f"iters={self.assignment_iters} sp_backend={self.sp_backend}: {rule}")
            _banner_done = True
        self._init_betweenness()
        self.reset(damaged_ratio=damaged_ratio)

    # ------------------------------------------------------ GP path sets
    # RepairEnv.od_paths / od_path_flows (repair_env.py:199-200, 351-404).  With
    # assignment_method="gp" they live on the device; reading decodes them,
    # assigning (e.g. the greedy baseline's deepcopy restore,
    # src/baselines/__init__.py:46-65) uploads them before the next kernel call.
    def _gp_get(self, i):
        if self._vec.gp_state is None:
            return self._od_host[i]
        if self._gp_cache is None:
            self._gp_cache = list(self._vec.gp_paths(0))
        return self._gp_cache[i]

    def _gp_set(self, i, value):
        if self._vec.gp_state is None:
            self._od_host[i] = value
            return
        if self._gp_cache is None:
            self._gp_cache = list(self._vec.gp_paths(0))
        self._gp_cache[i] = value
        self._gp_dirty = True

    od_paths = property(lambda self: self._gp_get(0), lambda self, v: self._gp_set(0, v))
    od_path_flows = property(lambda self: self._gp_get(1), lambda self, v: self._gp_set(1, v))

    # ------------------------------------------------------ host <-> device
    def _push(self):
        v = self._vec
        if self._gp_dirty:
            v.set_gp_paths(0, self._gp_cache[0], self._gp_cache[1])
            self._gp_dirty = False
        v.flow[0].copy_(torch.from_numpy(np.asarray(self.flow, np.float32)))
        v.capacity[0].copy_(torch.from_numpy(np.asarray(self.capacities, np.float32)))
        v.damaged[0].copy_(torch.from_numpy(np.asarray(self.is_damaged, np.float32)))
        v.goal[0].copy_(torch.from_numpy(np.asarray(self.goal_mask, np.float32)))
        v.tstt[0] = float(self.tstt) if self.tstt is not None else 0.0
        v.initial_tstt[0] = float(self.initial_tstt) if self.initial_tstt is not None else -1.0

    def _pull(self):
        v = self._vec
        self._gp_cache = None
        self.flow = v.flow[0].cpu().numpy().copy()
        self.capacities = v.capacity[0].cpu().numpy().copy()
        self.is_damaged = v.damaged[0].cpu().numpy().copy()
        self.goal_mask = v.goal[0].cpu().numpy().copy()
        self.tstt = float(v.tstt[0])
        self.unassigned_demand = float(v.unassigned[0])

    def _init_betweenness(self):
        # One-off static betweenness of the full graph (repair_env.py:163-165).
        import networkx as nx
        G = nx.DiGraph()
        for e in self.edges:
            G.add_edge(e.u - 1, e.v - 1)
        bc = nx.betweenness_centrality(G, normalized=True)
        self.betweenness_vec = np.array([bc.get(i, 0.0) for i in range(self.num_nodes)], dtype=np.float32)

    # ----------------------------------------------------------------- API
    def reset(self, damaged_ratio: float = 0.3) -> EnvState:
        mask = self._sampler.sample(damaged_ratio)
        self._vec.reset(damaged=torch.from_numpy(mask)[None], observe=False)
        self._pull()
        self.initial_tstt = self.tstt
        if self._vec.gp_state is None:  # GP: the reset assignment rebuilt the device path sets
            self.od_paths = {}
            self.od_path_flows = {}
        self.is_reset = False
        return self.get_state()

    def step(self, action_edge_id: int) -> Tuple[EnvState, float, bool, Dict]:
        a = int(action_edge_id)
        if a < 0 or a >= self.num_edges:
            raise ValueError(f"action_edge_id {action_edge_id} out of range (0..{self.num_edges - 1})")
        prev_tstt = self.tstt
        self._push()
        _, reward, done, _ = self._vec.step(torch.tensor([a], dtype=torch.int32), observe=False, check=False)
        r = float(reward[0])
        d = bool(done[0])
        self._pull()
        if self.debug_reward and self.is_damaged[a] == 0:
            self._debug_step += 1
            if self.debug_reward_every <= 0 or self._debug_step % self.debug_reward_every == 0:
                print(f"[reward_debug] prev={prev_tstt:.6g} curr={self.tstt:.6g} diff={prev_tstt - self.tstt:.6g} "
                      f"reward={r:.6g}")
        return self.get_state(), r, d, {"tstt": self.tstt}

    def compute_flow_assignment(self):
        if self.assignment_iters <= 0:
            raise ValueError("assignment_iters must be > 0 to update TSTT.")
        if self.flow is None or self.is_reset:
            self.flow = np.zeros(self.num_edges, dtype=np.float32)
        self._push()
        self._vec.assign()
        self._pull()

    def get_state(self) -> EnvState:
        self._push()
        obs = self._vec.observe()
        nx_ = obs.node_x[0].cpu().numpy().copy()
        ex_ = obs.edge_x[0].cpu().numpy().copy()
        current = self.tstt if self.tstt is not None else self.initial_tstt
        log_tstt = float(np.log10(max(current, 1.0))) if current is not None else 0.0
        return EnvState(node_features=nx_, edge_features=ex_, edge_index=self.edge_index,
                        action_mask=self.is_damaged.astype(np.float32), log_tstt=log_tstt,
                        goal_mask=self.goal_mask.copy())

    def compute_reward(self, prev_tstt, curr_tstt, alpha=1.0, beta=10.0, gamma=0.1) -> float:
        delta = prev_tstt - curr_tstt
        bonus = beta if self.is_damaged.sum() == 0 else 0.0
        return alpha * delta + bonus - gamma

    def compute_reward_with_goal(self, prev_tstt, curr_tstt, goal_mask, damaged_mask, alpha=1.0, beta=10.0,
                                 gamma=0.1, mode="delta", clip=0.0) -> float:
        """Scalar host form of the device reward (repair_env.py:244-291), used
        by HER relabelling (src/train.py:805-823)."""
        complete = self.is_goal_complete(goal_mask, damaged_mask)
        bonus = beta if complete else 0.0
        if mode in ("minimize_tstt", "rel_improve"):
            base = self.initial_tstt if self.initial_tstt is not None else prev_tstt
            bb = max(base, 1.0)
            if mode == "minimize_tstt":
                reward = -alpha * (curr_tstt / bb)
            else:
                reward = alpha * (((prev_tstt - curr_tstt) / bb) * 100.0) - 1.0 * (curr_tstt / bb)
            reward = reward + bonus
        else:
            if mode == "neg_tstt":
                delta = -curr_tstt
            elif mode == "log_delta":
                delta = np.log10(max(prev_tstt, 1.0)) - np.log10(max(curr_tstt, 1.0))
            else:
                delta = prev_tstt - curr_tstt
            reward = alpha * delta + bonus - gamma
        if clip and clip > 0:
            reward = float(np.clip(reward, -clip, clip))
        return reward

    def is_goal_complete(self, goal_mask, damaged_mask) -> bool:
        return bool(np.sum(goal_mask * damaged_mask) == 0.0)

    def set_goal(self, goal_mask) -> None:
        self.goal_mask = np.asarray(goal_mask).astype(np.float32)

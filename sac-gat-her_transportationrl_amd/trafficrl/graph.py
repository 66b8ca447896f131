"""Device graph handle + host-side damage sampling.

TrafficGraph wraps trx_graph (include/trafficrl.h): the immutable,
device-resident network built from a GraphData exactly as RepairEnv.__init__
lays it out (src/env/repair_env.py:85-96).

DamageSampler reproduces RepairEnv.reset's damage draw
(repair_env.py:168-192): numpy PCG64 ``rng.choice(E, floor(E*ratio),
replace=False)`` with up to 50 rejections until the active-edge subgraph
(networkx edge_subgraph: only nodes incident to an active link) is strongly
connected.  The RNG stays on the host, so damage sets match the reference
seed-for-seed.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .data.tntp_parser import GraphData


class TrafficGraph:
    def __init__(self, graph_data: GraphData, device=None):
        import torch
        L = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("libtrafficrl needs a HIP device (MI355X); no CPU fallback is provided")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self.graph_data = graph_data
        self.num_nodes = int(graph_data.num_nodes)
        edges = graph_data.edges
        self.num_edges = len(edges)
        self.src = np.array([e.u - 1 for e in edges], dtype=np.int32)
        self.dst = np.array([e.v - 1 for e in edges], dtype=np.int32)
        self.edge_index = np.stack([self.src, self.dst]).astype(np.int64)
        self.t0 = np.array([e.t0 for e in edges], dtype=np.float32)
        self.cap0 = np.array([e.capacity for e in edges], dtype=np.float32)
        od = list(graph_data.od_demand.items())
        self.od_o = np.array([o - 1 for (o, _), _ in od], dtype=np.int32)
        self.od_d = np.array([d - 1 for (_, d), _ in od], dtype=np.int32)
        self.od_v = np.array([v for _, v in od], dtype=np.float64)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = L.trx_graph_create(
                self.num_nodes, self.num_edges, self.src.ctypes.data, self.dst.ctypes.data, self.t0.ctypes.data,
                self.cap0.ctypes.data, len(self.od_o), self.od_o.ctypes.data, self.od_d.ctypes.data,
                self.od_v.ctypes.data, ctypes.byref(handle))
        _lib.check(rc, "trx_graph_create")
        self._h = handle
        n, e, z, td = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_double()
        _lib.check(L.trx_graph_info(self._h, ctypes.byref(n), ctypes.byref(e), ctypes.byref(z), ctypes.byref(td)),
                   "trx_graph_info")
        self.num_origins = z.value
        self.total_demand = td.value  # float(np.sum(list(od_demand.values())))
        self.edge_id_map = {(int(u), int(v)): i for i, (u, v) in enumerate(zip(self.src, self.dst))}

    @property
    def handle(self):
        return self._h

    def workspace_bytes(self, num_envs: int) -> int:
        b = _lib.load().trx_workspace_bytes(self._h, int(num_envs))
        if b < 0:
            _lib.check(int(b), "trx_workspace_bytes")
        return int(b)

    def od_key_order(self):
        """1-based (o, d) keys in the device's OD order: grouped by origin
        ascending, dict order inside an origin (repair_env.py:490-491)."""
        if not hasattr(self, "_od_keys"):
            idx = sorted(range(len(self.od_o)), key=lambda k: (int(self.od_o[k]), k))
            self._od_keys = [(int(self.od_o[k]) + 1, int(self.od_d[k]) + 1) for k in idx]
        return self._od_keys

    def gp_state_bytes(self, num_envs: int, keep_paths: int) -> int:
        b = _lib.load().trx_gp_state_bytes(self._h, int(num_envs), int(keep_paths))
        if b < 0:
            _lib.check(int(b), "trx_gp_state_bytes")
        return int(b)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.trx_graph_destroy(h)
            self._h = None


def _strongly_connected_active(num_nodes, src, dst, active):
    """nx.is_strongly_connected(G.edge_subgraph(active edges)) for a small graph."""
    us, vs = src[active], dst[active]
    if us.size == 0:
        return False
    nodes = np.unique(np.concatenate([us, vs]))
    adj = [[] for _ in range(num_nodes)]
    radj = [[] for _ in range(num_nodes)]
    for u, v in zip(us.tolist(), vs.tolist()):
        adj[u].append(v)
        radj[v].append(u)

    def reach(start, g):
        seen = {start}
        stack = [start]
        while stack:
            x = stack.pop()
            for y in g[x]:
                if y not in seen:
                    seen.add(y)
                    stack.append(y)
        return seen

    s0 = int(nodes[0])
    need = set(nodes.tolist())
    return need <= reach(s0, adj) and need <= reach(s0, radj)


class DamageSampler:
    """Per-env damage draws (repair_env.py:168-192, 77-83)."""

    def __init__(self, graph: TrafficGraph, seed: int = 0, fixed_damage: bool = False,
                 fixed_damage_seed: int | None = None):
        self.g = graph
        self.rng = np.random.default_rng(seed)
        self.fixed_damage = bool(fixed_damage)
        self._fixed_rng = np.random.default_rng(fixed_damage_seed) if fixed_damage_seed is not None else None
        self._fixed_indices = None

    def sample(self, damaged_ratio: float = 0.3) -> np.ndarray:
        E = self.g.num_edges
        count = max(1, int(E * damaged_ratio))
        idx = self._fixed_indices if self.fixed_damage else None
        if idx is None:
            rng = self._fixed_rng if self.fixed_damage and self._fixed_rng is not None else self.rng
            for _ in range(50):
                cand = rng.choice(E, size=count, replace=False)
                active = np.ones(E, dtype=bool)
                active[cand] = False
                if not active.any():
                    continue
                if _strongly_connected_active(self.g.num_nodes, self.g.src, self.g.dst, active):
                    idx = cand
                    break
            if idx is None:
                idx = rng.choice(E, size=count, replace=False)
            if self.fixed_damage:
                self._fixed_indices = idx
        mask = np.zeros(E, dtype=np.float32)
        mask[idx] = 1.0
        return mask

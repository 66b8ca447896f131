"""Device graph handle + host-side damage sampling.

TrafficGraph wraps trx_graph (include/trafficrl.h): the immutable,
device-resident network built from a GraphData exactly as RepairEnv.__init__
lays it out (src/env/repair_env.py:85-96).

DamageSampler / damage_sample_batch reproduce RepairEnv.reset's damage draw
(repair_env.py:167-192): numpy PCG64 ``rng.choice(E, floor(E*ratio),
replace=False)`` with up to 50 rejections until the active-edge subgraph
(networkx DiGraph edge_subgraph: only nodes incident to an active arc) is
strongly connected -- natively (trx_damage_sample, csrc/damage_host.hip, a
restatement of numpy's Generator), for a whole env batch per call, so damage
sets AND generator states match the reference seed-for-seed.
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


PCG64_DTYPE = np.dtype([("state_hi", "<u8"), ("state_lo", "<u8"), ("inc_hi", "<u8"), ("inc_lo", "<u8"),
                        ("has_uint32", "<u4"), ("uinteger", "<u4")])   # trx_pcg64 (include/trafficrl.h)
_M64 = (1 << 64) - 1


def pcg_states(rngs) -> np.ndarray:
    """trx_pcg64 records of numpy Generators (PCG64) -- or of default_rng(seed)
    for int seeds -- in order."""
    out = np.zeros(len(rngs), PCG64_DTYPE)
    for i, r in enumerate(rngs):
        st = (np.random.default_rng(int(r)) if isinstance(r, (int, np.integer)) else r).bit_generator.state
        if st["bit_generator"] != "PCG64":
            raise ValueError(f"damage draws need a PCG64 generator, got {st['bit_generator']}")
        s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
        out[i] = (s >> 64, s & _M64, inc >> 64, inc & _M64, int(st["has_uint32"]), int(st["uinteger"]))
    return out


def set_generator_state(rng: np.random.Generator, rec) -> None:
    """Write a trx_pcg64 record back into a numpy Generator."""
    rng.bit_generator.state = {
        "bit_generator": "PCG64",
        "state": {"state": (int(rec["state_hi"]) << 64) | int(rec["state_lo"]),
                  "inc": (int(rec["inc_hi"]) << 64) | int(rec["inc_lo"])},
        "has_uint32": int(rec["has_uint32"]), "uinteger": int(rec["uinteger"])}


def damage_sample_batch(num_nodes: int, src: np.ndarray, dst: np.ndarray, states: np.ndarray,
                        damaged_ratio: float = 0.3, nthreads: int = 0, out: np.ndarray = None) -> np.ndarray:
    """RepairEnv.reset's damage draw for len(states) envs in one native call
    (trx_damage_sample): float32 masks [n, E] (into `out` when given, e.g. a
    view of pinned host memory); `states` (PCG64_DTYPE) advance in place
    exactly as each env's numpy Generator would."""
    E = len(src)
    count = max(1, int(E * damaged_ratio))
    if E > 10000:   # numpy's choice leaves its Floyd branch above 10000 (not restated natively)
        raise ValueError(f"damage draws support num_edges <= 10000 (numpy Generator.choice Floyd branch); got {E}")
    if not (isinstance(states, np.ndarray) and states.dtype == PCG64_DTYPE and states.flags.c_contiguous):
        raise TypeError("states must be a C-contiguous PCG64_DTYPE array (pcg_states)")
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    if out is None:
        out = np.zeros((len(states), E), np.float32)
    elif out.shape != (len(states), E) or out.dtype != np.float32 or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous float32 array [n, E]")
    L = _lib.load()
    _lib.check(L.trx_damage_sample(int(num_nodes), E, src.ctypes.data, dst.ctypes.data, count, 50, len(states),
                                   states.ctypes.data, out.ctypes.data, int(nthreads)), "trx_damage_sample")
    return out


class DamageSampler:
    """Per-env damage draws (repair_env.py:168-192, 77-83) through the native
    batch sampler; self.rng stays the env's numpy Generator, advanced exactly as
    the reference's self.rng is."""

    def __init__(self, graph: TrafficGraph, seed: int = 0, fixed_damage: bool = False,
                 fixed_damage_seed: int | None = None):
        self.g = graph
        self.rng = np.random.default_rng(seed)
        self.fixed_damage = bool(fixed_damage)
        self._fixed_rng = np.random.default_rng(fixed_damage_seed) if fixed_damage_seed is not None else None
        self._fixed_indices = None

    def sample(self, damaged_ratio: float = 0.3) -> np.ndarray:
        if self.fixed_damage and self._fixed_indices is not None:
            mask = np.zeros(self.g.num_edges, dtype=np.float32)
            mask[self._fixed_indices] = 1.0
            return mask
        rng = self._fixed_rng if self.fixed_damage and self._fixed_rng is not None else self.rng
        st = pcg_states([rng])
        mask = damage_sample_batch(self.g.num_nodes, self.g.src, self.g.dst, st, damaged_ratio)[0]
        set_generator_state(rng, st[0])
        if self.fixed_damage:
            self._fixed_indices = np.flatnonzero(mask)
        return mask

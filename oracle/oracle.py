"""ctypes front-end of the CPU oracle (oracle/trx_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.

Also holds the numpy restatement of the observation builder
(src/env/repair_env.py:751-819, RepairEnv.get_state) including networkx's
Brandes betweenness (networkx/algorithms/centrality/betweenness.py:
_single_source_shortest_path_basic + _accumulate_basic + _rescale) in pure
Python, used for small parity cases.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

METHODS = {"msa": 0, "fw": 1, "cfw": 2}
SP_RULES = {"scipy": 0, "torch": 1}   # _all_or_nothing scipy branch / _all_or_nothing_torch
REWARD_MODES = {"delta": 0, "log_delta": 1, "neg_tstt": 2, "minimize_tstt": 3, "rel_improve": 4}

_i32p = ctypes.POINTER(ctypes.c_int32)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)


class _Graph(ctypes.Structure):
    _fields_ = [
        ("N", ctypes.c_int), ("E", ctypes.c_int), ("P", ctypes.c_int),
        ("src", _i32p), ("dst", _i32p), ("t0", _f32p), ("cap0", _f32p),
        ("od_o", _i32p), ("od_d", _i32p), ("od_v", _f64p),
        ("indptr", _i32p), ("indices", _i32p), ("csr_eid", _i32p), ("eid_of", _i32p),
        ("org_ptr", _i32p), ("org_idx", _i32p), ("total_demand", ctypes.c_double),
    ]


def build():
    """Compile liboracle.so with gcc (no reference sources involved)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_graph_build.argtypes = [ctypes.POINTER(_Graph)]
        L.orc_graph_build.restype = ctypes.c_int
        L.orc_assign_batch.argtypes = [ctypes.POINTER(_Graph), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_float, ctypes.c_float, ctypes.c_double, _f32p, _f32p, _f32p,
                                       _f32p, _f64p, _f64p, _u8p, ctypes.c_int, ctypes.c_int]
        L.orc_assign_batch.restype = ctypes.c_int
        L.orc_aon_fw.argtypes = [ctypes.POINTER(_Graph), _f32p, _f32p, _i32p]
        L.orc_aon_fw.restype = ctypes.c_double
        L.orc_observe_batch.argtypes = [ctypes.POINTER(_Graph), ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _f64p,
                                        _f32p, _f32p, _f32p, ctypes.c_int]
        L.orc_observe_batch.restype = ctypes.c_int
        L.orc_all_pairs.argtypes = [ctypes.POINTER(_Graph), _f32p, _f64p, _i32p]
        L.orc_aon.argtypes = [ctypes.POINTER(_Graph), _f32p, _f32p]
        L.orc_aon.restype = ctypes.c_double
        L.orc_bpr.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _f32p, ctypes.c_float, ctypes.c_float, _f32p]
        L.orc_pairwise_sum_f32.argtypes = [_f32p, ctypes.c_long]
        L.orc_pairwise_sum_f32.restype = ctypes.c_float
        L.orc_reward.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                 ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double]
        L.orc_reward.restype = ctypes.c_double
        L.orc_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


class OracleGraph:
    """Graph arrays in reference order (src/env/repair_env.py:85-96)."""

    def __init__(self, num_nodes, src, dst, t0, cap0, od_o, od_d, od_v):
        self.N = int(num_nodes)
        self.src = np.ascontiguousarray(src, np.int32)
        self.dst = np.ascontiguousarray(dst, np.int32)
        self.t0 = np.ascontiguousarray(t0, np.float32)
        self.cap0 = np.ascontiguousarray(cap0, np.float32)
        self.od_o = np.ascontiguousarray(od_o, np.int32)
        self.od_d = np.ascontiguousarray(od_d, np.int32)
        self.od_v = np.ascontiguousarray(od_v, np.float64)
        self.E = len(self.src)
        g = _Graph()
        g.N, g.E, g.P = self.N, self.E, len(self.od_o)
        g.src, g.dst = _p(self.src, _i32p), _p(self.dst, _i32p)
        g.t0, g.cap0 = _p(self.t0, _f32p), _p(self.cap0, _f32p)
        g.od_o, g.od_d, g.od_v = _p(self.od_o, _i32p), _p(self.od_d, _i32p), _p(self.od_v, _f64p)
        rc = lib().orc_graph_build(ctypes.byref(g))
        if rc != 0:
            raise ValueError(f"oracle graph build failed ({rc})")
        self._g = g
        self.total_demand = g.total_demand

    @classmethod
    def from_npz(cls, path):
        z = np.load(path)
        return cls(int(z["num_nodes"]), z["src"], z["dst"], z["t0"], z["cap0"], z["od_o"], z["od_d"], z["od_v"])

    # ---------------------------------------------------------------- ops
    def bpr(self, flow, cap, damaged, alpha=0.15, beta=4.0):
        flow = np.ascontiguousarray(flow, np.float32)
        cap = np.ascontiguousarray(cap, np.float32)
        damaged = np.ascontiguousarray(damaged, np.float32)
        t = np.empty(self.E, np.float32)
        lib().orc_bpr(self.E, _p(flow, _f32p), _p(cap, _f32p), _p(self.t0, _f32p), _p(damaged, _f32p),
                      alpha, beta, _p(t, _f32p))
        return t

    def aon(self, t, sp="scipy"):
        """_all_or_nothing (scipy branch, repair_env.py:481-503) or, sp="torch",
        _all_or_nothing_torch (520-573).  Returns (aux, unassigned)."""
        t = np.ascontiguousarray(t, np.float32)
        aux = np.empty(self.E, np.float32)
        if sp == "torch":
            un = lib().orc_aon_fw(ctypes.byref(self._g), _p(t, _f32p), _p(aux, _f32p), None)
        else:
            un = lib().orc_aon(ctypes.byref(self._g), _p(t, _f32p), _p(aux, _f32p))
        return aux, un

    def next_hop(self, t):
        """The torch backend's float32 Floyd-Warshall next_hop matrix [N,N]."""
        t = np.ascontiguousarray(t, np.float32)
        aux = np.empty(self.E, np.float32)
        nh = np.empty((self.N, self.N), np.int32)
        lib().orc_aon_fw(ctypes.byref(self._g), _p(t, _f32p), _p(aux, _f32p), _p(nh, _i32p))
        return nh

    def observe(self, cap, damaged, goal, flow, tstt, nthreads=1):
        """Batched get_state (repair_env.py:751-819) in C: (node_x [B,N,4],
        edge_x [B,E,6], mask [B,E])."""
        cap = np.ascontiguousarray(np.atleast_2d(cap), np.float32)
        damaged = np.ascontiguousarray(np.atleast_2d(damaged), np.float32)
        goal = np.ascontiguousarray(np.atleast_2d(goal), np.float32)
        flow = np.ascontiguousarray(np.atleast_2d(flow), np.float32)
        tstt = np.ascontiguousarray(np.atleast_1d(tstt), np.float64)
        B = flow.shape[0]
        nx_ = np.empty((B, self.N, 4), np.float32)
        ex = np.empty((B, self.E, 6), np.float32)
        m = np.empty((B, self.E), np.float32)
        rc = lib().orc_observe_batch(ctypes.byref(self._g), B, _p(cap, _f32p), _p(damaged, _f32p), _p(goal, _f32p),
                                     _p(flow, _f32p), _p(tstt, _f64p), _p(nx_, _f32p), _p(ex, _f32p), _p(m, _f32p),
                                     int(nthreads))
        if rc != 0:
            raise RuntimeError("oracle observe failed")
        return nx_, ex, m

    def all_pairs(self, t):
        t = np.ascontiguousarray(t, np.float32)
        d = np.empty((self.N, self.N), np.float64)
        p = np.empty((self.N, self.N), np.int32)
        lib().orc_all_pairs(ctypes.byref(self._g), _p(t, _f32p), _p(d, _f64p), _p(p, _i32p))
        return d, p

    def assign(self, cap, damaged, flow, method="msa", iters=30, alpha=0.15, beta=4.0, penalty=1e4,
               env_mask=None, nthreads=1, sp="scipy"):
        """Batched compute_flow_assignment.  cap/damaged/flow: [B,E] (or [E]).
        sp: "scipy" (Dijkstra, the default backend here) or "torch" (the
        reference's sp_backend="torch" Floyd-Warshall).
        Returns (flow_out, t_out, tstt[B], unassigned[B])."""
        single = np.ndim(flow) == 1
        cap = np.ascontiguousarray(np.atleast_2d(cap), np.float32)
        damaged = np.ascontiguousarray(np.atleast_2d(damaged), np.float32)
        flow = np.array(np.atleast_2d(flow), np.float32, copy=True, order="C")
        B = flow.shape[0]
        t = np.zeros_like(flow)
        tstt = np.zeros(B, np.float64)
        un = np.zeros(B, np.float64)
        mask = None if env_mask is None else np.ascontiguousarray(env_mask, np.uint8)
        rc = lib().orc_assign_batch(ctypes.byref(self._g), B, METHODS[method], int(iters), alpha, beta, penalty,
                                    _p(cap, _f32p), _p(damaged, _f32p), _p(flow, _f32p), _p(t, _f32p),
                                    _p(tstt, _f64p), _p(un, _f64p), None if mask is None else _p(mask, _u8p),
                                    int(nthreads), SP_RULES[sp])
        if rc != 0:
            raise RuntimeError("oracle assign failed")
        if single:
            return flow[0], t[0], float(tstt[0]), float(un[0])
        return flow, t, tstt, un


def pairwise_sum_f32(a):
    a = np.ascontiguousarray(a, np.float32)
    return float(lib().orc_pairwise_sum_f32(_p(a, _f32p), len(a)))


def reward(mode, prev, curr, initial, complete, alpha=1.0, beta=10.0, gamma=0.1, clip=0.0):
    return lib().orc_reward(REWARD_MODES[mode], prev, curr, -1.0 if initial is None else initial, int(complete),
                            alpha, beta, gamma, clip)


def max_threads():
    return lib().orc_max_threads()


# ------------------------------------------------------ observation oracle
def nx_node_order(src, dst):
    """Node insertion order of the reference's nx.DiGraph (repair_env.py:106-109)."""
    order, seen = [], set()
    for u, v in zip(src, dst):
        for n in (int(u), int(v)):
            if n not in seen:
                seen.add(n)
                order.append(n)
    return order


def betweenness_active(N, src, dst, damaged):
    """nx.betweenness_centrality(G.edge_subgraph(active), normalized=True),
    restated (networkx 3.4 betweenness.py) for the reference's DiGraph."""
    order = nx_node_order(src, dst)
    adj = {n: [] for n in order}
    for u, v in zip(src, dst):  # edge insertion order == adjacency order
        adj[int(u)].append(int(v))
    act = set()
    for e, (u, v) in enumerate(zip(src, dst)):
        if damaged[e] == 0:
            act.add((int(u), int(v)))
    nodes = [n for n in order if any((n == a or n == b) for (a, b) in act)]
    nodeset = set(nodes)
    sub = {n: [w for w in adj[n] if (n, w) in act] for n in nodes}
    bc = dict.fromkeys(nodes, 0.0)
    for s in nodes:
        S, P, sigma, D = [], {}, dict.fromkeys(nodes, 0.0), {}
        for v in nodes:
            P[v] = []
        sigma[s] = 1.0
        D[s] = 0
        Q = [s]
        qi = 0
        while qi < len(Q):
            v = Q[qi]; qi += 1
            S.append(v)
            Dv, sigmav = D[v], sigma[v]
            for w in sub[v]:
                if w not in D:
                    Q.append(w)
                    D[w] = Dv + 1
                if D[w] == Dv + 1:
                    sigma[w] += sigmav
                    P[w].append(v)
        delta = dict.fromkeys(S, 0)
        while S:
            w = S.pop()
            coeff = (1 + delta[w]) / sigma[w]
            for v in P[w]:
                delta[v] += sigma[v] * coeff
            if w != s:
                bc[w] += delta[w]
    n = len(nodes)
    if n > 2:
        scale = 1 / ((n - 1) * (n - 2))
        for v in bc:
            bc[v] *= scale
    out = np.zeros(N, np.float32)
    for v in nodeset:
        out[v] = bc[v]
    return out


def observation(src, dst, N, t0, cap0, capacities, damaged, goal, flow, tstt, total_demand):
    """numpy restatement of RepairEnv.get_state (repair_env.py:751-819)."""
    E = len(src)
    bw = betweenness_active(N, src, dst, damaged)
    bw_max = float(np.max(bw)) if bw.size else 0.0
    if bw_max > 0:
        bw = bw / bw_max
    raw_vc = np.zeros(E, np.float32)
    for i in range(E):
        raw_vc[i] = flow[i] / max(capacities[i], 1e-6)
    vc = np.where(damaged > 0, 0.0, raw_vc)
    vc = np.clip(np.log1p(vc), 0.0, 10.0)
    goal_total = float(np.sum(goal))
    remaining = float(np.sum(goal * damaged))
    remaining_ratio = remaining / max(goal_total, 1.0)
    avg_flow = float(np.mean(flow[damaged == 0])) if np.sum(damaged == 0) > 0 else 0.0
    avg_flow_norm = avg_flow / max(total_demand / max(E, 1), 1.0)
    log_tstt = float(np.log10(max(tstt, 1.0)))
    node = np.stack([bw, np.full(N, remaining_ratio, np.float32), np.full(N, avg_flow_norm, np.float32),
                     np.full(N, log_tstt, np.float32)], axis=1)
    max_t0 = float(np.max(t0)); max_cap = float(np.max(cap0))
    t0_norm = np.log10(t0 + 1.0) / np.log10(max_t0 + 1.0)
    cap_norm = np.log10(capacities + 1.0) / np.log10(max_cap + 1.0)
    eid = np.arange(E, dtype=np.float32) / max(E - 1, 1)
    edge = np.stack([t0_norm.astype(np.float32), cap_norm.astype(np.float32), vc, damaged, goal, eid], axis=1)
    return node.astype(np.float32), edge.astype(np.float32), damaged.astype(np.float32)


# ------------------------------------------- path-based (GP) assignment oracle
class GPPaths:
    """Per-env path sets of the GP assignment: RepairEnv.od_paths /
    od_path_flows (repair_env.py:351-419).  Keys (0-based (o, d)) keep their
    insertion order; each key holds [edge-id tuple] paths and float64 flows."""

    def __init__(self):
        self.paths = {}
        self.flows = {}

    def copy(self):
        c = GPPaths()
        c.paths = {k: list(v) for k, v in self.paths.items()}
        c.flows = {k: list(v) for k, v in self.flows.items()}
        return c


def _f32_path_cost(t, path):
    """_path_cost (repair_env.py:346-349): float(np.sum(t[path])) -- numpy's
    float32 pairwise sum over the path's links in path order."""
    if not path:
        return float("inf")
    return float(np.sum(t[list(path)]))


def gp_assign(og: OracleGraph, cap, damaged, flow, state: GPPaths, iters, gp_step=1.0, keep=3, reset=False,
              alpha=0.15, beta=4.0, penalty=1e4):
    """One env's _compute_flow_assignment_gp (repair_env.py:351-419) followed by
    compute_tstt, restated over the oracle's scipy-order shortest paths.
    Mutates `state`; returns (flow, t, tstt, unassigned)."""
    cap = np.ascontiguousarray(cap, np.float32)
    damaged = np.ascontiguousarray(damaged, np.float32)
    t = og.bpr(flow, cap, damaged, alpha, beta)
    if reset or not state.paths:
        state.paths.clear()
        state.flows.clear()
    # OD entries grouped by origin, dict order inside an origin (the reference
    # scans origins ascending and filters the dict for each)
    by_origin = {}
    for o, d, v in zip(og.od_o.tolist(), og.od_d.tolist(), og.od_v.tolist()):
        by_origin.setdefault(o, []).append((d, v))
    eid = {(int(u), int(v)): e for e, (u, v) in enumerate(zip(og.src, og.dst))}
    unassigned = 0.0
    for it in range(iters):
        unassigned = 0.0
        step = gp_step if gp_step > 0 else 1.0 / (it + 1.0)
        _, pred = og.all_pairs(t)
        for origin in sorted(by_origin):
            for dest, demand in by_origin[origin]:
                if dest == origin or pred[origin, dest] < 0:
                    unassigned += demand
                    continue
                nodes = [dest]
                while nodes[-1] != origin:
                    nodes.append(int(pred[origin, nodes[-1]]))
                nodes.reverse()
                sp = tuple(eid[(nodes[i], nodes[i + 1])] for i in range(len(nodes) - 1))
                key = (origin, dest)
                if key not in state.paths:
                    state.paths[key] = [sp]
                    state.flows[key] = [float(demand)]
                    continue
                paths, flows = state.paths[key], state.flows[key]
                if sp not in paths:
                    paths.append(sp)
                    flows.append(0.0)
                costs = [_f32_path_cost(t, p) for p in paths]
                best = int(np.argmin(costs))
                if len(flows) > 1:
                    moved = 0.0
                    for i in range(len(flows)):
                        if i != best:
                            tr = step * flows[i]
                            flows[i] -= tr
                            moved += tr
                    flows[best] += moved
                if keep > 0 and len(paths) > keep:
                    order = np.argsort(costs)[:keep]
                    new_p = [paths[i] for i in order]
                    new_f = [flows[i] for i in order]
                    tot = float(np.sum(new_f))
                    if tot > 0:
                        new_f = [f * demand / tot for f in new_f]
                    else:
                        new_f = [0.0] * len(new_f)
                        new_f[0] = float(demand)
                    state.paths[key], state.flows[key] = new_p, new_f
        new_flow = np.zeros(og.E, np.float32)
        for key, paths in state.paths.items():
            for p, f in zip(paths, state.flows[key]):
                if f <= 0:
                    continue
                for e in p:
                    new_flow[e] += f
        flow = new_flow
        t = og.bpr(flow, cap, damaged, alpha, beta)
    td = max(og.total_demand, 1.0)
    tstt = pairwise_sum_f32(flow * t) / td + (penalty * (unassigned / td) if unassigned > 0 else 0.0)
    return flow, t, tstt, unassigned

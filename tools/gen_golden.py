#!/usr/bin/env python3
"""Generate the golden parity fixtures under tests/golden/ by running the
reference environment read-only in THIS container.

The reference (pop-pop-pOp-dev/SAC-GAT-HER_transportationRL) is plain Python on
numpy/scipy/networkx, importable from /root/reference.  Nothing from it is
copied: this script imports it, drives it through its own public methods and
stores inputs/outputs as small .npz/.json data files.  The reference never
travels to the GPU box; the fixtures do.

Two variants of every env fixture are written:

* ``native``: the reference exactly as it runs on this host.  Its BPR power
  ``vc ** 4.0`` (src/env/repair_env.py:673) is numpy's float32 ``power``, which
  on this AVX-512 host dispatches to an SVML kernel that is *not* correctly
  rounded (~21 % of results differ by 1 ulp from the exact value).  That last
  ulp therefore depends on which CPU runs the reference.
* ``crpow``: identical code, except the float32 power is evaluated as
  ``float32((double(vc)^2)^2)`` -- the host-independent definition this
  framework (oracle + HIP) adopts.  Every other operation is the reference's.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from src.data.tntp_parser import load_graph_data  # noqa: E402
from src.env.repair_env import RepairEnv  # noqa: E402
from src.baselines import select_greedy_one_step  # noqa: E402

NET = os.path.join(REF, "data/SiouxFalls/SiouxFalls_net.tntp")
TRIPS = os.path.join(REF, "data/SiouxFalls/SiouxFalls_trips.tntp")

# configs/sioux_falls.yaml reward / damage settings (the trainer's config)
ENV_KW = dict(
    damaged_ratio=0.3,
    sp_backend="scipy",
    reward_mode="rel_improve",
    reward_alpha=1.0,
    reward_beta=0.0,
    reward_gamma=0.0,
    reward_clip=2.0,
    capacity_damage=1e-3,
    unassigned_penalty=1e4,
)


class CRPowEnv(RepairEnv):
    """Reference env whose BPR power is evaluated host-independently.

    Same statement sequence as src/env/repair_env.py:667-677 except that
    ``vc ** beta`` is float32(((double)vc^2)^2) for beta == 4.
    """

    def compute_travel_time(self, flow):
        flow_np = np.asarray(flow, dtype=np.float32)
        cap = np.maximum(self.capacities, 1e-6)
        vc = np.clip(flow_np / cap, 0.0, 10.0)
        assert self.bpr_beta == 4.0
        v = vc.astype(np.float64)
        v2 = v * v
        p = (v2 * v2).astype(np.float32)
        t = self.t0 * (1.0 + self.bpr_alpha * p)
        damaged_mask = self.is_damaged > 0.5
        t = t.astype(np.float32)
        t[damaged_mask] = 1e6
        return t


def make_env(cls, **kw):
    graph = load_graph_data(NET, TRIPS)
    args = dict(ENV_KW)
    args.update(kw)
    return cls(graph, **args)


def graph_arrays():
    g = load_graph_data(NET, TRIPS)
    src = np.array([e.u - 1 for e in g.edges], dtype=np.int32)
    dst = np.array([e.v - 1 for e in g.edges], dtype=np.int32)
    cap = np.array([e.capacity for e in g.edges], dtype=np.float32)
    t0 = np.array([e.t0 for e in g.edges], dtype=np.float32)
    od = list(g.od_demand.items())
    od_o = np.array([o - 1 for (o, _), _ in od], dtype=np.int32)
    od_d = np.array([d - 1 for (_, d), _ in od], dtype=np.int32)
    od_v = np.array([v for _, v in od], dtype=np.float64)
    np.savez_compressed(
        os.path.join(OUT, "sf_graph.npz"),
        num_nodes=np.int32(g.num_nodes), src=src, dst=dst, cap0=cap, t0=t0,
        od_o=od_o, od_d=od_d, od_v=od_v,
    )
    return g


def state_arrays(s):
    return s.node_features.astype(np.float32), s.edge_features.astype(np.float32), s.action_mask.astype(np.float32)


def fixed_seed_resets(variant, cls):
    """(ii) fixed_damage_seed=42 resets for msa/fw/cfw."""
    out = {}
    for method, iters in [("msa", 30), ("fw", 30), ("cfw", 60), ("msa", 60), ("fw", 50), ("msa", 1), ("fw", 2)]:
        env = make_env(cls, assignment_method=method, assignment_iters=iters,
                       fixed_damage=True, fixed_damage_seed=42, seed=42)
        t = env.compute_travel_time(env.flow)
        key = f"{method}{iters}"
        out[f"{key}_damaged"] = env.is_damaged.copy()
        out[f"{key}_flow"] = env.flow.copy()
        out[f"{key}_t"] = t
        out[f"{key}_tstt"] = np.float64(env.tstt)
        out[f"{key}_unassigned"] = np.float64(env.unassigned_demand)
    np.savez_compressed(os.path.join(OUT, f"sf_reset_seed42_{variant}.npz"), **out)


def iteration_trace(variant, cls):
    """(iv) per-iteration aux/flow/t for the first 3 MSA iterations of the
    seed-42 reset, using the env's own BPR/AON methods (repair_env.py:308-343)."""
    env = make_env(cls, assignment_method="msa", assignment_iters=3,
                   fixed_damage=True, fixed_damage_seed=42, seed=42)
    flow = np.zeros(env.num_edges, dtype=np.float32)
    env.flow = flow
    t = env.compute_travel_time(flow)
    out = {"t_init": t.copy(), "damaged": env.is_damaged.copy(), "capacities": env.capacities.copy()}
    for it in range(3):
        aux, un = env._all_or_nothing(t)
        step = 1.0 / (it + 1.0)
        flow = (1 - step) * flow + step * aux
        t = env.compute_travel_time(flow)
        out[f"aux_{it}"] = aux
        out[f"flow_{it}"] = flow.copy()
        out[f"t_{it}"] = t.copy()
        out[f"unassigned_{it}"] = np.float64(un)
    np.savez_compressed(os.path.join(OUT, f"sf_trace_seed42_{variant}.npz"), **out)


def greedy_episode(variant, cls, method, iters):
    """(iii)+(vi) greedy one-step episode (src/baselines/__init__.py:35-101)
    recording every transition: action, reward, done, tstt, flow, obs."""
    env = make_env(cls, assignment_method=method, assignment_iters=iters,
                   fixed_damage=True, fixed_damage_seed=42, seed=42)
    state = env.reset()
    rec = {"actions": [], "rewards": [], "dones": [], "tstt": [], "flows": [], "node_x": [], "edge_x": [], "mask": []}
    nx0, ex0, m0 = state_arrays(state)
    rec0 = {"reset_node_x": nx0, "reset_edge_x": ex0, "reset_mask": m0,
            "reset_flow": env.flow.copy(), "initial_tstt": np.float64(env.initial_tstt)}
    # greedy what-if candidate TSTTs for the first decision (22 candidates)
    cand = np.where(state.action_mask > 0)[0]
    saved = (env.is_damaged.copy(), env.capacities.copy(), env.flow.copy(), env.tstt, env.unassigned_demand)
    cand_tstt = []
    for a in cand:
        env.is_damaged[a] = 0.0
        env.capacities[a] = env.initial_capacities[a]
        env.compute_flow_assignment()
        cand_tstt.append(env.tstt)
        env.is_damaged[:] = saved[0]
        env.capacities[:] = saved[1]
        env.flow = saved[2].copy()
        env.tstt = saved[3]
        env.unassigned_demand = saved[4]
    rec0["first_candidates"] = cand.astype(np.int32)
    rec0["first_candidate_tstt"] = np.array(cand_tstt, dtype=np.float64)
    done = False
    while not done:
        a = select_greedy_one_step(env, state)
        state, r, done, info = env.step(a)
        nx_, ex_, m_ = state_arrays(state)
        rec["actions"].append(a)
        rec["rewards"].append(r)
        rec["dones"].append(done)
        rec["tstt"].append(info["tstt"])
        rec["flows"].append(env.flow.copy())
        rec["node_x"].append(nx_)
        rec["edge_x"].append(ex_)
        rec["mask"].append(m_)
    out = {k: np.array(v) for k, v in rec.items()}
    out["actions"] = out["actions"].astype(np.int32)
    out["rewards"] = out["rewards"].astype(np.float64)
    out["tstt"] = out["tstt"].astype(np.float64)
    out.update(rec0)
    np.savez_compressed(os.path.join(OUT, f"sf_greedy_{method}{iters}_{variant}.npz"), **out)
    return out


def random_seed_resets(variant, cls, seeds):
    """(vii) damage index sets for seeds (numpy PCG64 via RepairEnv(seed=s)),
    MSA-30 reset flows/TSTT, plus 3 random valid steps per seed
    (actions from default_rng(7+seed)), incl. an invalid (repaired) action."""
    E = 76
    dam = np.zeros((len(seeds), E), np.float32)
    flow = np.zeros((len(seeds), E), np.float32)
    tstt = np.zeros(len(seeds), np.float64)
    step_actions = np.zeros((len(seeds), 4), np.int32)
    step_flow = np.zeros((len(seeds), 4, E), np.float32)
    step_tstt = np.zeros((len(seeds), 4), np.float64)
    step_reward = np.zeros((len(seeds), 4), np.float64)
    step_done = np.zeros((len(seeds), 4), np.bool_)
    for i, s in enumerate(seeds):
        env = make_env(cls, assignment_method="msa", assignment_iters=30, seed=s)
        dam[i] = env.is_damaged
        flow[i] = env.flow
        tstt[i] = env.tstt
        rng = np.random.default_rng(7 + s)
        first = None
        for j in range(4):
            if j == 2 and first is not None:
                a = first  # already repaired -> reward -1, no assignment (repair_env.py:210-212)
            else:
                cands = np.where(env.is_damaged > 0)[0]
                a = int(rng.choice(cands))
                if first is None:
                    first = a
            _, r, d, info = env.step(a)
            step_actions[i, j] = a
            step_flow[i, j] = env.flow
            step_tstt[i, j] = info["tstt"]
            step_reward[i, j] = r
            step_done[i, j] = d
    np.savez_compressed(
        os.path.join(OUT, f"sf_random_resets_{variant}.npz"),
        seeds=np.array(seeds, np.int32), damaged=dam, flow=flow, tstt=tstt,
        step_actions=step_actions, step_flow=step_flow, step_tstt=step_tstt,
        step_reward=step_reward, step_done=step_done,
    )


def scipy_pred_matrices(seeds):
    """(v) scipy dijkstra pred/dist at t = BPR(0) for several damage patterns,
    with tie flags (OD rows where >1 shortest-path tail attains dist)."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    g = load_graph_data(NET, TRIPS)
    src = np.array([e.u - 1 for e in g.edges]); dst = np.array([e.v - 1 for e in g.edges])
    t0 = np.array([e.t0 for e in g.edges], dtype=np.float32)
    N = g.num_nodes
    preds, dists, weights, ties = [], [], [], []
    for s in seeds:
        env = make_env(CRPowEnv, assignment_method="msa", assignment_iters=1, seed=s)
        t = env.compute_travel_time(np.zeros(76, np.float32))
        gr = csr_matrix((t.copy(), (src, dst)), shape=(N, N))
        d, p = dijkstra(gr, directed=True, indices=range(N), return_predecessors=True)
        tie = np.zeros((N, N), np.bool_)
        for o in range(N):
            for v in range(N):
                if v == o:
                    continue
                tails = [src[e] for e in range(76) if dst[e] == v and d[o, src[e]] + np.float64(t[e]) == d[o, v]]
                tie[o, v] = len(tails) > 1
        preds.append(p.astype(np.int32)); dists.append(d); weights.append(t); ties.append(tie)
    np.savez_compressed(os.path.join(OUT, "sf_scipy_pred.npz"), seeds=np.array(seeds, np.int32),
                        pred=np.array(preds), dist=np.array(dists), t=np.array(weights), tie=np.array(ties))


def undamaged_anchors(variant, cls):
    """(viii) undamaged-network UE anchors (sum flow*t)."""
    out = {}
    for method, iters in [("msa", 30), ("fw", 30), ("fw", 200)]:
        env = make_env(cls, assignment_method=method, assignment_iters=iters, fixed_damage=True,
                       fixed_damage_seed=42, seed=0)
        env.is_damaged[:] = 0.0
        env.capacities = env.initial_capacities.copy()
        env.flow = np.zeros(env.num_edges, np.float32)
        env.compute_flow_assignment()
        t = env.compute_travel_time(env.flow)
        out[f"{method}{iters}_flow"] = env.flow.copy()
        out[f"{method}{iters}_tstt"] = np.float64(env.tstt)
        out[f"{method}{iters}_sum_ft"] = np.float64(np.sum(env.flow * t))
    np.savez_compressed(os.path.join(OUT, f"sf_undamaged_{variant}.npz"), **out)


def main():
    os.makedirs(OUT, exist_ok=True)
    t_start = time.time()
    graph_arrays()
    scipy_pred_matrices(list(range(24)))
    summary = {}
    for variant, cls in [("crpow", CRPowEnv), ("native", RepairEnv)]:
        fixed_seed_resets(variant, cls)
        iteration_trace(variant, cls)
        random_seed_resets(variant, cls, list(range(32)))
        undamaged_anchors(variant, cls)
        g_msa = greedy_episode(variant, cls, "msa", 30)
        g_fw = greedy_episode(variant, cls, "fw", 30)
        summary[variant] = {
            "greedy_msa30_actions": g_msa["actions"].tolist(),
            "greedy_msa30_tstt": g_msa["tstt"].tolist(),
            "greedy_fw30_actions": g_fw["actions"].tolist(),
            "greedy_fw30_tstt": g_fw["tstt"].tolist(),
        }
    summary["generated_by"] = "tools/gen_golden.py (reference imported read-only from /root/reference)"
    import scipy, networkx
    summary["versions"] = {"numpy": np.__version__, "scipy": scipy.__version__, "networkx": networkx.__version__}
    with open(os.path.join(OUT, "sf_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(f"golden fixtures written in {time.time() - t_start:.1f}s")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Golden fixtures for the large-graph path on the
seeded synthetic Anaheim-sized network (416 nodes / 914 links / 38 zones,
trafficrl/data/AnaheimSynth/*.tntp), produced by running the REFERENCE env
read-only in this container -- the same procedure as tools/gen_golden.py
(which covers Sioux Falls), only the network differs.

Variant: ``crpow`` (host-independent float32 BPR power, see gen_golden.py).

Writes tests/golden/ana_*.npz:
  ana_graph.npz        graph arrays + OD dict order
  ana_resets_crpow.npz fixed_damage_seed=42 resets (msa30, fw30): damaged, flow,
                       t, tstt, unassigned; get_state tensors after the msa30 reset
  ana_steps_crpow.npz  3 random-seed envs (msa30): reset + 3 steps each (one of
                       them an already-repaired link), flows/tstt/rewards/dones,
                       observations after every step
  ana_scipy_pred.npz   scipy dijkstra predecessors from the 38 origins at
                       t = BPR(0) for 6 damage patterns + tie flags

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_large.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (reference import + CRPowEnv + ENV_KW)

OUT = G.OUT
DATA = os.path.join(HERE, "..", "sac-gat-her_transportationrl_amd", "trafficrl", "data", "AnaheimSynth")
NET = os.path.join(DATA, "AnaheimSynth_net.tntp")
TRIPS = os.path.join(DATA, "AnaheimSynth_trips.tntp")


def make_env(**kw):
    graph = G.load_graph_data(NET, TRIPS)
    args = dict(G.ENV_KW)
    args.update(kw)
    return G.CRPowEnv(graph, **args)


def graph_arrays():
    g = G.load_graph_data(NET, TRIPS)
    od = list(g.od_demand.items())
    np.savez_compressed(
        os.path.join(OUT, "ana_graph.npz"),
        num_nodes=np.int32(g.num_nodes),
        src=np.array([e.u - 1 for e in g.edges], np.int32), dst=np.array([e.v - 1 for e in g.edges], np.int32),
        cap0=np.array([e.capacity for e in g.edges], np.float32), t0=np.array([e.t0 for e in g.edges], np.float32),
        od_o=np.array([o - 1 for (o, _), _ in od], np.int32), od_d=np.array([d - 1 for (_, d), _ in od], np.int32),
        od_v=np.array([v for _, v in od], np.float64),
    )
    return g


def resets():
    out = {}
    for method, iters in [("msa", 30), ("fw", 30)]:
        t0 = time.time()
        env = make_env(assignment_method=method, assignment_iters=iters, fixed_damage=True,
                       fixed_damage_seed=42, seed=42)
        key = f"{method}{iters}"
        out[f"{key}_damaged"] = env.is_damaged.copy()
        out[f"{key}_flow"] = env.flow.copy()
        out[f"{key}_t"] = env.compute_travel_time(env.flow)
        out[f"{key}_tstt"] = np.float64(env.tstt)
        out[f"{key}_unassigned"] = np.float64(env.unassigned_demand)
        if key == "msa30":
            nx_, ex_, m_ = G.state_arrays(env.get_state())
            out["msa30_node_x"], out["msa30_edge_x"], out["msa30_mask"] = nx_, ex_, m_
        print(f"  reset {key}: {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(OUT, "ana_resets_crpow.npz"), **out)


def steps(seeds):
    E = 914
    S = len(seeds)
    rec = dict(damaged=np.zeros((S, E), np.float32), flow=np.zeros((S, E), np.float32), tstt=np.zeros(S),
               actions=np.zeros((S, 3), np.int32), step_flow=np.zeros((S, 3, E), np.float32),
               step_tstt=np.zeros((S, 3)), step_reward=np.zeros((S, 3)), step_done=np.zeros((S, 3), np.bool_),
               node_x=np.zeros((S, 3, 416, 4), np.float32), edge_x=np.zeros((S, 3, E, 6), np.float32))
    for i, s in enumerate(seeds):
        env = make_env(assignment_method="msa", assignment_iters=30, seed=s)
        rec["damaged"][i] = env.is_damaged
        rec["flow"][i] = env.flow
        rec["tstt"][i] = env.tstt
        rng = np.random.default_rng(7 + s)
        first = None
        for j in range(3):
            if j == 1:
                a = first  # already repaired: reward -1, no assignment (repair_env.py:210-212)
            else:
                a = int(rng.choice(np.where(env.is_damaged > 0)[0]))
                first = a if first is None else first
            st, r, d, info = env.step(a)
            rec["actions"][i, j] = a
            rec["step_flow"][i, j] = env.flow
            rec["step_tstt"][i, j] = info["tstt"]
            rec["step_reward"][i, j] = r
            rec["step_done"][i, j] = d
            nx_, ex_, _ = G.state_arrays(st)
            rec["node_x"][i, j] = nx_
            rec["edge_x"][i, j] = ex_
    rec["seeds"] = np.array(seeds, np.int32)
    np.savez_compressed(os.path.join(OUT, "ana_steps_crpow.npz"), **rec)


def scipy_preds(seeds):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    g = G.load_graph_data(NET, TRIPS)
    src = np.array([e.u - 1 for e in g.edges]); dst = np.array([e.v - 1 for e in g.edges])
    N, E = g.num_nodes, len(g.edges)
    origins = sorted({o - 1 for (o, _) in g.od_demand})
    preds, weights, ties = [], [], []
    for s in seeds:
        env = make_env(assignment_method="msa", assignment_iters=1, seed=s)
        t = env.compute_travel_time(np.zeros(E, np.float32))
        gr = csr_matrix((t.copy(), (src, dst)), shape=(N, N))
        d, p = dijkstra(gr, directed=True, indices=origins, return_predecessors=True)
        tie = np.zeros((len(origins), N), np.bool_)
        for oi in range(len(origins)):
            ach = d[oi, src] + t.astype(np.float64) == d[oi, dst]
            for v in range(N):
                tails = d[oi, src[ach & (dst == v)]]
                tie[oi, v] = len(tails) > 1 and np.sum(tails == tails.min()) > 1
        preds.append(p.astype(np.int32)); weights.append(t); ties.append(tie)
    np.savez_compressed(os.path.join(OUT, "ana_scipy_pred.npz"), seeds=np.array(seeds, np.int32),
                        origins=np.array(origins, np.int32), pred=np.array(preds), t=np.array(weights),
                        tie=np.array(ties))


def main():
    t0 = time.time()
    graph_arrays()
    scipy_preds(list(range(6)))
    resets()
    steps([0, 1, 2])
    print(f"large-graph fixtures written in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()

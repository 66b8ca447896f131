"""Seeded synthetic Anaheim-sized network.

The Anaheim TNTP files are not part of the reference checkout and there is no
network to fetch them, so config #5 ("Anaheim TNTP (416 nodes / 914 links),
1024 envs, FW assignment") runs on a deterministic stand-in of the same size:
416 nodes, 914 directed links (457 two-way streets), 38 origin/destination
zones (nodes 1..38, like Anaheim's centroids), integer OD demands.

Construction (numpy ``default_rng(seed)``, seed 416 by default):
  * node coordinates uniform in a 12 x 12 km square;
  * the Euclidean minimum spanning tree (Prim, 415 streets) plus the 42
    shortest remaining 4-nearest-neighbour pairs -> 457 streets, both
    directions -> a strongly connected road graph;
  * free-flow time = length / speed (speed 0.5, 0.8 or 1.2 km/min), rounded to
    1e-4 min and >= 0.01; capacity uniform in [800, 6000] veh/h, 2 decimals;
  * demand: each ordered zone pair (o != d) carries an integer demand in
    [1, 160) with probability 0.75 (Anaheim's total is ~1e5 trips; the
    framework's exact fp32 AON contract needs integral demands < 2^24 total).

``write_tntp`` emits the pair of TNTP files the reference's own parser
(src/data/tntp_parser.py:33-99) reads; the committed copies under
``data/AnaheimSynth/`` are what tests, fixtures and bench.py load, so the
reference (fixture generation) and this framework parse byte-identical input.
"""
from __future__ import annotations

import os

import numpy as np

from .tntp_parser import EdgeData, GraphData, load_graph_data

_HERE = os.path.dirname(os.path.abspath(__file__))
ANAHEIM_SYNTH_DIR = os.path.join(_HERE, "AnaheimSynth")


def _mst_prim(xy: np.ndarray) -> list:
    n = len(xy)
    d = np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1))
    in_tree = np.zeros(n, bool)
    in_tree[0] = True
    best = d[0].copy()
    parent = np.zeros(n, np.int64)
    best[0] = np.inf
    out = []
    for _ in range(n - 1):
        cand = np.where(in_tree, np.inf, best)
        v = int(np.argmin(cand))
        out.append((int(min(parent[v], v)), int(max(parent[v], v))))
        in_tree[v] = True
        upd = (d[v] < best) & ~in_tree
        best = np.where(upd, d[v], best)
        parent = np.where(upd, v, parent)
        best[v] = np.inf
    return out


def synthetic_network(num_nodes: int = 416, num_streets: int = 457, num_zones: int = 38,
                      seed: int = 416) -> GraphData:
    rng = np.random.default_rng(seed)
    xy = rng.uniform(0.0, 12.0, size=(num_nodes, 2))
    streets = set(_mst_prim(xy))
    d = np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1))
    np.fill_diagonal(d, np.inf)
    knn = np.argsort(d, axis=1)[:, :4]
    extra = sorted({(min(i, int(j)), max(i, int(j))) for i in range(num_nodes) for j in knn[i]} - streets,
                   key=lambda p: (d[p[0], p[1]], p))
    for p in extra[: num_streets - len(streets)]:
        streets.add(p)
    links = sorted([(u, v) for u, v in streets] + [(v, u) for u, v in streets])
    speeds = np.array([0.5, 0.8, 1.2])
    edges = []
    for u, v in links:
        length = round(float(d[u, v]), 4)
        t0 = max(round(length / float(speeds[rng.integers(0, 3)]), 4), 0.01)
        cap = round(float(rng.uniform(800.0, 6000.0)), 2)
        edges.append(EdgeData(u=u + 1, v=v + 1, capacity=cap, t0=t0, length=length, b=0.15, power=4.0))
    od = {}
    for o in range(1, num_zones + 1):
        for dd in range(1, num_zones + 1):
            if o != dd and rng.random() < 0.75:
                od[(o, dd)] = float(rng.integers(1, 160))
    return GraphData(num_nodes=num_nodes, edges=edges, od_demand=od)


def write_tntp(graph: GraphData, net_path: str, trips_path: str, num_zones: int) -> None:
    with open(net_path, "w") as fh:
        fh.write(f"<NUMBER OF ZONES> {num_zones}\n<NUMBER OF NODES> {graph.num_nodes}\n")
        fh.write(f"<FIRST THRU NODE> 1\n<NUMBER OF LINKS> {len(graph.edges)}\n")
        # the reference parser starts the link table at a non-'~' line naming
        # "init node" (tntp_parser.py:47-49), as SiouxFalls_net.tntp's header does
        fh.write("<ORIGINAL HEADER>~ \tInit node \tTerm node \tCapacity \tLength \tFree Flow Time \tB\tPower\t;\n")
        fh.write("<END OF METADATA>\n\n\n")
        fh.write("~\tinit_node\tterm_node\tcapacity\tlength\tfree_flow_time\tb\tpower\tspeed\ttoll\tlink_type\t;\n")
        for e in graph.edges:
            fh.write(f"\t{e.u}\t{e.v}\t{e.capacity:.2f}\t{e.length:.4f}\t{e.t0:.4f}\t0.15\t4\t0\t0\t1\t;\n")
    total = sum(graph.od_demand.values())
    with open(trips_path, "w") as fh:
        fh.write(f"<NUMBER OF ZONES> {num_zones}\n<TOTAL OD FLOW> {total:.1f}\n<END OF METADATA>\n\n\n")
        for o in range(1, num_zones + 1):
            fh.write(f"Origin \t{o} \n")
            row = [(dd, graph.od_demand.get((o, dd), 0.0)) for dd in range(1, num_zones + 1)]
            for i in range(0, len(row), 5):
                fh.write("".join(f"{dd:5d} : {v:8.1f}; " for dd, v in row[i:i + 5]) + "\n")
            fh.write("\n")


def anaheim_synthetic() -> GraphData:
    """The committed seed-416 network (416 nodes, 914 links, 38 zones)."""
    return load_graph_data(os.path.join(ANAHEIM_SYNTH_DIR, "AnaheimSynth_net.tntp"),
                           os.path.join(ANAHEIM_SYNTH_DIR, "AnaheimSynth_trips.tntp"))


if __name__ == "__main__":  # regenerate the committed files
    os.makedirs(ANAHEIM_SYNTH_DIR, exist_ok=True)
    g = synthetic_network()
    write_tntp(g, os.path.join(ANAHEIM_SYNTH_DIR, "AnaheimSynth_net.tntp"),
               os.path.join(ANAHEIM_SYNTH_DIR, "AnaheimSynth_trips.tntp"), 38)
    print(g.num_nodes, len(g.edges), len(g.od_demand), sum(g.od_demand.values()))

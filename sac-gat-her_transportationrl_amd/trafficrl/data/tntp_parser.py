"""TNTP network / trip-table reader with the reference's semantics
(src/data/tntp_parser.py:10-105).

* Links are kept in FILE order -- the edge ids every other array uses.
* Node count comes from the ``<NUMBER OF NODES>`` header.
* Per-link ``b``/``power`` are parsed but the env uses the global BPR alpha/beta
  (repair_env.py:27-28), like the reference.
* OD demands keep dict (file) order and only entries with demand > 0.
* ``<FIRST THRU NODE>`` is ignored, as in the reference.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from typing import Dict, List, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))


@dataclass
class EdgeData:
    u: int
    v: int
    capacity: float
    t0: float
    length: float
    b: float
    power: float


@dataclass
class GraphData:
    num_nodes: int
    edges: List[EdgeData]
    od_demand: Dict[Tuple[int, int], float]


def _lines(path: str):
    with open(path, "r", encoding="utf-8", errors="ignore") as fh:
        for raw in fh:
            line = raw.strip()
            if line and not line.startswith("~"):
                yield line


def parse_net_tntp(path: str) -> Tuple[int, List[EdgeData]]:
    num_nodes = 0
    edges: List[EdgeData] = []
    in_table = False
    for line in _lines(path):
        low = line.lower()
        if "number of nodes" in low:
            num_nodes = int(line.split(">")[-1] if ">" in line else line.split()[-1])
        if "init_node" in low or "init node" in low:
            in_table = True
            continue
        if not in_table:
            continue
        cols = line.replace(";", " ").split()
        if len(cols) < 6:
            continue
        u, v = int(cols[0]), int(cols[1])
        cap, length, t0 = float(cols[2]), float(cols[3]), float(cols[4])
        b = float(cols[5])
        power = float(cols[6]) if len(cols) > 6 else 4.0
        edges.append(EdgeData(u=u, v=v, capacity=cap, t0=t0, length=length, b=b, power=power))
    return num_nodes, edges


_PAIR = re.compile(r"(\d+)\s*:\s*([-+0-9.eE]+)")


def parse_trips_tntp(path: str) -> Dict[Tuple[int, int], float]:
    demand: Dict[Tuple[int, int], float] = {}
    origin = None
    for line in _lines(path):
        if line.lower().startswith("origin"):
            origin = int(line.split()[1])
            continue
        if origin is None:
            continue
        for part in line.split(";"):
            if ":" not in part:
                continue
            dest_s, val_s = part.split(":")
            val = float(val_s.strip())
            if val > 0:
                demand[(origin, int(dest_s.strip()))] = val
    return demand


def load_graph_data(net_path: str, trips_path: str) -> GraphData:
    n, edges = parse_net_tntp(net_path)
    return GraphData(num_nodes=n, edges=edges, od_demand=parse_trips_tntp(trips_path))


def sioux_falls() -> GraphData:
    """The Sioux Falls network shipped with this package (same files as the
    reference's data/SiouxFalls)."""
    d = os.path.join(_HERE, "SiouxFalls")
    return load_graph_data(os.path.join(d, "SiouxFalls_net.tntp"), os.path.join(d, "SiouxFalls_trips.tntp"))

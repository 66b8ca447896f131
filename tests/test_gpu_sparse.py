"""GPU parity of the sparse-relaxation env kernels -- the pair kernel
(csrc/assign_pair.hip, env_kernel_pair<NP, RS, FULL>, out-degree <= 8) and the
quad kernel (csrc/assign_sparse.hip, env_kernel_s<NP, R>, out-degree <= 16) --
on small random networks the Sioux Falls fixtures do not reach: every node
padding (NP 8/16/24/32), FULL graphs (N == NP, every node reachable) and
non-FULL ones (N < NP, a node no origin reaches), out-degrees above 4 and 8
(R = 2 and 4 out-slot rounds), parallel-free random digraphs with integer
free-flow times (many equal-length paths: the tie detection and the exact
scipy-heap replay), unreachable destinations, and all three methods.  Checker:
the C oracle (oracle/trx_oracle.c, scipy 1.15.3 Dijkstra restated),
bit-exact.  The quad kernel is also run on the pair kernel's cases with
TRX_KERNEL=sparse in a worker process (tests/sparse_worker.py)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def random_network(n, extra, zones, seed, one_way=0, source=False, max_deg=64):
    """Ring (strongly connected) + `extra` random directed links, integer t0;
    `source`: node 0 keeps no in-link (no other origin reaches it)."""
    from trafficrl.data.tntp_parser import EdgeData, GraphData
    rng = np.random.default_rng(seed)
    links = {(i, (i + 1) % n) for i in range(n)} | {((i + 1) % n, i) for i in range(n - one_way)}
    if source:
        links = {(u, v) for u, v in links if v != 0}
    deg = np.zeros(n, int)
    for u, _ in links:
        deg[u] += 1
    while len(links) < 2 * n + extra - (2 if source else 0):
        u, v = (int(x) for x in rng.integers(0, n, 2))
        if u != v and not (source and v == 0) and (u, v) not in links and deg[u] < max_deg:
            links.add((u, v))
            deg[u] += 1
    edges = [EdgeData(u=u + 1, v=v + 1, capacity=float(rng.integers(200, 4000)), t0=float(rng.integers(1, 6)),
                      length=1.0, b=0.15, power=4.0) for u, v in sorted(links)]
    od = {}
    for o in range(1, zones + 1):
        for d in range(1, n + 1):
            if o != d and rng.random() < 0.7:
                od[(o, d)] = float(rng.integers(1, 300))
    return GraphData(num_nodes=n, edges=edges, od_demand=od)


CASES = [  # (nodes, extra links, zones, seed, one-way ring links, source node, max out-degree, kernel)
    (7, 6, 5, 1, 0, False, 64, "env_kernel_pair"),      # NP 8, N < NP
    (13, 40, 9, 2, 0, False, 8, "env_kernel_pair"),     # NP 16, out-degree > 4
    (16, 110, 12, 3, 0, False, 64, "env_kernel_s"),     # NP 16, out-degree > 8 (R = 4)
    (22, 30, 22, 4, 3, False, 64, "env_kernel_pair"),   # NP 24
    (31, 90, 14, 5, 0, False, 64, "env_kernel_s"),      # NP 32, out-degree > 8
    (8, 10, 8, 6, 0, False, 8, "env_kernel_pair"),      # NP 8 FULL
    (16, 40, 16, 7, 0, False, 8, "env_kernel_pair"),    # NP 16 FULL
    (24, 45, 20, 8, 0, False, 7, "env_kernel_pair"),    # NP 24 FULL, odd max out-degree
    (32, 60, 12, 9, 0, False, 8, "env_kernel_pair"),    # NP 32 FULL
    (24, 30, 18, 10, 0, True, 8, "env_kernel_pair"),    # NP 24, node 0 unreachable (not FULL)
    (15, 8, 9, 11, 2, False, 3, "env_kernel_pair"),     # NP 16, out-degree <= 3 (RS = 2)
    (16, 0, 10, 12, 0, False, 2, "env_kernel_pair"),    # NP 16 FULL, the bare ring: out-degree 2 (RS = 1)
]
IDS = [f"n{c[0]}s{c[3]}" for c in CASES]


def env_penalty():
    """VecRepairEnv's unassigned_penalty default (the oracle's own default is 1e4)."""
    import inspect
    from trafficrl.env import VecRepairEnv
    return inspect.signature(VecRepairEnv).parameters["unassigned_penalty"].default


def case_network(case):
    n, extra, zones, seed, one_way, source, max_deg, _ = case
    return random_network(n, extra, zones, seed, one_way, source, max_deg)


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("method", ["msa", "fw", "cfw"])
def test_sparse_kernel_vs_oracle(case, method):
    from trafficrl.env import VecRepairEnv
    from trafficrl.graph import TrafficGraph
    n, zones, seed, kname = case[0], case[2], case[3], case[7]
    gd = case_network(case)
    tg = TrafficGraph(gd)
    og = O.OracleGraph(n, tg.src, tg.dst, tg.t0, tg.cap0, tg.od_o, tg.od_d, tg.od_v)
    E = tg.num_edges
    # the sparse kernel's preconditions (capi.hip sparse_ok -> packed_ok), so that it is the one tested
    _, ex = np.frexp(float(tg.t0.min()))
    bound = (n - 1) * max(1e6, float(tg.t0.max()) * (1 + 0.15 * 10.0 ** 4)) * 1.0001
    assert bound < np.ldexp(1.0, int(ex) - 1 - 23 + 48) and E <= 255 and n <= 32
    rng = np.random.default_rng(100 + seed)
    B = 96
    dmg = (rng.random((B, E)) < 0.25).astype(np.float32)
    cap = np.where(dmg > 0, np.float32(1e-3), tg.cap0).astype(np.float32)
    flow0 = np.zeros((B, E), np.float32)
    flow0[B // 2:] = (rng.random((B - B // 2, E)) * 3000).astype(np.float32)   # half cold (ties), half warm
    iters = 8
    f_o, t_o, ts_o, un_o = og.assign(cap, dmg, flow0, method=method, iters=iters, nthreads=8,
                                     penalty=env_penalty())
    env = VecRepairEnv(gd, B, device="cuda", assignment_method=method, assignment_iters=iters, graph=tg, reset=False)
    assert env.kernel_name == kname, (env.kernel_name, kname)
    env.capacity.copy_(torch.from_numpy(cap))
    env.damaged.copy_(torch.from_numpy(dmg))
    env.flow.copy_(torch.from_numpy(flow0))
    env.assign()
    np.testing.assert_array_equal(env.flow.cpu().numpy(), f_o)
    np.testing.assert_array_equal(env.t.cpu().numpy(), t_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), ts_o)


def test_quad_sparse_kernel_on_pair_cases():
    """TRX_KERNEL=sparse: the quad-per-tree kernel env_kernel_s on the cases the
    pair kernel takes by default, and on the Sioux Falls reference fixtures."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TRX_KERNEL="sparse")
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "quad_worker.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sparse worker ok" in r.stdout

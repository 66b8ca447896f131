"""GPU parity of the sparse-relaxation env kernel (csrc/assign_sparse.hip,
env_kernel_s<NP, R>) on small random networks the Sioux Falls fixtures do not
reach: every node padding (NP 8/16/24/32), out-degrees above 4 and 8 (R = 2
and 4 out-slot rounds), parallel-free random digraphs with integer free-flow
times (many equal-length paths: the tie detection and the exact scipy-heap
replay), unreachable destinations, and all three methods.  Checker: the C
oracle (oracle/trx_oracle.c, scipy 1.15.3 Dijkstra restated), bit-exact.
The packed kernel (TRX_KERNEL=packed in another process) is not needed here:
both are pinned to the same oracle."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def random_network(n, extra, zones, seed, one_way=0):
    """Ring (strongly connected) + `extra` random directed links, integer t0."""
    from trafficrl.data.tntp_parser import EdgeData, GraphData
    rng = np.random.default_rng(seed)
    links = {(i, (i + 1) % n) for i in range(n)} | {((i + 1) % n, i) for i in range(n - one_way)}
    while len(links) < 2 * n + extra:
        u, v = (int(x) for x in rng.integers(0, n, 2))
        if u != v:
            links.add((u, v))
    edges = [EdgeData(u=u + 1, v=v + 1, capacity=float(rng.integers(200, 4000)), t0=float(rng.integers(1, 6)),
                      length=1.0, b=0.15, power=4.0) for u, v in sorted(links)]
    od = {}
    for o in range(1, zones + 1):
        for d in range(1, n + 1):
            if o != d and rng.random() < 0.7:
                od[(o, d)] = float(rng.integers(1, 300))
    return GraphData(num_nodes=n, edges=edges, od_demand=od)


CASES = [  # (nodes, extra links, zones, seed, one-way ring links)
    (7, 6, 5, 1, 0),      # NP 8
    (13, 40, 9, 2, 0),    # NP 16, out-degree > 4
    (16, 110, 12, 3, 0),  # NP 16, out-degree > 8 (R = 4)
    (22, 30, 22, 4, 3),   # NP 24
    (31, 90, 14, 5, 0),   # NP 32
]


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}" for c in CASES])
@pytest.mark.parametrize("method", ["msa", "fw", "cfw"])
def test_sparse_kernel_vs_oracle(case, method):
    from trafficrl.env import VecRepairEnv
    from trafficrl.graph import TrafficGraph
    n, extra, zones, seed, one_way = case
    gd = random_network(n, extra, zones, seed, one_way)
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
    f_o, t_o, ts_o, un_o = og.assign(cap, dmg, flow0, method=method, iters=iters, nthreads=8)
    env = VecRepairEnv(gd, B, device="cuda", assignment_method=method, assignment_iters=iters, graph=tg, reset=False)
    env.capacity.copy_(torch.from_numpy(cap))
    env.damaged.copy_(torch.from_numpy(dmg))
    env.flow.copy_(torch.from_numpy(flow0))
    env.assign()
    np.testing.assert_array_equal(env.flow.cpu().numpy(), f_o)
    np.testing.assert_array_equal(env.t.cpu().numpy(), t_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), ts_o)

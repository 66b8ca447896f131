"""GPU parity of the general small-graph env kernel (csrc/assign_quad.hip,
env_kernel_q) on the graphs the dispatcher (csrc/capi.hip select_env_kernel)
routes to it: networks outside the sparse kernel's preconditions (out-degree
> 16, no exact-label headroom, more than 255 links) and, for the torch rule,
outside env_kernel_t's budget (E > 255).  trx_env_kernel_name pins which
kernel runs.  Checker: the C oracle (oracle/trx_oracle.c: scipy 1.15.3
Dijkstra incl. its Fibonacci-heap tie order, or the torch rule's fp32
Floyd-Warshall + next-hop walk), bit-exact: reset (cold start) and
warm-started assignments for msa / fw / cfw.  Plus the Sioux Falls reference
fixtures with the quad kernel forced (TRX_KERNEL=quad, in a subprocess)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import oracle as O
from test_gpu_sparse import random_network

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def hub_network(n, seed):
    """Ring + a hub (node 0) with links to and from every other node: out-degree
    n - 1 > 16 (sparse_ok fails on the degree), integer t0 (many ties)."""
    from trafficrl.data.tntp_parser import EdgeData, GraphData
    rng = np.random.default_rng(seed)
    links = {(i, (i + 1) % n) for i in range(n)} | {((i + 1) % n, i) for i in range(n)}
    links |= {(0, v) for v in range(1, n)} | {(v, 0) for v in range(1, n)}
    edges = [EdgeData(u=u + 1, v=v + 1, capacity=float(rng.integers(200, 4000)), t0=float(rng.integers(1, 6)),
                      length=1.0, b=0.15, power=4.0) for u, v in sorted(links)]
    od = {(o, d): float(rng.integers(1, 300)) for o in range(1, n + 1) for d in range(1, n + 1)
          if o != d and rng.random() < 0.5}
    return GraphData(num_nodes=n, edges=edges, od_demand=od)


def wide_t0_network(n, seed):
    """Random network whose free-flow times span 1e-3 .. 1e4 (float32, not
    integral): the exact-label headroom check fails, so labels cannot carry
    node ids in their low mantissa bits."""
    gd = random_network(n, 20, n - 4, seed)
    rng = np.random.default_rng(seed + 7)
    for e in gd.edges:
        e.t0 = float(np.float32(10.0 ** rng.uniform(-3, 4)))
    return gd


def dense_network(n, links, seed):
    """More than 255 links on N <= 32 (u8 link ids of env_kernel_s / env_kernel_t do not fit)."""
    return random_network(n, links - 2 * n, n - 8, seed)


CASES = [  # (id, builder, sp rules)
    ("hub24", lambda: hub_network(24, 11), ("scipy",)),
    ("widet0_20", lambda: wide_t0_network(20, 12), ("scipy",)),
    ("dense32", lambda: dense_network(32, 300, 13), ("scipy", "torch")),
]


def _run_case(gd, sp, method):
    from trafficrl.env import VecRepairEnv
    from trafficrl.graph import TrafficGraph
    tg = TrafficGraph(gd)
    n = gd.num_nodes
    og = O.OracleGraph(n, tg.src, tg.dst, tg.t0, tg.cap0, tg.od_o, tg.od_d, tg.od_v)
    E = tg.num_edges
    B, iters = 64, 6
    env = VecRepairEnv(gd, B, device="cuda", assignment_method=method, assignment_iters=iters, graph=tg,
                       reset=False, sp_backend=sp)
    assert env.kernel_name == "env_kernel_q", env.kernel_name
    rng = np.random.default_rng(E + iters)
    dmg = (rng.random((B, E)) < 0.2).astype(np.float32)
    cap = np.where(dmg > 0, np.float32(1e-3), tg.cap0).astype(np.float32)
    # reset: cold start (capacity from the damage mask, flow 0)
    env.reset(damaged=torch.from_numpy(dmg), observe=False)
    f_o, t_o, ts_o, un_o = og.assign(cap, dmg, np.zeros((B, E), np.float32), method=method, iters=iters,
                                     nthreads=8, sp=sp)
    np.testing.assert_array_equal(env.flow.cpu().numpy(), f_o)
    np.testing.assert_array_equal(env.t.cpu().numpy(), t_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), ts_o)
    np.testing.assert_array_equal(env.unassigned.cpu().numpy(), un_o)
    # warm start from random flows (non-integer costs)
    flow0 = (rng.random((B, E)) * 3000).astype(np.float32)
    env.flow.copy_(torch.from_numpy(flow0))
    env.assign()
    f_o, t_o, ts_o, _ = og.assign(cap, dmg, flow0, method=method, iters=iters, nthreads=8, sp=sp)
    np.testing.assert_array_equal(env.flow.cpu().numpy(), f_o)
    np.testing.assert_array_equal(env.t.cpu().numpy(), t_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), ts_o)


@pytest.mark.parametrize("method", ["msa", "fw", "cfw"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_quad_fallback_vs_oracle(case, method):
    _, build, rules = case
    gd = build()
    for sp in rules:
        _run_case(gd, sp, method)


def test_kernel_selection():
    """Sioux Falls takes the specialised kernels; each fallback case the quad kernel."""
    from trafficrl.data import sioux_falls
    from trafficrl.env import VecRepairEnv
    sf = sioux_falls()
    assert VecRepairEnv(sf, 2, device="cuda", reset=False, sp_backend="scipy").kernel_name == "env_kernel_pair"
    assert VecRepairEnv(sf, 2, device="cuda", reset=False, sp_backend="torch").kernel_name == "env_kernel_t"
    assert VecRepairEnv(sf, 2, device="cuda", reset=False, assignment_method="gp").kernel_name == "gp_kernel"
    for _, build, rules in CASES:
        for sp in rules:
            assert VecRepairEnv(build(), 2, device="cuda", reset=False, sp_backend=sp).kernel_name == "env_kernel_q"


def test_forced_quad_on_sf_fixtures():
    """TRX_KERNEL=quad: the Sioux Falls reference fixtures (both rules) through env_kernel_q."""
    env = dict(os.environ, TRX_KERNEL="quad")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "quad_worker.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "quad worker ok" in r.stdout

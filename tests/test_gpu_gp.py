"""GPU parity of the path-based (GP) assignment, RepairEnv(assignment_method=
"gp") (src/env/repair_env.py:351-419), gp_kernel.hip via the C ABI.

Bar: link flows, travel times, TSTT, rewards, dones BIT-EXACT vs the
reference's own outputs (tests/golden/sf_gp_crpow.npz, tools/gen_golden_gp.py)
-- including fractional path flows (gp_step 0.5 and 1/(it+1)), whose float32
link loading is order-dependent -- and the decoded path sets equal to the
oracle's (oracle.gp_assign).
"""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu

CASES = {"s1k2i30": (1.0, 2, 30), "s1k3i10": (1.0, 3, 10), "s0k3i10": (0.0, 3, 10), "s05k2i8": (0.5, 2, 8)}


@pytest.fixture(scope="module")
def gd():
    from trafficrl.data import sioux_falls
    return sioux_falls()


@pytest.fixture(scope="module")
def tgraph(gd):
    from trafficrl.graph import TrafficGraph
    return TrafficGraph(gd)


def make_vec(gd, tg, B, step, keep, iters):
    from trafficrl.env import VecRepairEnv
    return VecRepairEnv(gd, B, device="cuda", assignment_method="gp", assignment_iters=iters, gp_step=step,
                        gp_keep_paths=keep, reward_mode="rel_improve", reward_beta=0.0, reward_gamma=0.0,
                        reward_clip=2.0, unassigned_penalty=1e4, graph=tg, reset=False)


@pytest.mark.parametrize("tag", sorted(CASES))
def test_gp_reset_seed42_bitexact(gd, tgraph, tag):
    step, keep, iters = CASES[tag]
    z = np.load(golden("sf_gp_crpow.npz"))
    env = make_vec(gd, tgraph, 3, step, keep, iters)
    env.reset(damaged=torch.from_numpy(np.repeat(z[f"reset_{tag}_damaged"][None], 3, 0)), observe=False)
    for b in range(3):
        np.testing.assert_array_equal(env.flow[b].cpu().numpy(), z[f"reset_{tag}_flow"])
        np.testing.assert_array_equal(env.t[b].cpu().numpy(), z[f"reset_{tag}_t"])
        assert float(env.tstt[b]) == float(z[f"reset_{tag}_tstt"])


@pytest.mark.parametrize("tag", sorted(CASES))
def test_gp_steps_carry_path_sets_bitexact(gd, tgraph, tag):
    step, keep, iters = CASES[tag]
    z = np.load(golden("sf_gp_crpow.npz"))
    dm = z[f"steps_{tag}_damaged"]
    env = make_vec(gd, tgraph, len(dm), step, keep, iters)
    env.reset(damaged=torch.from_numpy(dm), observe=False)
    np.testing.assert_array_equal(env.flow.cpu().numpy(), z[f"steps_{tag}_flow"])
    for j in range(3):
        _, rew, done, _ = env.step(torch.from_numpy(z[f"steps_{tag}_actions"][:, j]), observe=False)
        np.testing.assert_array_equal(env.flow.cpu().numpy(), z[f"steps_{tag}_step_flow"][:, j])
        np.testing.assert_array_equal(env.tstt.cpu().numpy(), z[f"steps_{tag}_step_tstt"][:, j])
        np.testing.assert_array_equal(rew.cpu().numpy(), z[f"steps_{tag}_step_reward"][:, j])
        np.testing.assert_array_equal(done.cpu().numpy(), z[f"steps_{tag}_step_done"][:, j])


def test_gp_path_sets_match_oracle(gd, tgraph, oracle_graph):
    """Decoded device path sets (keys in insertion order, paths, float64 flows)
    == the oracle's after a fractional-step reset and one step."""
    step, keep, iters = 0.5, 2, 8
    og = oracle_graph
    z = np.load(golden("sf_gp_crpow.npz"))
    d = z["steps_s05k2i8_damaged"][1].copy()
    env = make_vec(gd, tgraph, 2, step, keep, iters)
    env.reset(damaged=torch.from_numpy(np.repeat(d[None], 2, 0)), observe=False)
    st = O.GPPaths()
    cap = np.where(d > 0, np.float32(1e-3), og.cap0).astype(np.float32)
    f, _, _, _ = O.gp_assign(og, cap, d, np.zeros(og.E, np.float32), st, iters, step, keep, reset=True)
    a = int(np.where(d > 0)[0][3])
    env.step(torch.tensor([a, a], dtype=torch.int32), observe=False)
    d[a] = 0.0
    cap[a] = og.cap0[a]
    f, _, _, _ = O.gp_assign(og, cap, d, f, st, iters, step, keep)
    paths, flows = env.gp_paths(1)
    want_p = {(o + 1, dd + 1): v for (o, dd), v in st.paths.items()}
    want_f = {(o + 1, dd + 1): v for (o, dd), v in st.flows.items()}
    assert list(paths) == list(want_p)
    assert paths == want_p
    assert flows == want_f
    np.testing.assert_array_equal(env.flow[1].cpu().numpy(), f)


def test_gp_facade_greedy_and_path_roundtrip(gd):
    """RepairEnv(assignment_method='gp') facade: od_paths decode/restore round
    trip and the batched greedy what-if (every candidate starts from the same
    path sets) picks the oracle's action."""
    from trafficrl.baselines import select_greedy_one_step
    from trafficrl.env import RepairEnv
    og = O.OracleGraph.from_npz(golden("sf_graph.npz"))
    env = RepairEnv(gd, assignment_iters=6, assignment_method="gp", gp_step=1.0, gp_keep_paths=2,
                    fixed_damage=True, fixed_damage_seed=42, seed=42, reward_mode="rel_improve",
                    unassigned_penalty=1e4)
    paths, flows = env.od_paths, env.od_path_flows
    assert len(paths) == 528 and all(len(v) <= 2 for v in paths.values())
    env.od_paths, env.od_path_flows = dict(paths), dict(flows)  # restore path (baselines 64-65)
    state = env.get_state()
    a = select_greedy_one_step(env, state)
    st0 = O.GPPaths()
    d = env.is_damaged.copy()
    cap = env.capacities.copy()
    st0.paths = {(o - 1, dd - 1): list(v) for (o, dd), v in paths.items()}
    st0.flows = {(o - 1, dd - 1): list(v) for (o, dd), v in flows.items()}
    best, best_ts = None, float("inf")
    for c in np.where(d > 0)[0]:
        dc, cc = d.copy(), cap.copy()
        dc[c], cc[c] = 0.0, og.cap0[c]
        _, _, ts, _ = O.gp_assign(og, cc, dc, env.flow.copy(), st0.copy(), 6, 1.0, 2)
        if ts < best_ts:
            best, best_ts = int(c), ts
    assert a == best

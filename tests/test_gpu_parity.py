"""GPU parity: the gfx950 kernels (through the C ABI) vs the reference's own
outputs (tests/golden, 'crpow' = host-independent BPR power) and vs the CPU
oracle on seeded inputs.

Bar: link flows, travel times, TSTT, rewards and greedy actions BIT-EXACT
(integer-exact AON + identically rounded fp32 updates + scipy tie order).
Observation features: node betweenness bit-exact, log-based features within
4 ulp (numpy's float32 log10/log1p are SVML on the reference host).
"""
import json

import numpy as np
import pytest
import torch

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu

KEYS = ["msa30", "fw30", "msa60", "fw50", "msa1", "fw2", "cfw60"]


def split_key(k):
    m = k.rstrip("0123456789")
    return m, int(k[len(m):])


@pytest.fixture(scope="module")
def gd():
    from trafficrl.data import sioux_falls
    return sioux_falls()


@pytest.fixture(scope="module")
def tgraph(gd):
    from trafficrl.graph import TrafficGraph
    return TrafficGraph(gd)


def make_vec(gd, tgraph, B, method="msa", iters=30, **kw):
    from trafficrl.env import VecRepairEnv
    kw.setdefault("reward_mode", "rel_improve")
    kw.setdefault("reward_beta", 0.0)
    kw.setdefault("reward_gamma", 0.0)
    kw.setdefault("reward_clip", 2.0)
    kw.setdefault("unassigned_penalty", 1e4)
    return VecRepairEnv(gd, B, device="cuda", assignment_method=method, assignment_iters=iters, graph=tgraph,
                        reset=False, **kw)


@pytest.mark.parametrize("key", KEYS)
def test_reset_seed42_bitexact(gd, tgraph, key):
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    m, k = split_key(key)
    env = make_vec(gd, tgraph, 3, m, k)
    dmg = torch.from_numpy(np.repeat(r[key + "_damaged"][None], 3, 0))
    env.reset(damaged=dmg, observe=False)
    torch.cuda.synchronize()
    flow = env.flow.cpu().numpy()
    t = env.t.cpu().numpy()
    tstt = env.tstt.cpu().numpy()
    if m == "cfw":  # reference dot = BLAS sdot: compare to the oracle (same fp64 order) instead
        gr = np.load(golden("sf_graph.npz"))
        cap = np.where(r[key + "_damaged"] > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)
        og = O.OracleGraph.from_npz(golden("sf_graph.npz"))
        f_o, t_o, ts_o, _ = og.assign(cap, r[key + "_damaged"], np.zeros(76, np.float32), method="cfw", iters=k)
        for b in range(3):
            np.testing.assert_array_equal(flow[b], f_o)
            assert tstt[b] == ts_o
        assert abs(tstt[0] - float(r[key + "_tstt"])) <= 1e-6 * float(r[key + "_tstt"])
        return
    for b in range(3):
        np.testing.assert_array_equal(flow[b], r[key + "_flow"])
        np.testing.assert_array_equal(t[b], r[key + "_t"])
        assert tstt[b] == float(r[key + "_tstt"])
    np.testing.assert_array_equal(env.initial_tstt.cpu().numpy(), tstt)


def test_random_resets_and_steps_bitexact(gd, tgraph):
    """32 RNG damage patterns (ties at reset exercise the exact scipy-heap
    replay) + 4 steps each, including an already-repaired action."""
    z = np.load(golden("sf_random_resets_crpow.npz"))
    B = len(z["seeds"])
    env = make_vec(gd, tgraph, B)
    env.reset(damaged=torch.from_numpy(z["damaged"]), observe=False)
    np.testing.assert_array_equal(env.flow.cpu().numpy(), z["flow"])
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), z["tstt"])
    for j in range(4):
        _, rew, done, info = env.step(torch.from_numpy(z["step_actions"][:, j]), observe=False)
        np.testing.assert_array_equal(env.flow.cpu().numpy(), z["step_flow"][:, j])
        np.testing.assert_array_equal(env.tstt.cpu().numpy(), z["step_tstt"][:, j])
        np.testing.assert_array_equal(rew.cpu().numpy(), z["step_reward"][:, j])
        np.testing.assert_array_equal(done.cpu().numpy(), z["step_done"][:, j])


def test_tied_resets_match_scipy_heap_order(gd, tgraph):
    """Damage seeds whose reset has tied shortest paths: flows must follow
    scipy's Fibonacci-heap predecessor choice (oracle), not index order."""
    zp = np.load(golden("sf_scipy_pred.npz"))
    assert zp["tie"].sum() > 0
    og = O.OracleGraph.from_npz(golden("sf_graph.npz"))
    gr = np.load(golden("sf_graph.npz"))
    rng = np.random.default_rng(11)
    B = 256
    dmg = np.zeros((B, 76), np.float32)
    for b in range(B):
        dmg[b, rng.choice(76, 22, replace=False)] = 1.0
    cap = np.where(dmg > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)
    f_o, t_o, ts_o, un_o = og.assign(cap, dmg, np.zeros((B, 76), np.float32), iters=5, nthreads=8)
    env = make_vec(gd, tgraph, B, "msa", 5)
    env.reset(damaged=torch.from_numpy(dmg), observe=False)
    np.testing.assert_array_equal(env.flow.cpu().numpy(), f_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), ts_o)
    np.testing.assert_array_equal(env.unassigned.cpu().numpy(), un_o)


@pytest.mark.parametrize("method", ["msa", "fw", "cfw"])
def test_warm_start_assign_vs_oracle(gd, tgraph, method):
    """Random warm-start flows/damage (non-integer costs), B=512."""
    og = O.OracleGraph.from_npz(golden("sf_graph.npz"))
    gr = np.load(golden("sf_graph.npz"))
    rng = np.random.default_rng(5)
    B = 512
    dmg = (rng.random((B, 76)) < 0.2).astype(np.float32)
    cap = np.where(dmg > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)
    flow0 = (rng.random((B, 76)) * 20000).astype(np.float32)
    f_o, t_o, ts_o, _ = og.assign(cap, dmg, flow0, method=method, iters=12, nthreads=8)
    env = make_vec(gd, tgraph, B, method, 12)
    env.capacity.copy_(torch.from_numpy(cap))
    env.damaged.copy_(torch.from_numpy(dmg))
    env.flow.copy_(torch.from_numpy(flow0))
    env.assign()
    np.testing.assert_array_equal(env.flow.cpu().numpy(), f_o)
    np.testing.assert_array_equal(env.t.cpu().numpy(), t_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), ts_o)


def test_env_mask_leaves_other_envs_untouched(gd, tgraph):
    env = make_vec(gd, tgraph, 16)
    z = np.load(golden("sf_random_resets_crpow.npz"))
    env.reset(damaged=torch.from_numpy(z["damaged"][:16]), observe=False)
    before = env.flow.clone()
    mask = torch.zeros(16, dtype=torch.uint8, device="cuda")
    mask[3] = 1
    env.flow[3].zero_()
    env.assign(mask)
    keep = torch.ones(16, dtype=torch.bool)
    keep[3] = False
    assert torch.equal(env.flow[keep.cuda()], before[keep.cuda()])


@pytest.mark.parametrize("method,iters", [("msa", 30), ("fw", 30), ("msa", 60)])
def test_greedy_episode_bitexact(method, iters):
    """Config #1: greedy one-step episode through the drop-in RepairEnv facade
    + batched what-if; actions and TSTT curve == reference golden (K = 60 is
    configs/sioux_falls.yaml's assignment_iters)."""
    from trafficrl.baselines import run_episode, select_greedy_one_step
    from trafficrl.data import sioux_falls
    from trafficrl.env import RepairEnv
    z = np.load(golden(f"sf_greedy_{method}{iters}_crpow.npz"))
    env = RepairEnv(sioux_falls(), assignment_iters=iters, assignment_method=method, fixed_damage=True,
                    fixed_damage_seed=42, seed=42, reward_mode="rel_improve", reward_alpha=1.0, reward_beta=0.0,
                    reward_gamma=0.0, reward_clip=2.0, unassigned_penalty=1e4)
    assert env.initial_tstt == float(z["initial_tstt"])
    np.testing.assert_array_equal(env.flow, z["reset_flow"])
    actions = []

    def pol(s):
        a = select_greedy_one_step(env, s)
        actions.append(a)
        return a

    out = run_episode(env, pol)
    assert actions == z["actions"].tolist()
    np.testing.assert_array_equal(np.array(out["tstt_curve"]), z["tstt"])


def test_greedy_first_decision_candidate_tstts(gd, tgraph):
    from trafficrl.baselines import greedy_actions
    z = np.load(golden("sf_greedy_msa30_crpow.npz"))
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    env = make_vec(gd, tgraph, 4)
    env.reset(damaged=torch.from_numpy(np.repeat(r["msa30_damaged"][None], 4, 0)), observe=False)
    a = greedy_actions(env)
    assert a.tolist() == [int(z["actions"][0])] * 4


def test_observation_vs_reference(gd, tgraph):
    """get_state features on the greedy trajectory vs the reference's
    (native fixtures: numpy SVML log10/log1p -> ulp tolerance)."""
    z = np.load(golden("sf_greedy_msa30_native.npz"))
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    env = make_vec(gd, tgraph, 1)
    env.reset(damaged=torch.from_numpy(r["msa30_damaged"][None]), observe=False)
    obs = env.observe()
    nx_ = obs.node_x[0].cpu().numpy()
    ex_ = obs.edge_x[0].cpu().numpy()
    np.testing.assert_array_equal(nx_[:, 0], z["reset_node_x"][:, 0])
    np.testing.assert_allclose(nx_, z["reset_node_x"], rtol=4e-7, atol=0)
    np.testing.assert_allclose(ex_, z["reset_edge_x"], rtol=5e-7, atol=1e-7)
    for j, a in enumerate(z["actions"][:6]):
        obs, *_ = env.step(torch.tensor([int(a)]))
        np.testing.assert_array_equal(obs.node_x[0, :, 0].cpu().numpy(), z["node_x"][j][:, 0])
        np.testing.assert_allclose(obs.node_x[0].cpu().numpy(), z["node_x"][j], rtol=4e-7, atol=0)
        np.testing.assert_allclose(obs.edge_x[0].cpu().numpy(), z["edge_x"][j], rtol=5e-7, atol=1e-7)
        np.testing.assert_array_equal(obs.action_mask[0].cpu().numpy(), z["mask"][j])


def test_facade_errors_and_invalid_action():
    from trafficrl.data import sioux_falls
    from trafficrl.env import RepairEnv
    env = RepairEnv(sioux_falls(), assignment_iters=5, fixed_damage=True, fixed_damage_seed=42, seed=42)
    with pytest.raises(ValueError):
        env.step(76)
    with pytest.raises(ValueError):
        env.step(-1)
    repaired = int(np.where(env.is_damaged == 0)[0][0])
    tstt = env.tstt
    _, r, d, info = env.step(repaired)
    assert r == -1.0 and d is False and info["tstt"] == tstt


def test_big_batch_properties(gd, tgraph):
    """At the benchmark size (B=4096): replicated envs give identical rows,
    two runs are bit-identical, flows finite/non-negative, sampled rows ==
    oracle."""
    B = 4096
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    env = make_vec(gd, tgraph, B)
    dmg = torch.from_numpy(np.repeat(r["msa30_damaged"][None], B, 0))
    env.reset(damaged=dmg, observe=False)
    f1 = env.flow.clone()
    assert torch.equal(f1, f1[:1].expand_as(f1))
    np.testing.assert_array_equal(f1[0].cpu().numpy(), r["msa30_flow"])
    gen = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(3):
        scores = torch.rand(B, 76, device="cuda", generator=gen) * env.damaged
        env.step(scores.argmax(1).to(torch.int32), observe=False)
    fa, ta = env.flow.clone(), env.tstt.clone()
    assert torch.isfinite(fa).all() and (fa >= 0).all()
    # replay the same trajectory: bit-identical
    env.reset(damaged=dmg, observe=False)
    gen = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(3):
        scores = torch.rand(B, 76, device="cuda", generator=gen) * env.damaged
        env.step(scores.argmax(1).to(torch.int32), observe=False)
    assert torch.equal(fa, env.flow) and torch.equal(ta, env.tstt)
    # sample rows against the oracle (one warm-start assign)
    og = O.OracleGraph.from_npz(golden("sf_graph.npz"))
    rows = np.random.default_rng(0).choice(B, 48, replace=False)
    cap = env.capacity.cpu().numpy()[rows]
    dm = env.damaged.cpu().numpy()[rows]
    fl = env.flow.cpu().numpy()[rows]
    f_o, _, ts_o, _ = og.assign(cap, dm, fl, iters=30, nthreads=8)
    env.assign()
    np.testing.assert_array_equal(env.flow.cpu().numpy()[rows], f_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy()[rows], ts_o)


def test_big_batch_fw30_vs_oracle(gd, tgraph):
    """Config #3's env path at its size: B = 4096 FW-30 envs (random damage,
    tie-heavy resets), reset + 3 random repairs; sampled rows == the oracle."""
    og = O.OracleGraph.from_npz(golden("sf_graph.npz"))
    gr = np.load(golden("sf_graph.npz"))
    rng = np.random.default_rng(23)
    B = 4096
    dmg = np.zeros((B, 76), np.float32)
    for b in range(B):
        dmg[b, rng.choice(76, 22, replace=False)] = 1.0
    env = make_vec(gd, tgraph, B, "fw", 30)
    env.reset(damaged=torch.from_numpy(dmg), observe=False)
    rows = rng.choice(B, 48, replace=False)
    cap = np.where(dmg > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)
    f_o, _, ts_o, _ = og.assign(cap[rows], dmg[rows], np.zeros((48, 76), np.float32), method="fw", iters=30,
                                nthreads=8)
    np.testing.assert_array_equal(env.flow.cpu().numpy()[rows], f_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy()[rows], ts_o)
    gen = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(3):
        cap_b, dm_b, fl_b = env.capacity.cpu().numpy(), env.damaged.cpu().numpy(), env.flow.cpu().numpy()
        a = (torch.rand(B, 76, device="cuda", generator=gen) * env.damaged).argmax(1).to(torch.int32)
        env.step(a, observe=False)
        an = a.cpu().numpy()[rows]
        C, D = cap_b[rows].copy(), dm_b[rows].copy()
        C[np.arange(48), an] = gr["cap0"][an]
        D[np.arange(48), an] = 0.0
        f_o, _, ts_o, _ = og.assign(C, D, fl_b[rows], method="fw", iters=30, nthreads=8)
        np.testing.assert_array_equal(env.flow.cpu().numpy()[rows], f_o)
        np.testing.assert_array_equal(env.tstt.cpu().numpy()[rows], ts_o)

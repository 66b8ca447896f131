"""sp_backend="torch": the reference's GPU shortest-path backend
(_all_or_nothing_torch, src/env/repair_env.py:520-573 -- float32 Floyd-Warshall
with strict <, k ascending, next_hop walk), which configs/sioux_falls.yaml
(sp_backend: torch, force_gpu_sp: true) and run_greedy.py select.

Pinned to tests/golden/sf_torchsp_crpow.npz (tools/gen_golden_r2.py: the
reference's own _all_or_nothing_torch run on the CPU device): the AON at
t = BPR(0) for 24 damage patterns (integer costs, so tied shortest paths --
the rule differs from scipy's there), seed-42 resets, 32 random resets + 4
steps and a greedy MSA-30 episode.  Bar: bit-exact (flows, TSTT, rewards,
actions).
"""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import golden


def _z():
    return np.load(golden("sf_torchsp_crpow.npz"))


def _cap(gr, d):
    return np.where(d > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)


def test_oracle_fw_aon_vs_reference(oracle_graph, sf_graph_npz):
    z = _z()
    differs = 0
    for s in range(len(z["aon_aux"])):
        d = z["aon_damaged"][s]
        t = oracle_graph.bpr(np.zeros(76, np.float32), _cap(sf_graph_npz, d), d)
        aux, un = oracle_graph.aon(t, sp="torch")
        np.testing.assert_array_equal(aux, z["aon_aux"][s])
        assert un == z["aon_unassigned"][s]
        differs += not np.array_equal(aux, oracle_graph.aon(t)[0])
    assert differs >= 10   # tied resets: the torch rule is a different tie-break than scipy's


def test_oracle_fw_assign_vs_reference(oracle_graph, sf_graph_npz):
    z = _z()
    for key in ("msa30", "fw30", "msa60"):
        d = z[key + "_damaged"]
        f, t, ts, _ = oracle_graph.assign(_cap(sf_graph_npz, d), d, np.zeros(76, np.float32), method=key[:-2],
                                          iters=int(key[-2:]), sp="torch")
        np.testing.assert_array_equal(f, z[key + "_flow"])
        np.testing.assert_array_equal(t, z[key + "_t"])
        assert ts == z[key + "_tstt"]
    d = z["rand_damaged"]
    f, _, ts, _ = oracle_graph.assign(_cap(sf_graph_npz, d), d, np.zeros_like(d), iters=30, sp="torch", nthreads=8)
    np.testing.assert_array_equal(f, z["rand_flow"])
    np.testing.assert_array_equal(ts, z["rand_tstt"])


def test_sp_rule_resolution():
    from trafficrl import _lib
    from trafficrl.env.vec_env import resolve_sp_rule
    assert resolve_sp_rule("torch", 24) == _lib.SP_TORCH
    assert resolve_sp_rule("TORCH", 24, True) == _lib.SP_TORCH
    for b in ("auto", "scipy", None, "cupy", "cugraph"):
        assert resolve_sp_rule(b, 24) == _lib.SP_SCIPY
    with pytest.raises(RuntimeError):
        resolve_sp_rule("torch", 416)


def _vec(B, iters=30, method="msa", **kw):
    from trafficrl.data import sioux_falls
    from trafficrl.env import VecRepairEnv
    return VecRepairEnv(sioux_falls(), B, device="cuda", assignment_method=method, assignment_iters=iters,
                        reward_mode="rel_improve", reward_beta=0.0, reward_gamma=0.0, reward_clip=2.0,
                        unassigned_penalty=1e4, reset=False, sp_backend="torch", **kw)


@pytest.mark.gpu
def test_device_fw_aon_tied_resets():
    """K = 1 MSA from zero flow: flow == the AON loading at t = BPR(0)."""
    z = _z()
    env = _vec(len(z["aon_aux"]), iters=1)
    env.reset(damaged=torch.from_numpy(z["aon_damaged"]), observe=False)
    np.testing.assert_array_equal(env.flow.cpu().numpy(), z["aon_aux"])
    np.testing.assert_array_equal(env.unassigned.cpu().numpy(), z["aon_unassigned"])


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["msa30", "fw30", "msa60"])
def test_device_fw_resets(key):
    z = _z()
    env = _vec(3, iters=int(key[-2:]), method=key[:-2])
    env.reset(damaged=torch.from_numpy(np.repeat(z[key + "_damaged"][None], 3, 0)), observe=False)
    for b in range(3):
        np.testing.assert_array_equal(env.flow[b].cpu().numpy(), z[key + "_flow"])
        np.testing.assert_array_equal(env.t[b].cpu().numpy(), z[key + "_t"])
        assert float(env.tstt[b]) == float(z[key + "_tstt"])


@pytest.mark.gpu
def test_device_fw_random_resets_and_steps():
    z = _z()
    B = len(z["rand_seeds"])
    env = _vec(B)
    env.reset(damaged=torch.from_numpy(z["rand_damaged"]), observe=False)
    np.testing.assert_array_equal(env.flow.cpu().numpy(), z["rand_flow"])
    np.testing.assert_array_equal(env.tstt.cpu().numpy(), z["rand_tstt"])
    for j in range(4):
        _, rew, _, _ = env.step(torch.from_numpy(z["rand_step_actions"][:, j]), observe=False)
        np.testing.assert_array_equal(env.flow.cpu().numpy(), z["rand_step_flow"][:, j])
        np.testing.assert_array_equal(env.tstt.cpu().numpy(), z["rand_step_tstt"][:, j])
        np.testing.assert_array_equal(rew.cpu().numpy(), z["rand_step_reward"][:, j])


@pytest.mark.gpu
def test_device_fw_greedy_episode():
    """run_greedy.py's setup (sp_backend="torch", force_gpu_sp=True) through
    the drop-in facade: actions and TSTT curve == the reference's."""
    from trafficrl.baselines import run_episode, select_greedy_one_step
    from trafficrl.data import sioux_falls
    from trafficrl.env import RepairEnv
    z = _z()
    env = RepairEnv(sioux_falls(), assignment_iters=30, assignment_method="msa", fixed_damage=True,
                    fixed_damage_seed=42, seed=42, reward_mode="rel_improve", reward_alpha=1.0, reward_beta=0.0,
                    reward_gamma=0.0, reward_clip=2.0, unassigned_penalty=1e4, sp_backend="torch",
                    force_gpu_sp=True, use_torch=True)
    assert env.initial_tstt == float(z["greedy_initial_tstt"])
    actions = []

    def pol(s):
        a = select_greedy_one_step(env, s)
        actions.append(a)
        return a

    out = run_episode(env, pol)
    assert actions == z["greedy_actions"].tolist()
    np.testing.assert_array_equal(np.array(out["tstt_curve"]), z["greedy_tstt"])


@pytest.mark.gpu
def test_device_fw_big_batch_vs_oracle(oracle_graph):
    """B = 4096 random damage (tie-heavy resets) + one random step each:
    sampled rows == the oracle's Floyd-Warshall restatement."""
    gr = np.load(golden("sf_graph.npz"))
    rng = np.random.default_rng(17)
    B = 4096
    dmg = np.zeros((B, 76), np.float32)
    for b in range(B):
        dmg[b, rng.choice(76, 22, replace=False)] = 1.0
    env = _vec(B)
    env.reset(damaged=torch.from_numpy(dmg), observe=False)
    rows = rng.choice(B, 64, replace=False)
    f_o, _, ts_o, un_o = oracle_graph.assign(_cap(gr, dmg[rows]), dmg[rows], np.zeros((64, 76), np.float32),
                                             iters=30, sp="torch", nthreads=8)
    np.testing.assert_array_equal(env.flow.cpu().numpy()[rows], f_o)
    np.testing.assert_array_equal(env.tstt.cpu().numpy()[rows], ts_o)
    np.testing.assert_array_equal(env.unassigned.cpu().numpy()[rows], un_o)

"""Every reward mode of RepairEnv.compute_reward_with_goal
(src/env/repair_env.py:244-291) -- delta, log_delta (the reference's default,
:36), neg_tstt, minimize_tstt, rel_improve -- with non-zero beta/gamma and
clips, pinned to reference-generated episodes (tests/golden/sf_rewards_crpow.npz,
tools/gen_golden_r2.py: fixed seed 42 and two random damage seeds, 22 repairs
+ one already-repaired action each).

Bar: TSTT and done bit-exact; rewards bit-exact for delta / neg_tstt /
minimize_tstt / rel_improve (float64 arithmetic in the reference's order).
log_delta takes log10 of float64 TSTTs: the reference's numpy log10 and the
device's (OCML) are each within 1 ulp of the exact value but not always the
same double, so log_delta rewards are compared within
LOG_ATOL = 4 ulp(log10(max TSTT)) * alpha (measured: see DESIGN.md §3).
"""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import golden

LOG_ULPS = 4


def _fixture():
    return np.load(golden("sf_rewards_crpow.npz"))


def _log_atol(z, ci):
    alpha = float(z["cfg_params"][ci][0])
    return LOG_ULPS * np.spacing(np.log10(float(z["tstt"].max()))) * alpha


def test_oracle_reward_modes_vs_reference():
    """The C restatement (oracle/trx_oracle.c orc_reward) on the reference's
    own TSTT sequences reproduces the reference's rewards."""
    z = _fixture()
    for ci, mode in enumerate(z["cfg_modes"]):
        alpha, beta, gamma, clip = (float(v) for v in z["cfg_params"][ci])
        for si in range(z["actions"].shape[0]):
            prev = float(z["initial_tstt"][ci, si])
            repaired = set()
            for j in range(z["actions"].shape[1]):
                curr = float(z["tstt"][ci, si, j])
                ref = float(z["reward"][ci, si, j])
                a = int(z["actions"][si, j])
                if a in repaired:  # already-repaired link: -1, no assignment (repair_env.py:210-212)
                    assert ref == -1.0 and curr == prev
                    continue
                repaired.add(a)
                r = O.reward(str(mode), prev, curr, float(z["initial_tstt"][ci, si]), bool(z["done"][ci, si, j]),
                             alpha, beta, gamma, clip)
                if str(mode) == "log_delta":
                    assert abs(r - ref) <= _log_atol(z, ci), (mode, si, j, r, ref)
                else:
                    assert r == ref, (mode, si, j, r, ref)
                prev = curr


def test_fixture_covers_modes_and_bonus():
    z = _fixture()
    assert set(z["cfg_modes"].tolist()) == {"delta", "log_delta", "neg_tstt", "minimize_tstt", "rel_improve"}
    assert z["done"][:, :, -1].all() and not z["done"][:, :, :-1].any()
    # clips bind somewhere, the completion bonus shows in the last reward
    assert (np.abs(z["reward"][3]) == 1.0).any() and (np.abs(z["reward"][6]) == 0.5).any()
    assert (z["reward"][2, :, -1] > 5.0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(9))
def test_device_reward_modes_vs_reference(ci):
    from trafficrl.data import sioux_falls
    from trafficrl.env import VecRepairEnv
    z = _fixture()
    mode = str(z["cfg_modes"][ci])
    alpha, beta, gamma, clip = (float(v) for v in z["cfg_params"][ci])
    S = z["actions"].shape[0]
    env = VecRepairEnv(sioux_falls(), S, device="cuda", assignment_method="msa", assignment_iters=30,
                       reward_mode=mode, reward_alpha=alpha, reward_beta=beta, reward_gamma=gamma,
                       reward_clip=clip, capacity_damage=1e-3, unassigned_penalty=1e4, reset=False)
    env.reset(damaged=torch.from_numpy(z["damaged"]), observe=False)
    np.testing.assert_array_equal(env.initial_tstt.cpu().numpy(), z["initial_tstt"][ci])
    for j in range(z["actions"].shape[1]):
        _, rew, done, _ = env.step(torch.from_numpy(z["actions"][:, j]), observe=False)
        np.testing.assert_array_equal(env.tstt.cpu().numpy(), z["tstt"][ci, :, j])
        np.testing.assert_array_equal(done.cpu().numpy(), z["done"][ci, :, j])
        r = rew.cpu().numpy()
        if mode == "log_delta":
            np.testing.assert_allclose(r, z["reward"][ci, :, j], rtol=0, atol=_log_atol(z, ci))
        else:
            np.testing.assert_array_equal(r, z["reward"][ci, :, j])


@pytest.mark.gpu
def test_facade_default_reward_is_log_delta():
    """RepairEnv's default reward mode is the reference's log_delta (:36)."""
    from trafficrl.data import sioux_falls
    from trafficrl.env import RepairEnv
    z = _fixture()
    env = RepairEnv(sioux_falls(), assignment_iters=30, fixed_damage=True, fixed_damage_seed=42, seed=42,
                    unassigned_penalty=1e4)
    assert env.reward_mode == "log_delta"
    np.testing.assert_array_equal(env.is_damaged, z["damaged"][0])
    for j in range(z["actions"].shape[1]):
        _, r, d, info = env.step(int(z["actions"][0, j]))
        assert info["tstt"] == z["tstt"][0, 0, j]
        assert abs(r - z["reward"][0, 0, j]) <= _log_atol(z, 0)
        assert d == bool(z["done"][0, 0, j])

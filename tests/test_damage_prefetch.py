"""Damage prefetch (VecRepairEnv.enable_damage_prefetch): the next whole-batch
reset's masks are drawn on a host thread into pinned memory while the
device steps.  The masks, the generator states and the resets must be those
of drawing at reset time (src/env/repair_env.py:167-192 per env's
default_rng(seed) stream), including after a partial reset, which discards
the prefetched draw."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _env(prefetch):
    from trafficrl.data import sioux_falls
    from trafficrl.env import VecRepairEnv
    env = VecRepairEnv(sioux_falls(), 64, device="cuda:0", assignment_iters=5, reset=False,
                       seeds=[1000 + i for i in range(64)])
    assert env.enable_damage_prefetch(prefetch) == prefetch
    return env


def test_prefetched_resets_equal_reset_time_draws():
    a, b = _env(False), _env(True)
    for step in range(6):
        if step == 3:   # partial reset: the prefetch is discarded, both draw from the true states
            ids = [1, 5, 9]
            a.reset(env_ids=ids, observe=False)
            b.reset(env_ids=ids, observe=False)
        else:
            a.reset(observe=False)
            b.reset(observe=False)
        torch.cuda.synchronize()
        assert torch.equal(a.damaged, b.damaged), step
        assert torch.equal(a.tstt, b.tstt), step
        assert np.array_equal(a._rng_states, b._rng_states), step
    # the public draw continues both streams identically as well
    assert torch.equal(a.draw_damage(), b.draw_damage())
    b.close()

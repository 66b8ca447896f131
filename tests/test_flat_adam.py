"""trx_sac_adam (csrc/sac_optim.hip via rl/flat_adam.py): the optimizer step
over the fused update's flat gradient buffer against the torch path of
DiscreteSAC.apply_gradients (clip_grad_norm_ per optimizer, torch.optim.Adam,
log_alpha clamps, Polyak targets; src/rl/sac.py:224-263), from identical
gradients.  The two differ only in float rounding (lerp vs multiply-add
moments, norm of per-tensor norms vs one sum), so after a few steps every
parameter, target and log_alpha agrees to 1e-5 relative + 1e-7 absolute
(Adam's first steps move each weight by ~lr = 1e-4).  Also the handoff of
the moments to the torch optimizers and back (an autograd-path update in
the middle of fused ones)."""
import copy

import pytest
import torch

from test_sac_e2e import _update_batch, make_agent

pytestmark = pytest.mark.gpu

MODS = ("actor", "critic1", "critic2", "target1", "target2")


def _compare(a, b, rtol=1e-5, atol=1e-7):
    for m in MODS:
        for (k, pa), pb in zip(getattr(a, m).state_dict().items(), getattr(b, m).state_dict().values()):
            torch.testing.assert_close(pa, pb, rtol=rtol, atol=atol, msg=f"{m}.{k}")
    torch.testing.assert_close(a.log_alpha.detach(), b.log_alpha.detach(), rtol=rtol, atol=atol)


def _steps(paths, B=256):
    """agent a: updates along `paths` (fused -> trx_sac_adam, autograd ->
    torch optimizers after the handoff); agent b: the same gradients (copied
    from a's) through the torch optimizers every time."""
    from trafficrl.rl import sac
    batch = _update_batch(B)
    w = torch.rand(B, device="cuda") * 0.5 + 0.5
    a = make_agent(hidden=256, embed=256)
    b = copy.deepcopy(a)
    for path in paths:
        sac.FUSED_UPDATE = path == "fused"
        try:
            a.compute_gradients(batch, weights=w)
        finally:
            sac.FUSED_UPDATE = True
        assert a.last_update_path == path
        for pa, pb in zip(a._all_params(), b._all_params()):
            pb.grad = pa.grad.detach().clone()
        norm_c = float(torch.sqrt(sum((p.grad.double() ** 2).sum() for p in a.critic_params)))
        a.apply_gradients()
        sac.FLAT_ADAM = False
        try:
            b.apply_gradients()
        finally:
            sac.FLAT_ADAM = True
        if path == "fused":   # the critic group's gradient norm, as the kernel saw it
            assert abs(float(a._flat_adam.scal[3]) - norm_c) <= 1e-5 * norm_c
    return a, b


def test_flat_adam_vs_torch_optimizers():
    a, b = _steps(["fused"] * 4)
    assert a._flat_adam.owner == "flat" and getattr(b, "_flat_adam", None) is None
    _compare(a, b)


def test_flat_adam_handoff_to_torch_and_back():
    a, b = _steps(["fused", "fused", "autograd", "fused"])
    assert a._flat_adam.owner == "flat"
    _compare(a, b)
    a._flat_adam.export_torch()
    st = a.actor_opt.state[next(a.actor.parameters())]
    assert float(st["step"]) == 4.0

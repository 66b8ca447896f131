"""The fused MFMA tail (csrc/gat_tail.hip, trx_gat_tail_infer: the last GATConv
+ LayerNorm + ELU + pool and the edge scorer, src/models/gat_encoder.py:47-53,
src/rl/sac.py:38-46, 69-78) against the layer-kernel path it replaces
(hipBLASLt lin GEMM + trx_gat_layer_infer + two GEMMs + trx_edge_head_infer).

Both paths round at the same points (bf16 xh, p, c; bf16 logits) and the
tail replays the layer and edge kernels' summation orders, so they differ only
where the two GEMM implementations' fp32 accumulation orders round a bf16
output differently.  Bounds: logits within 1e-2 x their RMS (measured in the
docstring of each test), probabilities within 1e-3, and the in-kernel draw
picks the same link wherever the drawn uniform is not within the two paths'
CDF difference of a boundary.  The fp32 restatement check of the whole acting
pass (tests/test_sac_e2e.py::test_fused_bf16_acting_vs_fp32_restatement) runs
through the tail as well."""
import pytest
import torch

from test_sac_e2e import flat, make_agent, observations

pytestmark = pytest.mark.gpu


def _both(fn):
    from trafficrl.models import fused
    old = fused.TAIL
    try:
        fused.TAIL = True
        a = fn()
        fused.TAIL = False
        b = fn()
    finally:
        fused.TAIL = old
    return a, b


@pytest.mark.parametrize("B", [4096, 6])
def test_tail_actor_matches_layer_path(B):
    """B = 6: a partial last workgroup (4 + 2 graphs)."""
    env, obs, _ = observations(B)
    agent = make_agent()
    nx_, ei, ex_, mask, bv = flat(env, obs, B)
    u = torch.rand(B, device="cuda", generator=torch.Generator("cuda").manual_seed(5))

    def run():
        with torch.no_grad(), agent._amp():
            out = agent.actor._fused(nx_, ei, ex_, bv, B, mask=mask, u=u)
        assert out is not None
        return [t.clone() for t in out]

    (lt, pt, at), (lr, pr, ar) = _both(run)
    v = mask > 0
    rms = float(lr[v].pow(2).mean().sqrt())
    dl = float((lt - lr)[v].abs().max())
    print(f"B={B}: logit max diff {dl:.3e} (rms {rms:.3e}), prob max diff {float((pt - pr).abs().max()):.3e}, "
          f"identical logits {float((lt == lr)[v].float().mean()):.4f}, same draws {float((at == ar).float().mean()):.4f}")
    assert dl <= 1e-2 * rms
    assert torch.equal(lt[~v], lr[~v])
    assert float((pt - pr).abs().max()) < 1e-3
    # draws: identical unless u lies within the CDF difference of a boundary
    E = lt.numel() // B
    cdf_t, cdf_r = pt.view(B, E).cumsum(1), pr.view(B, E).cumsum(1)
    near = ((cdf_t - u[:, None]).abs() < 1e-4).any(1) | ((cdf_r - u[:, None]).abs() < 1e-4).any(1)
    assert bool((at == ar)[~near].all()), int((at != ar)[~near].sum())
    assert int((at >= 0).sum()) == B and int((at < E).sum()) == B


def test_tail_critic_matches_layer_path():
    B = 512
    env, obs, _ = observations(B)
    agent = make_agent()
    nx_, ei, ex_, mask, bv = flat(env, obs, B)

    def run():
        with torch.no_grad(), agent._amp():
            out = agent.critic1._fused(nx_, ei, ex_, bv, B)
        assert out is not None
        return out.clone()

    qt, qr = _both(run)
    rms = float(qr.pow(2).mean().sqrt())
    d = float((qt - qr).abs().max())
    print(f"critic: q max diff {d:.3e} (rms {rms:.3e}), identical {float((qt == qr).float().mean()):.4f}")
    assert d <= 1e-2 * rms

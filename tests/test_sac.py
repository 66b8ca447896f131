"""SAC layer (src/rl/sac.py) checks.

CPU: parameter counts, the factored edge-MLP equals the
reference's concat formulation (sac.py:42-43), segment softmax == PyG softmax.
GPU: update() with the three backward passes reordered (one bucketed
gradient all-reduce point) gives exactly the parameters the reference's
sequential critic->actor->alpha order gives; batched acting respects masks.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT


def test_param_counts_match_survey():
    from trafficrl.rl.sac import Actor, Critic
    a = Actor(4, 6, 256, 256, 3)
    c = Critic(4, 6, 256, 256, 3)
    assert sum(p.numel() for p in a.parameters()) == 1_611_797
    assert 2 * sum(p.numel() for p in c.parameters()) == 3_223_594


def test_factored_edge_mlp_equals_concat():
    from trafficrl.rl.sac import Actor
    torch.manual_seed(0)
    a = Actor(4, 6, 64, 32, 3).double()
    Nt, Et, B = 48, 152, 2
    h = torch.randn(Nt, 32, dtype=torch.float64)
    ctx = torch.randn(B, 64, dtype=torch.float64)
    e = torch.randn(Et, 6, dtype=torch.float64)
    src = torch.randint(0, Nt, (Et,))
    dst = torch.randint(0, Nt, (Et,))
    eb = torch.randint(0, B, (Et,))
    got = a.edge_scores(h, ctx, e, src, dst, eb)
    ref = a.edge_mlp(torch.cat([h[src], h[dst], e, ctx[eb]], dim=1)).squeeze(-1)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12)


def test_listwise_clip_matches_sequential_torch_semantics():
    from trafficrl.rl.sac import clip_grad_norm_listwise_
    torch.manual_seed(5)
    a = torch.nn.Parameter(torch.randn(10))
    b = torch.nn.Parameter(torch.randn(4))
    ga, gb = torch.randn(10) * 3, torch.randn(4) * 3
    a.grad, b.grad = ga.clone(), gb.clone()
    total = clip_grad_norm_listwise_([a, b, a], 1.0)
    ref_total = torch.sqrt(2 * ga.square().sum() + gb.square().sum())
    c = 1.0 / (ref_total + 1e-6)
    torch.testing.assert_close(total, ref_total)
    torch.testing.assert_close(a.grad, ga * c * c)
    torch.testing.assert_close(b.grad, gb * c)
    # plain lists: identical to torch (foreach=False)
    a.grad, b.grad = ga.clone(), gb.clone()
    clip_grad_norm_listwise_([a, b], 1.0)
    a2 = torch.nn.Parameter(a.detach().clone())
    b2 = torch.nn.Parameter(b.detach().clone())
    a2.grad, b2.grad = ga.clone(), gb.clone()
    torch.nn.utils.clip_grad_norm_([a2, b2], 1.0, foreach=False)
    torch.testing.assert_close(a.grad, a2.grad)
    torch.testing.assert_close(b.grad, b2.grad)


def test_segment_softmax_matches_pyg():
    from trafficrl.rl.sac import segment_softmax
    torch.manual_seed(1)
    x = torch.randn(4 * 76)
    x[::7] = -1e9
    idx = torch.arange(4).repeat_interleave(76)
    ex = torch.exp(x - x.view(4, 76).amax(1).repeat_interleave(76))
    ref = ex / (torch.zeros(4).index_add_(0, idx, ex).repeat_interleave(76) + 1e-16)
    torch.testing.assert_close(segment_softmax(x, idx, 4, 76), ref)
    torch.testing.assert_close(segment_softmax(x, idx, 4), ref)


def _batch(B, dev, gen):
    z = np.load(os.path.join(ROOT, "tests", "golden", "sf_graph.npz"))
    src = torch.as_tensor(z["src"], dtype=torch.long)
    dst = torch.as_tensor(z["dst"], dtype=torch.long)
    N, E = int(z["num_nodes"]), len(src)
    off = (torch.arange(B) * N).repeat_interleave(E)
    ei = torch.stack([src.repeat(B) + off, dst.repeat(B) + off]).to(dev)
    bv = torch.arange(B).repeat_interleave(N).to(dev)
    mask = (torch.rand(B * E, generator=gen) < 0.3).float().to(dev)
    mask.view(B, E)[:, 0] = 1.0
    nmask = mask.clone()
    nmask.view(B, E)[:, 0] = 0.0
    nmask.view(B, E)[:, 1] = 1.0
    act = torch.stack([torch.nonzero(mask.view(B, E)[b])[0, 0] + b * E for b in range(B)])
    return (torch.randn(B * N, 4, generator=gen).to(dev), ei, torch.randn(B * E, 6, generator=gen).to(dev), mask, bv,
            act, torch.randn(B, generator=gen).to(dev), torch.randn(B * N, 4, generator=gen).to(dev),
            torch.randn(B * E, 6, generator=gen).to(dev), nmask, bv, (torch.rand(B, generator=gen) < 0.2).float().to(dev))


def _reference_order_update(agent, batch, weights, alpha_max):
    """The reference's update (sac.py:157-263), statement order preserved."""
    (node_x, edge_index, edge_attr, action_mask, batch_vec, action, reward, next_node_x, next_edge_attr,
     next_action_mask, next_batch_vec, done) = batch
    from trafficrl.rl.sac import clip_grad_norm_listwise_ as clip_
    from trafficrl.rl.sac import scatter_sum
    B = reward.shape[0]
    w = torch.as_tensor(weights, device=reward.device, dtype=reward.dtype)
    edge_batch = batch_vec[edge_index[0]]
    with torch.no_grad():
        _, next_probs, _ = agent.actor(next_node_x, edge_index, next_edge_attr, next_action_mask, next_batch_vec, num_graphs=B)
        q_next = torch.min(agent.target1(next_node_x, edge_index, next_edge_attr, next_batch_vec, B),
                           agent.target2(next_node_x, edge_index, next_edge_attr, next_batch_vec, B))
        v_next = scatter_sum(next_probs * (q_next - agent.alpha * torch.log(next_probs + 1e-8)), edge_batch, B)
        target = reward + (1.0 - done) * agent.gamma * v_next
    q1_all = agent.critic1(node_x, edge_index, edge_attr, batch_vec, B)
    q2_all = agent.critic2(node_x, edge_index, edge_attr, batch_vec, B)
    q1, q2 = q1_all[action], q2_all[action]
    critic_loss = (w * (F.mse_loss(q1, target, reduction="none") + F.mse_loss(q2, target, reduction="none"))).mean()
    _, probs, _ = agent.actor(node_x, edge_index, edge_attr, action_mask, batch_vec, num_graphs=B)
    q_all = torch.min(q1_all, q2_all).detach()
    actor_loss = scatter_sum(probs * (agent.alpha * torch.log(probs + 1e-8) - q_all), edge_batch, B).mean()
    valid = scatter_sum((action_mask > 0).float(), edge_batch, B)
    te = (agent.target_entropy_ratio * torch.log(valid + 1e-8)).mean()
    log_probs = torch.log(probs + 1e-8).detach()
    alpha_loss = -(agent.log_alpha * scatter_sum(probs.detach() * (log_probs + te), edge_batch, B)).mean()
    agent.critic_opt.zero_grad()
    critic_loss.backward()
    clip_(list(agent.critic1.parameters()) + list(agent.critic2.parameters()), agent.grad_clip)
    agent.critic_opt.step()
    agent.actor_opt.zero_grad()
    actor_loss.backward()
    clip_(list(agent.actor.parameters()), agent.grad_clip)
    agent.actor_opt.step()
    agent.alpha_opt.zero_grad()
    alpha_loss.backward()
    clip_([agent.log_alpha], agent.grad_clip)
    agent.alpha_opt.step()
    agent.log_alpha.data.clamp_(max=float(np.log(alpha_max)))
    agent.log_alpha.data.clamp_(min=float(np.log(0.01)))
    if agent.share_critic_encoder:  # sac.py:245-248
        agent._soft_update(agent.critic_encoder, agent.target_encoder)
        agent._soft_update(agent.critic1.edge_mlp, agent.target1.edge_mlp)
        agent._soft_update(agent.critic2.edge_mlp, agent.target2.edge_mlp)
    else:
        agent._soft_update(agent.critic1, agent.target1)
        agent._soft_update(agent.critic2, agent.target2)


@pytest.mark.gpu
@pytest.mark.parametrize("share", [False, True])
def test_update_matches_reference_order(share):
    from trafficrl.rl.sac import DiscreteSAC
    torch.manual_seed(3)
    kw = dict(hidden=64, embed=64, num_layers=3, lr=1e-3, grad_clip=1.0, gamma=0.99, target_tau=0.01,
              alpha_init=0.1, target_entropy_ratio=0.2, share_critic_encoder=share, device="cuda")
    a1 = DiscreteSAC(4, 6, **kw)
    a2 = DiscreteSAC(4, 6, **kw)
    for m1, m2 in zip((a1.actor, a1.critic1, a1.critic2, a1.target1, a1.target2),
                      (a2.actor, a2.critic1, a2.critic2, a2.target1, a2.target2)):
        m2.load_state_dict(m1.state_dict())
    # SGD: parameter deltas are proportional to the gradients, so the comparison
    # checks gradient equality (Adam's normalisation would blow last-bit noise of
    # index_add_ atomics on near-zero gradients up to +-lr)
    for a in (a1, a2):
        a.actor_opt = torch.optim.SGD(a.actor.parameters(), lr=1e-2)
        a.critic_opt = torch.optim.SGD(a.critic_params, lr=1e-2)
        a.alpha_opt = torch.optim.SGD([a.log_alpha], lr=1e-2)
    gen = torch.Generator().manual_seed(0)
    mods1 = (a1.actor, a1.critic1, a1.critic2, a1.target1, a1.target2)
    mods2 = (a2.actor, a2.critic1, a2.critic2, a2.target1, a2.target2)

    def compare(rtol, atol):
        for name, m1, m2 in zip(("actor", "critic1", "critic2", "target1", "target2"), mods1, mods2):
            for (k, p1), p2 in zip(m1.state_dict().items(), m2.state_dict().values()):
                d = (p1 - p2).abs().max().item()
                assert torch.allclose(p1, p2, rtol=rtol, atol=atol), f"{name}.{k}: max|diff|={d:.3e}"

    # one update from identical states: semantics (only atomics-order noise)
    batch = _batch(8, "cuda", gen)
    w = torch.rand(8, generator=gen).numpy().astype(np.float32)
    out = a1.update(batch, weights=w, alpha_max=2.5)
    _reference_order_update(a2, batch, w, 2.5)
    compare(1e-6, 1e-7)
    # two more coupled updates: index_add_ atomics noise compounds, looser bound
    for _ in range(2):
        batch = _batch(8, "cuda", gen)
        w = torch.rand(8, generator=gen).numpy().astype(np.float32)
        out = a1.update(batch, weights=w, alpha_max=2.5)
        _reference_order_update(a2, batch, w, 2.5)
    assert isinstance(out["critic_loss"], float) and len(out["td_errors"]) == 8
    compare(1e-3, 1e-4)
    torch.testing.assert_close(a1.log_alpha, a2.log_alpha)


@pytest.mark.gpu
def test_batched_acting_respects_mask():
    from trafficrl.rl.sac import DiscreteSAC
    torch.manual_seed(4)
    agent = DiscreteSAC(4, 6, 64, 64, device="cuda", amp_dtype=torch.bfloat16)
    gen = torch.Generator().manual_seed(1)
    node_x, ei, ea, mask, bv, *_ = _batch(64, "cuda", gen)
    acts = agent.select_actions(node_x, ei, ea, mask, bv, num_graphs=64)
    assert acts.shape == (64,)
    m = mask.view(64, 76)
    assert bool((m[torch.arange(64, device="cuda"), acts] > 0).all())
    one = agent.select_action(node_x[:24], ei[:, :76], ea[:76], mask[:76])
    assert mask[one.action] > 0

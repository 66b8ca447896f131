"""Replay (src/train.py:27-91), HER (805-823) and the vectorised trainer.

GPU: sum-tree sampling == a numpy restatement of ReplayBuffer.sample's
descent on the same uniforms (float64 tree); add() priority growth
(max_p + k*eps), last-wins duplicate updates; HER relabel quirks; a short
training run (acting + env + PER updates) writes a checkpoint with the
reference's keys.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def ref_descent(tree, capacity, r):
    idx = 1
    while idx < capacity:
        left = 2 * idx
        if r <= tree[left]:
            idx = left
        else:
            r -= tree[left]
            idx = left + 1
    return idx - capacity


@pytest.mark.parametrize("cap", [8, 37, 1000])
def test_per_sampling_matches_reference_descent(cap):
    from trafficrl.rl.replay import DeviceReplay
    rb = DeviceReplay(cap, 24, 76, device="cuda")
    rng = np.random.default_rng(cap)
    n = min(cap, 3 * cap // 4)
    idx = torch.arange(n, device="cuda")
    leaf = torch.as_tensor(rng.random(n) + 0.01, device="cuda", dtype=torch.float64)
    rb._set(idx, leaf)
    tree = rb.tree.cpu().numpy()
    # tree consistency: every internal node = sum of children
    for k in range(1, cap):
        a = tree[2 * k] if 2 * k < 2 * cap else 0.0
        b = tree[2 * k + 1] if 2 * k + 1 < 2 * cap else 0.0
        assert abs(tree[k] - (a + b)) <= 1e-12 * max(1.0, tree[k])
    u = torch.rand(4096, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(0))
    out = torch.empty(4096, dtype=torch.int64, device="cuda")
    pri = torch.empty(4096, dtype=torch.float64, device="cuda")
    from trafficrl import _lib
    L = _lib.load()
    _lib.check(L.trx_per_sample(_lib.ptr(rb.tree), cap, _lib.ptr(u), 4096, _lib.ptr(out), _lib.ptr(pri), None), "s")
    ref = [ref_descent(tree, cap, float(x) * tree[1]) for x in u.cpu().numpy()]
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_add_priorities_and_last_wins():
    from trafficrl.rl.replay import DeviceReplay
    rb = DeviceReplay(16, 24, 76, alpha=0.6, eps=1e-6, device="cuda")
    B = 5
    z = lambda *s: torch.zeros(*s, device="cuda")  # noqa: E731
    rb.add_batch(z(B, 24, 4), z(B, 76, 6), z(B, 76), torch.zeros(B, dtype=torch.int64, device="cuda"), z(B),
                 z(B, 24, 4), z(B, 76, 6), z(B, 76), z(B), z(B, 76), z(B), z(B), z(B))
    leaves = rb.tree[16:16 + B].cpu().numpy()
    expect = [(1.0 + (k + 1) * 1e-6) ** 0.6 for k in range(B)]  # sequential reference adds
    np.testing.assert_allclose(leaves, expect, rtol=1e-14)
    rb.update_priorities(torch.tensor([2, 3, 2], device="cuda"), torch.tensor([0.5, -2.0, 4.0], device="cuda"))
    np.testing.assert_allclose(rb.tree[16 + 2].item(), (4.0 + 1e-6) ** 0.6, rtol=1e-12)
    np.testing.assert_allclose(rb.tree[16 + 3].item(), (2.0 + 1e-6) ** 0.6, rtol=1e-12)
    assert abs(rb.max_priority.item() - (4.0 + 1e-6)) < 1e-12
    s = rb.sample(64)
    assert s.weights.max().item() == pytest.approx(1.0)
    assert bool((s.idx < B).all())


@pytest.mark.parametrize("cap,lo,n", [(1000, 0, 1000), (1000, 377, 500), (65536, 61440, 4096), (24, 20, 4),
                                      (1_000_000, 995_904, 4096)])
def test_per_update_range_equals_general(cap, lo, n):
    """trx_per_update_range (ring adds) leaves the same float64 tree, bit for
    bit, as trx_per_update with idx = lo..lo+n-1 -- also for capacities that
    are not powers of two (leaves at two depths)."""
    from trafficrl import _lib
    L = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(cap + lo)
    base = torch.rand(2 * cap, device="cuda", dtype=torch.float64, generator=g)
    t1, t2 = base.clone(), base.clone()
    pri = torch.rand(n, device="cuda", dtype=torch.float64, generator=g) + 0.5
    idx = torch.arange(lo, lo + n, device="cuda", dtype=torch.int64)
    _lib.check(L.trx_per_update(_lib.ptr(t1), cap, _lib.ptr(idx), _lib.ptr(pri), n, None), "general")
    _lib.check(L.trx_per_update_range(_lib.ptr(t2), cap, lo, _lib.ptr(pri), n, None), "range")
    torch.cuda.synchronize()
    assert torch.equal(t1, t2)


@pytest.mark.parametrize("cap,lo,n", [(24, 20, 4), (1000, 377, 500), (1_000_000, 995_904, 4096)])
def test_per_add_range_equals_sequential_adds(cap, lo, n):
    """trx_per_add_range (one launch: leaves, ancestors, max_priority) ==
    n sequential reference adds (src/train.py:50-58): leaf k = (max_p +
    (k+1)*eps)**alpha, max_p -> max_p + n*eps; tree sums consistent."""
    from trafficrl import _lib
    L = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(cap + n)
    base = torch.rand(2 * cap, device="cuda", dtype=torch.float64, generator=g)
    t1, t2 = base.clone(), base.clone()
    mp = torch.tensor([1.75], device="cuda", dtype=torch.float64)
    eps, alpha = 1e-6, 0.6
    pri = (mp + eps * torch.arange(1, n + 1, device="cuda", dtype=torch.float64)) ** alpha
    _lib.check(L.trx_per_update_range(_lib.ptr(t1), cap, lo, _lib.ptr(pri), n, None), "range")
    mp2 = mp.clone()
    _lib.check(L.trx_per_add_range(_lib.ptr(t2), cap, lo, n, _lib.ptr(mp2), eps, alpha, None), "add_range")
    torch.cuda.synchronize()
    np.testing.assert_allclose(t2.cpu().numpy(), t1.cpu().numpy(), rtol=1e-14, atol=0)
    assert mp2.item() == 1.75 + eps * n
    leaves = t2[cap + lo:cap + lo + n].cpu().numpy()
    expect = [(1.75 + (k + 1) * eps) ** alpha for k in range(n)]
    np.testing.assert_allclose(leaves, expect, rtol=1e-14)


def test_staged_add_equals_add_batch():
    """Trainer path: stage_prev() before the env step + add_staged() after it
    (one multi-copy launch each, no clones) leaves the same ring contents and
    sum tree as add_batch(), including the wrap-around fallback."""
    from trafficrl.rl.replay import DeviceReplay
    g = torch.Generator(device="cuda").manual_seed(5)
    r = lambda *s: torch.rand(*s, device="cuda", generator=g)  # noqa: E731
    a, b = DeviceReplay(24, 24, 76, device="cuda"), DeviceReplay(24, 24, 76, device="cuda")
    for B in (10, 10, 10):          # the third add wraps (ptr 20 + 10 > 24)
        f = dict(node_x=r(B, 24, 4), edge_x=r(B, 76, 6), mask=r(B, 76), goal=r(B, 76),
                 prev=r(B).double(), action=torch.randint(0, 76, (B,), device="cuda", dtype=torch.int32),
                 reward=r(B).double(), nnx=r(B, 24, 4), nex=r(B, 76, 6), nm=r(B, 76), done=(r(B) > 0.5),
                 nt=r(B).double(), it=r(B).double())
        a.add_batch(f["node_x"], f["edge_x"], f["mask"], f["action"], f["reward"], f["nnx"], f["nex"], f["nm"],
                    f["done"].float(), f["goal"], f["prev"], f["nt"], f["it"])
        if b.stage_prev(f["node_x"], f["edge_x"], f["mask"], f["goal"], f["prev"]):
            b.add_staged(f["action"], f["reward"], f["nnx"], f["nex"], f["nm"], f["done"].float(), f["nt"], f["it"])
        else:
            b.add_batch(f["node_x"], f["edge_x"], f["mask"], f["action"], f["reward"], f["nnx"], f["nex"], f["nm"],
                        f["done"].float(), f["goal"], f["prev"], f["nt"], f["it"])
    for name in ("node_x", "edge_x", "mask", "next_node_x", "next_edge_x", "next_mask", "goal", "action", "reward",
                 "done", "prev_tstt", "next_tstt", "init_tstt", "tree", "max_priority"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert (a.ptr, a.size) == (b.ptr, b.size)


def test_her_relabel_quirks():
    from trafficrl.rl.replay import DeviceReplay, her_relabel
    rb = DeviceReplay(8, 24, 76, device="cuda")
    B = 4
    nm = (torch.rand(B, 76, device="cuda") < 0.3).float()
    ex = torch.rand(B, 76, 6, device="cuda")
    rb.add_batch(torch.zeros(B, 24, 4, device="cuda"), ex, nm, torch.zeros(B, dtype=torch.int64, device="cuda"),
                 torch.zeros(B, device="cuda"), torch.zeros(B, 24, 4, device="cuda"), ex, nm,
                 torch.zeros(B, device="cuda"), nm, torch.full((B,), 500.0, device="cuda"),
                 torch.full((B,), 400.0, device="cuda"), torch.full((B,), 1000.0, device="cuda"))
    s = rb.sample(16)
    s = her_relabel(s, 1.0, "rel_improve", 0.5, 1.0, 0.0, 0.0, 2.0)
    goal = 1.0 - s.next_mask
    assert torch.equal(s.edge_x[:, :, -1], goal)           # apply_goal writes column -1 (train.py:127)
    assert torch.equal(s.done, torch.ones_like(s.done))    # (1-m)*m == 0 -> always "complete"
    r = (100.0 * (500.0 - 400.0) / 1000.0 - 400.0 / 1000.0)
    torch.testing.assert_close(s.reward, torch.full_like(s.reward, min(r, 2.0) * 0.5))


def test_short_training_run(tmp_path):
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    cfg.update(num_envs=64, batch_start=128, batch_size=32, hidden_dim=32, embed_dim=32, episodes=64,
               eval_every=64, output_dir=str(tmp_path), update_every=1, update_unit="iterations", her_ratio=0.5)
    tr = Trainer(cfg, device="cuda", log=False)
    hist = tr.run(max_iters=30)
    assert tr.episodes_done >= 64 and len(hist) >= 1
    assert np.isfinite(float(tr.last_losses["critic_loss"]))
    assert tr.replay.size == 64 * 22 or tr.replay.size > 128
    sd = torch.load(os.path.join(str(tmp_path), "model_last.pt"), map_location="cpu", weights_only=True)
    assert set(sd) == {"actor", "critic1", "critic2", "target1", "target2", "log_alpha"}
    ev = tr.evaluate()
    assert np.isfinite(ev["tstt_last"])


def test_training_run_transition_schedule(tmp_path):
    """The reference's update schedule (update_unit "transitions", max_steps
    truncation; sf_sac.yaml) past batch_start: env.done is the env's uint8
    tensor, the per-env due counts reach the update loop, and the graph
    capture keeps the topology it reads alive when the caches are cleared."""
    from trafficrl.models import fused
    from trafficrl.train import Trainer, batched_topology, sf_config
    cfg = sf_config()
    cfg.update(num_envs=16, batch_start=64, batch_size=16, hidden_dim=32, embed_dim=32, episodes=10 ** 6,
               eval_every=0, output_dir=str(tmp_path), update_unit="transitions", update_every=4, max_steps=6)
    tr = Trainer(cfg, device="cuda", log=False)
    assert tr.env.done.dtype == torch.uint8
    seen = []
    orig = tr.update
    tr.update = lambda: (seen.append(1), orig())[1]
    tr.run(max_iters=14)
    assert len(seen) > 0 and np.isfinite(float(tr.last_losses["critic_loss"]))
    # evict every cached topology; the captured acting / update graphs keep theirs
    fused._topo_cache.clear()
    for _ in range(70):
        fused.topology(*batched_topology(tr.env.edge_index, tr.N, 3), 3)
    tr.run(max_iters=4)
    assert np.isfinite(float(tr.last_losses["critic_loss"]))


@pytest.mark.gpu
@pytest.mark.parametrize("her,hidden,embed", [(0.0, 32, 32), (0.5, 32, 32), (0.0, 64, 256)])
def test_graphed_update_matches_eager(tmp_path, her, hidden, embed):
    """The HIP-graph replayed update (train.GraphedUpdate) does the same
    arithmetic as the eager one: same RNG draws, same PER indices, parameters
    equal up to kernel-order rounding after several updates.  hidden 64 x 4
    heads / embed 256 puts the no-grad passes on the fused inference kernels
    inside the captured graph."""
    from trafficrl.train import Trainer, sf_config
    trs = []
    for graphed in (False, True):
        cfg = sf_config()
        cfg.update(num_envs=32, batch_start=64, batch_size=16, hidden_dim=hidden, embed_dim=embed, eval_every=0,
                   lr=1e-4, actor_lr=None, critic_lr=None, alpha_lr=None,
                   output_dir=str(tmp_path), update_every=1, update_unit="iterations", her_ratio=her,
                   graph_update=graphed)
        tr = Trainer(cfg, device="cuda", log=False)
        trs.append(tr)
    ag = trs[0].agent   # same (device-side step count) Adam arithmetic in both
    ag.capturable = True
    ad = dict(lr=1e-4, capturable=True, fused=True)
    ag.actor_opt = torch.optim.Adam(ag.actor.parameters(), **ad)
    ag.critic_opt = torch.optim.Adam(ag.critic_params, **ad)
    ag.alpha_opt = torch.optim.Adam([ag.log_alpha], **ad)
    # identical weights, identical replay contents
    for m_e, m_g in zip((trs[0].agent.actor, trs[0].agent.critic1, trs[0].agent.critic2, trs[0].agent.target1,
                         trs[0].agent.target2),
                        (trs[1].agent.actor, trs[1].agent.critic1, trs[1].agent.critic2, trs[1].agent.target1,
                         trs[1].agent.target2)):
        m_g.load_state_dict(m_e.state_dict())
    obs = []
    for tr in trs:
        tr._reset_envs(None)
        obs.append(tr.env.observe())
    for it in range(3):
        a = trs[0].act(obs[0])
        trs[1].act(obs[1])   # keep both generators in step
        for k, tr in enumerate(trs):
            o = obs[k]
            prev = (o.node_x.clone(), o.edge_x.clone(), o.action_mask.clone())
            goal, prev_t = tr.env.goal.clone(), tr.env.tstt.clone()
            nxt, rew, done, _ = tr.env.step(a.to(torch.int32), check=False)
            tr.replay.add_batch(prev[0], prev[1], prev[2], a, rew * 0.5, nxt.node_x, nxt.edge_x, nxt.action_mask,
                                done.float(), goal, prev_t, tr.env.tstt, tr.env.initial_tstt)
            obs[k] = nxt
    for step in range(6):   # 3 eager warm-up + capture + 2 replays on the graphed trainer
        outs = [tr.update() for tr in trs]
        torch.cuda.synchronize()
        d = (outs[1]["td_errors"] - outs[0]["td_errors"]).abs().max().item()
        print(f"update {step}: max|d td_error| {d:.3e}")
        torch.testing.assert_close(outs[1]["td_errors"], outs[0]["td_errors"], rtol=2e-3, atol=2e-4,
                                   msg=lambda m: f"update {step}: {m}")
    assert trs[1]._graphed.g_grads is not None
    for (k, p_e), p_g in zip(trs[0].agent.actor.state_dict().items(), trs[1].agent.actor.state_dict().values()):
        torch.testing.assert_close(p_g, p_e, rtol=1e-3, atol=1e-4, msg=k)
    torch.testing.assert_close(trs[1].replay.tree, trs[0].replay.tree, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(trs[1].agent.log_alpha, trs[0].agent.log_alpha)


@pytest.mark.gpu
def test_graphed_act_matches_eager(tmp_path):
    """train.GraphedAct: the replayed acting graph draws the same actions as
    the eager fused pass from the same generator state, across weight changes
    (prepared-weight slots refreshed in place) and new observations written
    into the env's persistent buffers."""
    from trafficrl.models import fused
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    cfg.update(num_envs=64, batch_start=64, batch_size=16, hidden_dim=64, embed_dim=256, eval_every=0,
               output_dir=str(tmp_path), update_unit="iterations")
    tr = Trainer(cfg, device="cuda", log=False)
    assert tr._graphed_act is not None
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(5):
        st = tr.gen.get_state()
        a_g = tr.act(obs).clone()
        st_after = tr.gen.get_state()
        tr.gen.set_state(st)
        a_e = tr._act(obs)
        assert torch.equal(tr.gen.get_state(), st_after)     # same number of draws
        assert tr.agent.last_act_path == "fused"
        assert torch.equal(a_g, a_e), it
        if it >= 1:
            assert tr._graphed_act.g is not None
        with torch.no_grad():   # an "update": new weights, same parameter storage
            for p in tr.agent.actor.parameters():
                p.add_(0.05 * torch.randn_like(p))
        fused.weights_changed()
        obs = tr.env.step(a_e.to(torch.int32), check=False)[0]


@pytest.mark.gpu
def test_graph_memset_replay_selftest():
    """capture_graph rewrites captured memset nodes into fill kernels, so a
    small hipMemsetAsync replays correctly (ROCm 7.2 packet-capture defect)
    and the trainer keeps HIP-graph updates enabled."""
    from trafficrl.train import graph_memset_replays_ok
    assert graph_memset_replays_ok(torch.device("cuda", 0))


@pytest.mark.gpu
def test_graphed_column_reduction_replays():
    """Multi-block column sums (Linear bias gradients; torch clears their
    semaphores with a small memset) equal eager on every replay."""
    from trafficrl.train import capture_graph
    x = torch.randn(6144, 1024, device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        x.sum(0)
    torch.cuda.current_stream().wait_stream(side)
    g, y = capture_graph(lambda: x.sum(0))
    for _ in range(4):
        x.normal_()
        g.replay()
        torch.testing.assert_close(y, x.double().sum(0).float(), rtol=1e-4, atol=1e-3)


def test_fw30_per_training_run(tmp_path):
    """Config #3 in small: FW-30 envs, SAC+GAT with PER (prioritised sampling,
    priority write-back) and HIP-graph updates; losses finite, priorities
    moved off the insertion maximum, a checkpoint written."""
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    cfg.update(num_envs=256, batch_start=256, batch_size=64, hidden_dim=32, embed_dim=32, eval_every=0,
               output_dir=str(tmp_path), update_every=1, update_unit="iterations", assignment_method="fw",
               assignment_iters=30, sp_backend="scipy", episodes=10 ** 6)
    tr = Trainer(cfg, device="cuda", log=False)
    tr.run(max_iters=12)
    assert tr._graphed is None or tr._graphed.g_grads is not None
    for k in ("critic_loss", "actor_loss", "alpha_loss"):
        assert np.isfinite(float(tr.last_losses[k])), k
    n = tr.replay.size
    leaves = tr.replay.tree[tr.replay.capacity:tr.replay.capacity + n]
    assert float(leaves.min()) < float(leaves.max())          # TD-error priorities written back
    assert tr.replay.tree.dtype == torch.float32      # the reference's float32 tree (per_tree default)
    # float32 deltas accumulated down the chain: the root drifts by a few ulps per update at most
    assert abs(float(tr.replay.tree[1]) - float(leaves.double().sum())) <= 1e-4 * float(leaves.double().sum())
    assert os.path.exists(os.path.join(str(tmp_path), "model_last.pt"))


@pytest.mark.gpu
def test_sample_rows_match_indexing():
    """sample() gathers every field in one trx_multi_gather launch: rows equal
    plain indexing, repeated indices included."""
    from trafficrl.rl.replay import DeviceReplay
    d = torch.device("cuda", 0)
    rb = DeviceReplay(64, 24, 76, device=d, tree_dtype="float32")
    g = torch.Generator(device=d).manual_seed(3)
    B = 48
    r = lambda *s, **kw: torch.rand(*s, device=d, generator=g, **kw)  # noqa: E731
    rb.add_batch(r(B, 24, 4), r(B, 76, 6), r(B, 76), torch.randint(0, 76, (B,), device=d, generator=g), r(B),
                 r(B, 24, 4), r(B, 76, 6), r(B, 76), r(B), r(B, 76), r(B, dtype=torch.float64),
                 r(B, dtype=torch.float64), r(B, dtype=torch.float64))
    u = torch.rand(200, dtype=torch.float64, device=d, generator=g)
    s = rb.sample(200, u=u)
    assert int(torch.unique(s.idx).numel()) < 200      # repeats present
    for name in ("node_x", "edge_x", "mask", "action", "reward", "next_node_x", "next_edge_x", "next_mask", "done",
                 "goal", "prev_tstt", "next_tstt", "init_tstt"):
        assert torch.equal(getattr(s, name), getattr(rb, name)[s.idx]), name


@pytest.mark.gpu
@pytest.mark.parametrize("max_steps", [0, 3])
def test_episode_step_kernel_matches_torch_ops(max_steps):
    """trx_episode_step == the trainer's torch bookkeeping (float64, same op order), bit for bit."""
    from trafficrl import _lib
    d = torch.device("cuda", 0)
    g = torch.Generator(device=d).manual_seed(9)
    B = 1000
    reward = torch.randn(B, dtype=torch.float64, device=d, generator=g) * 3
    done = (torch.rand(B, device=d, generator=g) < 0.3).to(torch.uint8)
    tstt = torch.rand(B, dtype=torch.float64, device=d, generator=g) * 1e6
    st = {k: torch.randn(B, dtype=torch.float64, device=d, generator=g) for k in ("rew", "sum", "auc", "prev")}
    ep_len = torch.randint(0, 4, (B,), device=d, generator=g)
    ref = {k: v.clone() for k, v in st.items()}
    ref_len = ep_len.clone()
    scale = 0.5
    # torch ops of Trainer.iteration (CPU branch)
    scaled_ref = reward * scale
    ref_len += 1
    trunc = (ref_len >= max_steps) if max_steps > 0 else torch.zeros_like(done, dtype=torch.bool)
    ref["rew"] += scaled_ref
    ref["sum"] += tstt
    ref["auc"] += 0.5 * (ref["prev"] + tstt) * (ref_len > 1)
    ref["prev"].copy_(tstt)
    fin_ref = done.bool() | trunc
    out = dict(scaled=torch.empty(B, dtype=torch.float64, device=d), s32=torch.empty(B, device=d),
               d32=torch.empty(B, device=d), fin=torch.empty(B, dtype=torch.uint8, device=d))
    L = _lib.load()
    _lib.check(L.trx_episode_step(B, _lib.ptr(reward), _lib.ptr(done), _lib.ptr(tstt), scale, max_steps,
                                  _lib.ptr(out["scaled"]), _lib.ptr(out["s32"]), _lib.ptr(out["d32"]), _lib.ptr(st["rew"]),
                                  _lib.ptr(st["sum"]), _lib.ptr(st["auc"]), _lib.ptr(st["prev"]), _lib.ptr(ep_len),
                                  _lib.ptr(out["fin"]), _lib.stream_ptr(d)), "trx_episode_step")
    torch.cuda.synchronize()
    assert torch.equal(out["scaled"], scaled_ref) and torch.equal(out["s32"], scaled_ref.float())
    assert torch.equal(out["d32"], done.float()) and torch.equal(out["fin"].bool(), fin_ref)
    assert torch.equal(ep_len, ref_len)
    for k in st:
        assert torch.equal(st[k], ref[k]), k

"""Trainer configuration (CPU): reference cfg.get fallbacks, YAML numeric
strings, and the update schedule (update-to-data ratio)."""
from types import SimpleNamespace

from trafficrl.train import DEFAULTS, Trainer, load_config, sf_config


def test_defaults_are_the_reference_fallbacks():
    # src/train.py cfg.get(key, default) fallbacks
    ref = dict(reward_mode="delta", reward_beta=10.0, reward_gamma=0.1, reward_clip=0.0, reward_scale=1.0,
               update_every=1, updates_per_step=1, fixed_damage=False, early_stop_patience=500,
               early_stop_min_delta=0.0, share_critic_encoder=True, target_entropy_ratio=0.6, max_steps=0,
               unassigned_penalty=2e7, eval_every=50, sp_backend="auto", force_gpu_sp=False, gp_keep_paths=3,
               per_alpha=0.6, per_beta=0.4, per_eps=1e-6, her_ratio=0.0, capacity_damage=1e-3, grad_clip=None,
               alpha_max=None, alpha_init=0.1)
    for k, v in ref.items():
        assert DEFAULTS[k] == v, k
    assert DEFAULTS["eval_seeds"] == [1001, 1002, 1003, 1004, 1005]
    assert DEFAULTS["amp"] is None   # fp32 like the reference


def test_yaml_numeric_strings(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("unassigned_penalty: 1.0e4\nbuffer_size: 1.0e6\nlr: 1.0e-4\neval_seeds: []\nsp_backend: torch\n")
    c = load_config(str(p))
    assert c["unassigned_penalty"] == 1e4 and isinstance(c["unassigned_penalty"], float)
    assert c["buffer_size"] == 1000000 and isinstance(c["buffer_size"], int)
    assert c["lr"] == 1e-4 and c["sp_backend"] == "torch"
    assert c["eval_seeds"] == [1001, 1002, 1003, 1004, 1005]


def test_sf_config_mirrors_reference_yaml():
    c = sf_config()
    assert c["sp_backend"] == "torch" and c["force_gpu_sp"] is True
    assert c["reward_mode"] == "rel_improve" and c["reward_clip"] == 2.0 and c["reward_scale"] == 0.5
    assert c["update_every"] == 4 and c["update_unit"] == "transitions"


def _fake(B, size, **cfg):
    import torch
    base = dict(batch_start=100, updates_per_step=1, update_every=4, update_unit="transitions", max_steps=0)
    base.update(cfg)
    # env.done is uint8, as VecRepairEnv keeps it (vec_env.py)
    return SimpleNamespace(cfg=base, B=B, replay=SimpleNamespace(size=size), _transitions=0, world=1,
                           _due_carry=0, ep_len=torch.zeros(B, dtype=torch.int64),
                           env=SimpleNamespace(done=torch.zeros(B, dtype=torch.uint8)))


def _episode(f, steps, done_at=None):
    import torch
    """Drive updates_due through one episode per env (ep_len as trx_episode_step advances it)."""
    out = []
    for it in range(steps):
        f.ep_len += 1
        if done_at is not None:
            f.env.done = (f.ep_len >= done_at).to(torch.uint8)
        out.append(Trainer.updates_due(f, it))
    return out


def test_update_schedule_transitions_follows_reference_episode_counter():
    # reference serial loop (src/train.py:919, 954-955): per-episode `steps`, an update
    # whenever steps % update_every == 0 -> 5 updates in a 22-step episode at update_every 4
    f = _fake(B=1, size=1000)
    n = _episode(f, 22, done_at=22)
    assert sum(n) == 5 and [i + 1 for i, k in enumerate(n) if k] == [4, 8, 12, 16, 20]
    f = _fake(B=1, size=1000, updates_per_step=2)
    assert _episode(f, 8) == [0, 0, 0, 2, 0, 0, 0, 2]
    # envs at different episode offsets: the iteration's count sums over envs
    f = _fake(B=3, size=1000)
    f.ep_len[:] = __import__("torch").tensor([0, 1, 3])
    assert _episode(f, 4) == [1, 0, 1, 1]   # counters 1,2,4 -> 2,3,5 -> 3,4,6 -> 4,5,7
    # truncation (max_steps reached, not done) breaks out before the update check (950-952)
    f = _fake(B=1, size=1000, max_steps=8)
    assert _episode(f, 8) == [0, 0, 0, 1, 0, 0, 0, 0]
    f = _fake(B=1, size=1000, max_steps=8)
    assert _episode(f, 8, done_at=8) == [0, 0, 0, 1, 0, 0, 0, 1]   # done on the last step: updated
    f = _fake(B=10, size=50)      # replay not yet past batch_start
    assert _episode(f, 4) == [0, 0, 0, 0] and f._transitions == 40


def test_update_schedule_iterations():
    f = _fake(B=4096, size=10 ** 6, update_unit="iterations", updates_per_step=1, update_every=4)
    assert [Trainer.updates_due(f, it) for it in range(8)] == [1, 0, 0, 0, 1, 0, 0, 0]


def _due_worker(rank, world, port, q):
    import os
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # uneven episode offsets per rank (random damage: different episode lengths)
    f = _fake(B=3 + rank, size=1000, max_steps=7)
    f.world = world
    f.ep_len[:] = torch.arange(3 + rank) * (1 + rank)
    got, own = [], 0
    for it in range(12):
        f.ep_len += 1
        f.env.done = ((f.ep_len % (5 + rank)) == 0).to(torch.uint8)
        due = ((f.ep_len % 4) == 0) & ~((f.ep_len >= 7) & ~f.env.done.bool())
        own += int(due.sum())
        got.append(Trainer.updates_due(f, it))
        f.ep_len[(f.ep_len >= 7) | f.env.done.bool()] = 0
    q.put((rank, got, own, f._due_carry))
    dist.destroy_process_group()


def test_update_schedule_transitions_world2_lockstep():
    """world > 1: ranks with different episode states must still run the same
    number of updates per iteration (each update all-reduces gradients)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_due_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(30)
    (_, g0, o0, c0), (_, g1, o1, c1) = res
    assert g0 == g1                                  # lockstep
    assert o0 != o1                                  # the ranks' own schedules did differ
    assert 2 * sum(g0) + c0 == o0 + o1 and c0 == c1  # every due update dealt out (carry < world)

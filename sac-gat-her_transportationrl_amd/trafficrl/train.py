"""Vectorised GAT-SAC trainer: the capabilities of src/train.py:216-1193 on
device-resident envs.

Same YAML keys as the reference configs (configs/sioux_falls.yaml): damage
(damaged_ratio, fixed_damage, fixed_damage_seed, capacity_damage), assignment
(assignment_iters, assignment_method), reward (reward_mode, reward_alpha/beta/
gamma/clip, reward_scale, unassigned_penalty), SAC (hidden_dim, embed_dim,
gat_layers, lr, actor_lr, critic_lr, alpha_lr, gamma, target_tau, grad_clip,
alpha_init, alpha_max, target_entropy_ratio, share_critic_encoder), replay
(buffer_size, batch_size, batch_start, update_every, updates_per_step,
per_alpha, per_beta, per_eps, her_ratio), loop (episodes, max_steps,
eval_every, eval_seeds, early_stop_patience, seed, output_dir).  New keys:
num_envs (envs stepped in lockstep per GPU; the reference's 1 env or
num_workers CPU processes, train.py:730-913) and amp (bf16 autocast for the
GAT/SAC GEMMs).

One iteration = every env takes one step: batched actor forward (one
multinomial per env) -> trx_step + trx_observe -> transitions appended to the
device replay -> the SAC updates due (Trainer.updates_due: by default the
reference's update-to-data ratio, updates_per_step / update_every updates per
transition) on PER samples (+HER).  Multi-GPU (torchrun): envs and replay are
per-rank shards; the only collective on the data path is one bucketed
all-reduce of all SAC gradients per update (RCCL over xGMI); episode
bookkeeping adds one 4-byte all-reduce per iteration and an all-gather of the
finished episodes' metrics, so every rank stops at the same iteration.
"""
from __future__ import annotations

import argparse
import json
import logging
import math
import os
import time
from typing import Dict, Optional

import numpy as np
import torch

from .data.tntp_parser import load_graph_data, sioux_falls
from .models import fused
from .models.tensor_cache import pinning
from .env.vec_env import VecRepairEnv
from .rl.replay import DeviceReplay, her_relabel
from . import _lib
from .rl.sac import DiscreteSAC

# Fallbacks of the reference trainer's cfg.get(...) calls (src/train.py:146-351):
# a reference yaml that omits a key trains the same way here.  Keys the
# reference reads without a default (cfg["..."]) take configs/sioux_falls.yaml's
# values.  The Sioux Falls training setup itself is trafficrl/sf_sac.yaml
# (sf_config()).  New keys: num_envs, amp (None = fp32 like the reference;
# "bf16" autocast), graph_update, update_unit, log_every, save_every.
DEFAULTS: Dict = dict(
    damaged_ratio=0.3, assignment_iters=30, assignment_method="msa", sp_backend="auto", force_gpu_sp=False,
    reward_mode="delta", reward_alpha=1.0, reward_beta=10.0, reward_gamma=0.1, reward_clip=0.0, reward_scale=1.0,
    capacity_damage=1e-3, unassigned_penalty=2e7, gp_step=1.0, gp_keep_paths=3, fixed_damage=False,
    fixed_damage_seed=None, episodes=2000, max_steps=0, buffer_size=1_000_000, batch_start=2000, batch_size=256,
    update_every=1, updates_per_step=1, update_unit="transitions", per_alpha=0.6, per_beta=0.4, per_eps=1e-6,
    per_tree="float32",
    her_ratio=0.0, hidden_dim=256, embed_dim=256, gat_layers=3, lr=1e-4, actor_lr=None, critic_lr=None,
    alpha_lr=None, gamma=0.99, target_tau=0.001, grad_clip=None, share_critic_encoder=True, alpha_init=0.1,
    alpha_max=None, target_entropy_ratio=0.6, eval_every=50, eval_seeds=[1001, 1002, 1003, 1004, 1005],
    early_stop_patience=500, early_stop_min_delta=0.0, seed=42, output_dir="outputs", num_envs=256, amp=None,
    log_every=10, save_every=50, net_path=None, trips_path=None, graph_update=True,
)
SF_CONFIG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sf_sac.yaml")


def load_config(path: Optional[str]) -> Dict:
    cfg = dict(DEFAULTS)
    if path:
        import yaml
        with open(path) as fh:
            cfg.update(yaml.safe_load(fh) or {})
    # PyYAML (YAML 1.1) reads exponents without a sign ("1.0e4", as in the
    # reference's configs/sioux_falls.yaml) as strings; the reference's float()
    # / arithmetic accepts them, so numeric-looking strings become numbers here
    for k, v in list(cfg.items()):
        if isinstance(v, str):
            try:
                f = float(v)
            except ValueError:
                continue
            cfg[k] = int(f) if isinstance(DEFAULTS.get(k), int) and not isinstance(DEFAULTS.get(k), bool) \
                and f == int(f) else f
    if not cfg.get("eval_seeds"):   # train.py:351 `cfg.get("eval_seeds") or [1001..1005]`
        cfg["eval_seeds"] = list(DEFAULTS["eval_seeds"])
    if os.environ.get("SEED_OVERRIDE") is not None:  # train.py:218-222
        cfg["seed"] = int(os.environ["SEED_OVERRIDE"])
        cfg["output_dir"] = os.path.join(cfg["output_dir"], f"seed_{cfg['seed']}")
    return cfg


GEMM_TUNING_GFX950 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_tuning_gfx950.csv")


def use_tuned_gemms(path: str) -> bool:
    """Select the GEMM kernels of the acting pass and the SAC update from a
    PyTorch TunableOp results file (hipBLASLt / rocBLAS solution per shape,
    measured on MI355X with this image's ROCm, hipBLASLt and torch: the file's
    validators must match or torch ignores it).  Lookup only -- no tuning at
    run time, nothing written; shapes not in the file keep torch's default.
    Same operands and fp32 accumulation: another kernel, not another precision.
    Process-wide (TunableOp is global)."""
    import torch.cuda.tunable as tunable
    if not (torch.cuda.is_available() and os.path.exists(path)):
        return False
    import tempfile
    try:
        tunable.enable(True)
        tunable.tuning_enable(False)
        # TunableOp's own output file (written at exit, if at all) goes to a scratch path
        tunable.set_filename(os.path.join(tempfile.gettempdir(), f"trx_tunableop_{os.getpid()}.csv"))
        if tunable.read_file(path):
            return True
    except Exception:   # an unreadable file or another torch build: torch's default kernels
        pass
    tunable.enable(False)
    return False


def sf_config() -> Dict:
    """The Sioux Falls GAT-SAC setup (trafficrl/sf_sac.yaml: the reference's
    configs/sioux_falls.yaml values plus num_envs / amp)."""
    return load_config(SF_CONFIG)


def batched_topology(edge_index: torch.Tensor, num_nodes: int, B: int):
    """edge_index / batch vector of B copies of one graph (PyG Batch layout)."""
    E = edge_index.shape[1]
    dev = edge_index.device
    off = (torch.arange(B, device=dev) * num_nodes).repeat_interleave(E)
    ei = torch.stack([edge_index[0].repeat(B) + off, edge_index[1].repeat(B) + off])
    batch = torch.arange(B, device=dev).repeat_interleave(num_nodes)
    return ei, batch


class GradAllReduce:
    """One bucketed all-reduce (sum / world) of every gradient per update.

    The fused update (rl/fused_update.py) produces every gradient as a view of
    one flat buffer (agent.grad_flat): that buffer is reduced in place -- one
    RCCL call, no concatenation, no copy back.  Other paths (autograd) are
    concatenated into a bucket and copied back."""

    def __init__(self, world: int, agent=None):
        import torch.distributed as dist
        self.dist, self.world, self.agent = dist, world, agent
        self.calls = {"flat": 0, "bucket": 0}   # which path ran (tests)

    def _flat_of(self, grads):
        flat = getattr(self.agent, "grad_flat", None) if self.agent is not None else None
        if flat is None or not grads:
            return None
        base = flat.untyped_storage().data_ptr()
        lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * 4
        for g in grads:
            if g.untyped_storage().data_ptr() != base or not (lo <= g.data_ptr() < hi):
                return None
        return flat

    def __call__(self, grads):
        flat = self._flat_of(grads)
        if flat is not None:
            self.calls["flat"] += 1
            self.dist.all_reduce(flat)
            flat.div_(self.world)
            return
        self.calls["bucket"] += 1
        flat = torch.cat([g.reshape(-1) for g in grads])
        self.dist.all_reduce(flat)
        flat.div_(self.world)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n


def capture_graph(fn, pool=None):
    """torch.cuda.graph capture of fn() with the memset nodes rewritten into
    fill kernels before instantiation (trx_graph_patch_memsets: ROCm 7.2's
    packet-capture replay skips small memset nodes, which torch's multi-block
    reductions use to clear their semaphores).

    Capture mode thread_local: under data parallelism the process group's
    watchdog thread polls the HIP events of finished RCCL work (hipEventQuery)
    at any time; in the default global mode such a call from another thread
    during a capture fails with hipErrorStreamCaptureUnsupported and the
    watchdog aborts the rank (seen in tests/test_dist_gpu.py's RCCL test).
    Only this thread's capture-unsafe calls are checked."""
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with pinning() as pins, torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
        out = fn()
    # cached tensors (topologies, CSR, int32 indices) the captured kernels read
    # stay alive as long as the graph, whatever the caches evict later
    g.trx_pins = pins
    _lib.patch_graph_memsets(g)
    g.instantiate()
    return g, out


def graph_memset_replays_ok(device) -> bool:
    """Self-test of capture_graph: a captured 4-byte hipMemsetAsync followed
    by an add must start from the cleared value on every replay."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return False
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    z = torch.zeros(1, dtype=torch.int32, device=device)

    def body():
        hip.hipMemsetAsync(ctypes.c_void_p(z.data_ptr()), 0, 4, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        z.add_(1)

    g, _ = capture_graph(body)
    vals = []
    for _ in range(3):
        g.replay()
        vals.append(int(z.item()))
    return vals == [1, 1, 1]


class GraphedUpdate:
    """Trainer.update replayed from HIP graphs (torch.cuda.CUDAGraph).

    One SAC update at batch 256 is ~1500 small kernels; launched from Python
    it is host-bound (~25 ms).  After `warmup` eager updates (on a side
    stream: optimizer state, CSR/layout caches, allocator) the whole update --
    PER sample, HER relabel, six forwards, three backwards, clipping, the Adam
    steps, the Polyak update and the priority write-back -- is captured once
    and replayed.  The random draws stay outside the graph: they are written
    into static buffers before each replay, from the trainer's generator.
    With data parallelism the update is captured as two graphs around the
    gradient all-reduce, which runs eagerly (one RCCL call per update)."""

    def __init__(self, trainer: "Trainer", warmup: int = 3):
        self.tr, self.warmup, self.calls = trainer, warmup, 0
        self.g_grads = self.g_apply = None
        self.out = None
        self.side = torch.cuda.Stream(trainer.device)

    def __call__(self):
        tr = self.tr
        u, her_u = tr._draw_update_randoms()
        if self.g_grads is None and self.calls < self.warmup:
            self.side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                out = tr._update_once(u, her_u)
            torch.cuda.current_stream().wait_stream(self.side)
            self.calls += 1
            return out
        if self.g_grads is None:
            self._capture(u, her_u)
        self._replay()
        return self.out

    def _replay(self):
        self.g_grads.replay()
        if self.tr.agent.grad_sync is not None:
            self.tr.agent.grad_sync(self.tr.agent.gradients())
        if self.g_apply is not None:
            self.g_apply.replay()

    def _capture(self, u, her_u):
        tr = self.tr
        torch.cuda.synchronize(tr.device)
        split = tr.agent.grad_sync is not None
        def grads_part():
            s, out = tr._update_grads(u, her_u)
            if not split:
                tr._update_apply(s, out)
            return s, out

        g1, (s, out) = capture_graph(grads_part)
        if split:
            self.g_apply, _ = capture_graph(lambda: tr._update_apply(s, out), pool=g1.pool())
        self.g_grads, self.out = g1, out


class GraphedAct:
    """Trainer.act (stochastic, fused path) replayed from a HIP graph.

    Acting one vector step is ~10 kernels (prologue, three GAT layers, two
    GEMMs, the edge head with its in-kernel draw) plus the Python that builds
    their argument blocks; at 4096 environments the host side is as long as
    the kernels.  The graph reads the environment's persistent observation
    buffers, the actor's prepared-weight slots (refreshed in place, eagerly,
    when an update changed the weights: models/fused.py refresh_static) and a
    static buffer of uniforms, drawn from the trainer's generator before each
    replay exactly as the eager path draws them (same stream of numbers)."""

    def __init__(self, trainer: "Trainer"):
        self.tr = trainer
        self.g = self.key = self.out = None
        self.disabled = False
        self.u = torch.empty(trainer.B, device=trainer.device)

    def __call__(self, obs):
        tr = self.tr
        torch.rand(tr.B, device=tr.device, generator=tr.gen, out=self.u)
        key = (obs.node_x.data_ptr(), obs.edge_x.data_ptr(), obs.action_mask.data_ptr())
        if self.disabled:
            return tr._act(obs, u=self.u)
        fused.refresh_static(tr.agent.actor)
        if self.g is None or key != self.key:
            out = tr._act(obs, u=self.u)       # eager: caches (topology, slots), and which path runs
            if tr.agent.last_act_path != "fused":
                self.disabled = True
                return out
            torch.cuda.synchronize(tr.device)
            with fused.static_weights():
                self.g, self.out = capture_graph(lambda: tr._act(obs, u=self.u))
            self.key = key
            return out
        self.g.replay()
        return self.out


class Trainer:
    def __init__(self, cfg: Dict, device="cuda", rank: int = 0, world: int = 1, log: bool = True):
        self.cfg, self.rank, self.world = cfg, rank, world
        self.device = torch.device(device)
        # opt-in (cfg gemm_tuning: a TunableOp results file, e.g. GEMM_TUNING_GFX950)
        self.tuned_gemms = bool(cfg.get("gemm_tuning")) and self.device.type == "cuda" and \
            use_tuned_gemms(cfg["gemm_tuning"])
        torch.manual_seed(int(cfg["seed"]) + rank)
        np.random.seed(int(cfg["seed"]) + rank)
        self.gen = torch.Generator(device=self.device).manual_seed(int(cfg["seed"]) * 1000 + rank)
        self.logger = logging.getLogger("trafficrl.train")
        if log and rank == 0 and not self.logger.handlers:
            os.makedirs(os.path.join(cfg["output_dir"], "logs"), exist_ok=True)
            fh = logging.FileHandler(os.path.join(cfg["output_dir"], "logs", "training.log"))
            fh.setFormatter(logging.Formatter("%(asctime)s - %(message)s"))
            self.logger.addHandler(fh)
            self.logger.addHandler(logging.StreamHandler())
            self.logger.setLevel(logging.INFO)
        gd = (load_graph_data(cfg["net_path"], cfg["trips_path"]) if cfg.get("net_path") else sioux_falls())
        B = int(cfg["num_envs"])
        self.B = B
        seeds = [int(cfg["seed"]) * 100003 + rank * B + i for i in range(B)]
        self.env = VecRepairEnv(
            gd, B, device=self.device, damaged_ratio=cfg["damaged_ratio"], assignment_iters=cfg["assignment_iters"],
            assignment_method=cfg["assignment_method"], reward_mode=cfg["reward_mode"],
            reward_alpha=cfg["reward_alpha"], reward_beta=cfg["reward_beta"], reward_gamma=cfg["reward_gamma"],
            reward_clip=cfg["reward_clip"], capacity_damage=cfg["capacity_damage"],
            unassigned_penalty=cfg["unassigned_penalty"], fixed_damage=cfg["fixed_damage"],
            fixed_damage_seed=cfg["fixed_damage_seed"], seeds=seeds, reset=False, sp_backend=cfg["sp_backend"],
            force_gpu_sp=cfg["force_gpu_sp"], gp_step=cfg["gp_step"], gp_keep_paths=cfg["gp_keep_paths"])
        self.N, self.E = self.env.num_nodes, self.env.num_edges
        if not cfg["fixed_damage"] and self.device.type == "cuda":
            self.env.enable_damage_prefetch(True)   # next masks drawn on a host thread meanwhile
        amp = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(str(cfg.get("amp")).lower())
        self.use_graphs = bool(cfg.get("graph_update", True)) and self.device.type == "cuda"
        if self.use_graphs and not graph_memset_replays_ok(self.device):
            self.logger.warning("HIP graph memset replay self-test failed; SAC updates run eagerly")
            self.use_graphs = False
        self.agent = DiscreteSAC(
            4, 6, cfg["hidden_dim"], cfg["embed_dim"], num_layers=cfg["gat_layers"], lr=cfg["lr"],
            actor_lr=cfg["actor_lr"], critic_lr=cfg["critic_lr"], alpha_lr=cfg["alpha_lr"],
            grad_clip=cfg["grad_clip"], gamma=cfg["gamma"], target_tau=cfg["target_tau"],
            share_critic_encoder=cfg["share_critic_encoder"], alpha_init=cfg["alpha_init"],
            target_entropy_ratio=cfg["target_entropy_ratio"], device=self.device, amp_dtype=amp,
            capturable=self.use_graphs, fp32_actor=bool(cfg.get("fp32_actor", True)))
        if cfg.get("deterministic_update"):   # the update on one stream (same bits as the default, slower)
            self.agent.max_streams = 1
        if world > 1:
            import torch.distributed as dist
            for m in (self.agent.actor, self.agent.critic1, self.agent.critic2, self.agent.target1,
                      self.agent.target2):
                for t in list(m.parameters()) + list(m.buffers()):
                    dist.broadcast(t.data, src=0)
            dist.broadcast(self.agent.log_alpha.data, src=0)
            self.agent.grad_sync = GradAllReduce(world, self.agent)
        cap = min(int(cfg["buffer_size"]), max(int(cfg["buffer_size"]) // world, B))
        self.replay = DeviceReplay(cap, self.N, self.E, alpha=cfg["per_alpha"], beta=cfg["per_beta"],
                                   eps=cfg["per_eps"], device=self.device, tree_dtype=cfg["per_tree"])
        # the float32 tree's ring adds beside the next acting pass (same results: the adds
        # keep their order on their own stream; updates join them first)
        self.replay.overlap_adds = self.device.type == "cuda" and bool(cfg.get("overlap_per_adds", True)) and \
            os.environ.get("TRX_PER_OVERLAP", "1") != "0"
        ei = self.env.edge_index
        self.act_ei, self.act_batch = batched_topology(ei, self.N, B)
        bs = int(cfg["batch_size"])
        self.upd_ei, self.upd_batch = batched_topology(ei, self.N, bs)
        self.upd_act_off = torch.arange(bs, device=self.device) * self.E   # graph offsets of the batch's actions
        self.fixed_mask = None
        # per-env episode accumulators (device)
        self.ep_reward = torch.zeros(B, dtype=torch.float64, device=self.device)
        self.ep_tstt_sum = torch.zeros(B, dtype=torch.float64, device=self.device)
        self.ep_auc = torch.zeros(B, dtype=torch.float64, device=self.device)
        self.ep_prev_tstt = torch.zeros(B, dtype=torch.float64, device=self.device)
        self.ep_len = torch.zeros(B, dtype=torch.int64, device=self.device)
        # per-step outputs of trx_episode_step (scaled reward f64 / f32, done as float, finished)
        self._scaled = torch.zeros(B, dtype=torch.float64, device=self.device)
        self._scaled32 = torch.zeros(B, dtype=torch.float32, device=self.device)
        self._done32 = torch.zeros(B, dtype=torch.float32, device=self.device)
        self._finished = torch.zeros(B, dtype=torch.uint8, device=self.device)
        self.episodes_done = 0
        self.updates_done = 0
        self.history = []
        self.last_losses: Dict = {}
        self._u = torch.empty(bs, dtype=torch.float64, device=self.device)      # PER draws
        self._her_u = torch.empty(bs, dtype=torch.float32, device=self.device)  # HER draws
        self._graphed = GraphedUpdate(self) if self.use_graphs else None
        self._graphed_act = GraphedAct(self) if self.use_graphs and cfg.get("graph_act", True) else None
        self._transitions = 0   # env transitions added so far (update schedule)
        self._due_carry = 0     # world > 1: summed due updates not yet dealt out

    # ------------------------------------------------------------ acting
    def act(self, obs, deterministic=False):
        if self._graphed_act is not None and not deterministic:
            return self._graphed_act(obs)
        return self._act(obs, deterministic)

    def _act(self, obs, deterministic=False, u=None):
        B = self.B
        return self.agent.select_actions(obs.node_x.reshape(B * self.N, 4), self.act_ei,
                                         obs.edge_x.reshape(B * self.E, 6), obs.action_mask.reshape(-1),
                                         self.act_batch, num_graphs=B, deterministic=deterministic,
                                         generator=self.gen, u=u)

    def _reset_envs(self, done_mask: Optional[torch.Tensor]):
        env = self.env
        if done_mask is None:
            env.reset(observe=False)
            if self.cfg["fixed_damage"]:
                self.fixed_mask = env.damaged[:1].clone()
            self.ep_prev_tstt.copy_(env.tstt)
            return
        if self.cfg["fixed_damage"] and self.fixed_mask is not None:
            # every env has the same damage: reset on device, no host round trip
            env.reset_where(done_mask, self.fixed_mask.expand(self.B, -1))
        else:
            ids = torch.nonzero(done_mask).squeeze(1).tolist()
            if len(ids) == self.B:   # every env at once: the prefetched draw (enable_damage_prefetch)
                env.reset(observe=False)
            elif ids:
                env.reset(env_ids=ids, observe=False)
        self.ep_prev_tstt = torch.where(done_mask, env.tstt, self.ep_prev_tstt)

    # ------------------------------------------------------------ update
    def update(self):
        """One SAC update on a PER batch (src/train.py:954-1024 update block)."""
        self.replay.sync_adds()   # the tree adds of the last iterations (side stream) before the sample
        if self._graphed is not None:
            out = self._graphed()
        else:
            out = self._update_once(*self._draw_update_randoms())
        fused.weights_changed()   # a graph replay changes parameters without bumping their versions
        self.last_losses = out
        self.updates_done += 1
        return out

    def _draw_update_randoms(self):
        self._u.uniform_(generator=self.gen)
        if self.cfg["her_ratio"] > 0:
            self._her_u.uniform_(generator=self.gen)
        return self._u, self._her_u

    def _update_once(self, u, her_u):
        s, out = self._update_grads(u, her_u)
        if self.agent.grad_sync is not None:
            self.agent.grad_sync(self.agent.gradients())
        self._update_apply(s, out)
        return out

    def _update_grads(self, u, her_u):
        cfg = self.cfg
        bs = int(cfg["batch_size"])
        s = self.replay.sample(bs, u=u)
        s = her_relabel(s, cfg["her_ratio"], cfg["reward_mode"], cfg["reward_scale"], cfg["reward_alpha"],
                        cfg["reward_beta"], cfg["reward_gamma"], cfg["reward_clip"], u=her_u)
        E, N = self.E, self.N
        action = self.upd_act_off + s.action
        batch = (s.node_x.reshape(bs * N, -1), self.upd_ei, s.edge_x.reshape(bs * E, -1), s.mask.reshape(-1),
                 self.upd_batch, action, s.reward, s.next_node_x.reshape(bs * N, -1), s.next_edge_x.reshape(bs * E, -1),
                 s.next_mask.reshape(-1), self.upd_batch, s.done)
        # the priority write-back (src/train.py:1017-1019) reads only the TD errors and
        # touches only the replay tree: it runs beside the backward passes
        out = self.agent.compute_gradients(batch, weights=s.weights,
                                           on_td=lambda td: self.replay.update_priorities(s.idx, td))
        return s, out

    def _update_apply(self, s, out):
        self.agent.apply_gradients(self.cfg.get("alpha_max"))

    def updates_due(self, it: int) -> int:
        """SAC updates to run after iteration `it` (its B transitions added).

        update_unit "transitions" (default) follows the reference's serial
        loop (src/train.py:915-955) per env: each env keeps its own episode
        step counter (ep_len, reset with the episode, like `steps = 0` at
        train.py:919); after an env's step, `updates_per_step` updates are due
        when ep_len % update_every == 0 -- except on a step that truncates the
        episode (max_steps reached and not done: the reference breaks out of
        the episode before its update check, 950-952).  The iteration's count
        is the sum over envs, so B = 1 reproduces the reference's schedule
        (e.g. 5 updates per 22-step episode at update_every 4).
        update_unit "iterations": `updates_per_step` updates every
        `update_every` vector iterations (B transitions each) -- the bench's
        throughput workload, a UTD ratio B * update_every times lower.
        No update until the replay holds more than batch_start transitions."""
        cfg = self.cfg
        ups, every = int(cfg["updates_per_step"]), int(cfg["update_every"])
        self._transitions += self.B
        if self.replay.size <= int(cfg["batch_start"]):
            return 0
        if str(cfg.get("update_unit", "transitions")) == "iterations":
            return ups if it % every == 0 else 0
        due = (self.ep_len % every) == 0
        ms = int(cfg["max_steps"])
        if ms > 0:
            # env.done is uint8: ~ on it would be a bitwise not (255/254)
            due &= ~((self.ep_len >= ms) & ~self.env.done.bool())
        n = due.sum()
        if self.world > 1:
            # every rank must run the same number of updates (each one all-reduces
            # its gradients): the ranks' due counts are summed and dealt out evenly,
            # the remainder carried to the next iteration -- the same on every rank
            import torch.distributed as dist
            n = n.to(torch.int64).reshape(1)
            dist.all_reduce(n)
            self._due_carry += int(n.item()) * ups
            k = self._due_carry // self.world
            self._due_carry -= k * self.world
            return k
        return int(n.item()) * ups

    def prime_update(self):
        """Run the eager warm-up updates and the HIP-graph capture now, so that
        later updates are graph replays (a steady-state timed region never
        contains an eager update or a capture)."""
        if self._graphed is None:
            return
        while self._graphed.g_grads is None:
            self.update()
        self.update()
        torch.cuda.synchronize(self.device)

    # -------------------------------------------------------------- loop
    def iteration(self, obs, it: int):
        cfg, env = self.cfg, self.env
        actions = self.act(obs)
        # pre-step fields go straight into the replay ring (no clones) unless the slots wrap
        staged = self.replay.stage_prev(obs.node_x, obs.edge_x, obs.action_mask, env.goal, env.tstt)
        if not staged:
            prev_obs = (obs.node_x.clone(), obs.edge_x.clone(), obs.action_mask.clone())
            goal = env.goal.clone()
            prev_tstt = env.tstt.clone()
        next_obs, reward, done, info = env.step(actions.to(torch.int32), check=False)
        if self.device.type == "cuda":
            # reward scaling + episode stats + truncation: one trx_episode_step launch
            L = _lib.load()
            _lib.check(L.trx_episode_step(self.B, _lib.ptr(env.reward), _lib.ptr(env.done), _lib.ptr(env.tstt),
                                          float(cfg["reward_scale"]), int(cfg["max_steps"]), _lib.ptr(self._scaled),
                                          _lib.ptr(self._scaled32), _lib.ptr(self._done32), _lib.ptr(self.ep_reward),
                                          _lib.ptr(self.ep_tstt_sum), _lib.ptr(self.ep_auc),
                                          _lib.ptr(self.ep_prev_tstt), _lib.ptr(self.ep_len), _lib.ptr(self._finished),
                                          _lib.stream_ptr(self.device)), "trx_episode_step")
            scaled, done_f = self._scaled32, self._done32
            finished = self._finished.view(torch.bool)
        else:
            scaled = reward * cfg["reward_scale"]
            self.ep_len += 1
            trunc = (self.ep_len >= int(cfg["max_steps"])) if cfg["max_steps"] > 0 else torch.zeros_like(done)
            self.ep_reward += scaled
            self.ep_tstt_sum += env.tstt
            self.ep_auc += 0.5 * (self.ep_prev_tstt + env.tstt) * (self.ep_len > 1)
            self.ep_prev_tstt.copy_(env.tstt)
            done_f = done.float()
            finished = done | trunc
        if staged:
            self.replay.add_staged(actions, scaled, next_obs.node_x, next_obs.edge_x, next_obs.action_mask,
                                   done_f, env.tstt, env.initial_tstt)
        else:
            self.replay.add_batch(prev_obs[0], prev_obs[1], prev_obs[2], actions, scaled, next_obs.node_x,
                                  next_obs.edge_x, next_obs.action_mask, done_f, goal, prev_tstt, env.tstt,
                                  env.initial_tstt)
        for _ in range(self.updates_due(it)):
            self.update()
        return next_obs, finished

    def _gather_episodes(self, finished: torch.Tensor):
        """Per-episode metrics of the envs that finished this iteration, over
        ALL ranks (env order: rank-major, env id within a rank), so that every
        rank takes the same stop / eval / patience decisions.  Columns: mask,
        reward, tstt_mean, tstt_last, auc."""
        f = finished
        ln = torch.clamp(self.ep_len, min=1).to(torch.float64)
        rows = torch.stack([f.to(torch.float64), self.ep_reward, self.ep_tstt_sum / ln, self.env.tstt,
                            self.ep_auc], dim=1)
        if self.world > 1:
            import torch.distributed as dist
            parts = [torch.empty_like(rows) for _ in range(self.world)]
            dist.all_gather(parts, rows)
            rows = torch.cat(parts)
        rows = rows[rows[:, 0] > 0].cpu().numpy()
        return rows

    def record(self, finished: torch.Tensor):
        """Book the finished episodes (all ranks) into history; returns their
        per-episode rows (see _gather_episodes)."""
        rows = self._gather_episodes(finished)
        n = len(rows)
        f = finished
        for t in (self.ep_reward, self.ep_tstt_sum, self.ep_auc):
            t.masked_fill_(f, 0.0)
        self.ep_len.masked_fill_(f, 0)
        if n == 0:
            return rows
        rec = {"episodes": n, "reward": float(rows[:, 1].mean()), "tstt_mean": float(rows[:, 2].mean()),
               "tstt_last": float(rows[:, 3].mean()), "auc": float(rows[:, 4].mean())}
        self.episodes_done += n
        self.history.append(rec)
        return rows

    def _any_finished(self, finished: torch.Tensor) -> bool:
        """finished.any() over all ranks (one tiny all-reduce per iteration
        when world > 1; the single-GPU path syncs on the flag as before)."""
        flag = finished.any().to(torch.int32).reshape(1)
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return bool(flag.item())

    def evaluate(self, seeds=None) -> Dict:
        """Deterministic-policy episodes (src/train.py:590-664) on a separate env."""
        cfg = self.cfg
        seeds = seeds or cfg["eval_seeds"]
        ev = VecRepairEnv(self.env.graph_data, len(seeds), device=self.device, graph=self.env.graph,
                          damaged_ratio=cfg["damaged_ratio"], assignment_iters=cfg["assignment_iters"],
                          assignment_method=cfg["assignment_method"], reward_mode=cfg["reward_mode"],
                          reward_alpha=cfg["reward_alpha"], reward_beta=cfg["reward_beta"],
                          reward_gamma=cfg["reward_gamma"], reward_clip=cfg["reward_clip"],
                          capacity_damage=cfg["capacity_damage"], unassigned_penalty=cfg["unassigned_penalty"],
                          fixed_damage=cfg["fixed_damage"], fixed_damage_seed=cfg["fixed_damage_seed"],
                          seeds=list(seeds), reset=False, sp_backend=cfg["sp_backend"],
                          force_gpu_sp=cfg["force_gpu_sp"], gp_step=cfg["gp_step"],
                          gp_keep_paths=cfg["gp_keep_paths"])
        obs = ev.reset()
        n = len(seeds)
        ei, bv = batched_topology(ev.edge_index, self.N, n)
        curves = []
        done_all = torch.zeros(n, dtype=torch.bool, device=self.device)
        for _ in range(int(cfg["max_steps"]) or 10 ** 6):
            a = self.agent.select_actions(obs.node_x.reshape(-1, 4), ei, obs.edge_x.reshape(-1, 6),
                                          obs.action_mask.reshape(-1), bv, num_graphs=n, deterministic=True)
            obs, _, done, _ = ev.step(a.to(torch.int32), check=False)
            curves.append(torch.where(done_all, torch.full_like(ev.tstt, float("nan")), ev.tstt))
            done_all |= done
            if bool(done_all.all()):
                break
        c = torch.stack(curves).cpu().numpy()
        auc = [float(np.trapezoid(c[~np.isnan(c[:, k]), k])) for k in range(n)]
        return {"tstt_last": float(np.nanmean([c[~np.isnan(c[:, k]), k][-1] for k in range(n)])),
                "tstt_mean": float(np.nanmean(c)), "auc": float(np.mean(auc))}

    def save(self, tag: str):
        if self.rank == 0:
            os.makedirs(self.cfg["output_dir"], exist_ok=True)
            self.agent.save(os.path.join(self.cfg["output_dir"], f"model_{tag}.pt"))

    def run(self, max_iters: Optional[int] = None):
        """Training loop (src/train.py:915-1041 serial path, vectorised).
        Early stopping follows the reference per finished episode: an episode
        whose TSTT mean beats the best by early_stop_min_delta resets the
        patience, any other adds one; stop at early_stop_patience.  Episodes
        are taken in a fixed (rank, env id) order from all ranks, so every
        rank stops at the same iteration (no rank is left in an all-reduce)."""
        cfg = self.cfg
        self._reset_envs(None)
        obs = self.env.observe()
        best, patience = math.inf, 0
        min_delta = float(cfg.get("early_stop_min_delta", 0.0) or 0.0)
        t0 = time.perf_counter()
        it = 0
        next_eval = int(cfg["eval_every"])
        stop = False
        while self.episodes_done < int(cfg["episodes"]) and not stop:
            if max_iters is not None and it >= max_iters:
                break
            obs, finished = self.iteration(obs, it)
            it += 1
            if not self._any_finished(finished):
                continue
            rows = self.record(finished)
            self._reset_envs(finished)
            obs = self.env.observe()
            if len(rows) == 0:
                continue
            rec = self.history[-1]
            if self.rank == 0:
                self.logger.info(f"it {it} episodes {self.episodes_done} reward {rec['reward']:.3f} "
                                 f"tstt_mean {rec['tstt_mean']:.2f} auc {rec['auc']:.1f} "
                                 f"steps/s {it * self.B * self.world / (time.perf_counter() - t0):.0f}")
            for tm in rows[:, 2]:   # train.py:1031-1041, one finished episode at a time
                if tm < best - min_delta:
                    best, patience = float(tm), 0
                else:
                    patience += 1
                if patience >= int(cfg["early_stop_patience"]):
                    stop = True
                    if self.rank == 0:
                        self.logger.info(f"Early stopping at episode {self.episodes_done}: no TSTT-mean "
                                         f"improvement for {patience} episodes")
                    break
            if not stop and self.episodes_done >= next_eval and cfg["eval_every"] > 0:
                # evaluations happen at iteration granularity: the next one after the
                # next multiple of eval_every episodes (src/train.py evaluates every
                # eval_every episodes; many envs finish episodes together here)
                next_eval = (self.episodes_done // int(cfg["eval_every"]) + 1) * int(cfg["eval_every"])
                ev = self.evaluate()
                if self.rank == 0:
                    self.logger.info(f"eval {ev}")
                self.save("last")
        self.save("last")
        if self.rank == 0:
            with open(os.path.join(cfg["output_dir"], "train_metrics.json"), "w") as fh:
                json.dump(self.history, fh)
        return self.history


def main(argv=None):
    ap = argparse.ArgumentParser(description="vectorised GAT-SAC training (src/train.py equivalent)")
    ap.add_argument("--config", default=SF_CONFIG)
    ap.add_argument("--num-envs", type=int, default=None)
    ap.add_argument("--episodes", type=int, default=None)
    ap.add_argument("--max-iters", type=int, default=None)
    args = ap.parse_args(argv)
    cfg = load_config(args.config)
    if args.num_envs:
        cfg["num_envs"] = args.num_envs
    if args.episodes:
        cfg["episodes"] = args.episodes
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    tr = Trainer(cfg, device=f"cuda:{local}", rank=rank, world=world)
    tr.run(args.max_iters)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmark: env steps/s (= full BPR user-equilibrium assignments/s) of N
vectorised Sioux Falls repair envs per MI355X (BASELINE.json configs[1]:
4096 envs, MSA 30 iterations, SAC+GAT bf16).

Default workload `train` (configs[1]): one step = the GAT-SAC actor (bf16
autocast) picks an action for every env from its observation, RepairEnv.step
runs for all envs (src/env/repair_env.py:207-237: repair, 30-iteration MSA
assignment, reward, done, get_state 751-819), transitions go to the device
PER replay, and every 4 steps one SAC update on a 256-graph PER batch
(src/train.py:954-1024).  Workload `env`: the same env steps with uniform
random valid actions (no agent).  Damage: fixed_damage_seed=42 for all envs;
episodes are 22 steps and all envs auto-reset together (the reset assignment
is inside the timed region but not counted as a step).

Multi-GPU: one process per GPU (torchrun), envs sharded with no data-path
collective (weak scaling); max elapsed over ranks; value = all ranks' steps /
that time.

Prints ONE JSON line on rank 0 (driver contract), with
  roofline:     algorithmic bytes per env_kernel launch (SURVEY.md §8(d):
                bytes(assign) x envs) / the kernel's mean duration measured
                with HIP events on its stream, vs 8 TB/s HBM peak;
  cpu_baseline: the C restatement (oracle/, kind "port") timed on host cores
                on a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env steps/sec (full BPR assigns/sec), N vectorised Sioux Falls envs, 1/2/4/8 GPU"
HBM_PEAK = 8.0e12  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)


def bytes_per_assign(N, E, Z, P, K):
    """SURVEY.md §8(d) algorithmic bytes of one full assignment (4-byte elements)."""
    return (K + 1) * 20 * E + K * (Z * (8 * E + 12 * N) + 4 * P + 4 * E + 12 * E) + 8 * E


NETWORKS = {
    # name: (GraphData loader, golden graph arrays for the CPU baseline, label)
    "sf": ("sioux_falls", "sf_graph.npz", "SiouxFalls (24 nodes, 76 links, 528 OD)"),
    "anaheim": ("anaheim_synthetic", "ana_graph.npz",
                "AnaheimSynth (seeded synthetic Anaheim-size: 416 nodes, 914 links, 38 zones, 1076 OD)"),
}


def load_network(name):
    import trafficrl.data as D
    return getattr(D, NETWORKS[name][0])()


def fixed_damage_mask(gd, seed=42, ratio=0.3):
    from trafficrl.graph import DamageSampler

    class _G:
        num_edges = len(gd.edges)
        num_nodes = gd.num_nodes
        src = np.array([e.u - 1 for e in gd.edges], np.int32)
        dst = np.array([e.v - 1 for e in gd.edges], np.int32)

    return DamageSampler(_G, 0, fixed_damage=True, fixed_damage_seed=seed).sample(ratio)


def cpu_baseline(network, method, iters, seconds=12.0):
    """Time the oracle's C restatement (same algorithm: scipy-order Dijkstra,
    predecessor path walk, fp32 MSA/FW) on the host cores, warm-started
    steps of the fixed-damage env (one assignment each)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only

    npz = os.path.join(ROOT, "tests", "golden", NETWORKS[network][1])
    og = O.OracleGraph.from_npz(npz)
    gr = np.load(npz)
    E = og.E
    dmg = fixed_damage_mask(load_network(network))
    cap = np.where(dmg > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)
    f0, _, _, _ = og.assign(cap, dmg, np.zeros(E, np.float32), method=method, iters=iters)
    threads = max(1, min(16, os.cpu_count() or 1, O.max_threads()))
    # repair one random damaged link per row, warm start from the reset flow
    rng = np.random.default_rng(7)
    B = (64 if network == "sf" else 4) * threads
    cand = np.where(dmg > 0)[0]
    C = np.repeat(cap[None], B, 0)
    D = np.repeat(dmg[None], B, 0)
    a = rng.choice(cand, B)
    C[np.arange(B), a] = gr["cap0"][a]
    D[np.arange(B), a] = 0.0
    F = np.repeat(f0[None], B, 0)
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        og.assign(C, D, F, method=method, iters=iters, nthreads=threads)
        done += B
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "env steps/s", "cores": threads, "kind": "port",
            "sample": f"{done} warm-started {method.upper()}-{iters} steps ({network}, fixed damage seed 42, one repaired "
                      f"link each) in {dt:.1f}s on {threads} host threads; oracle/trx_oracle.c"}


def measured_traffic(network):
    """HBM bytes per env-kernel launch from the committed rocprofv3 PMC summary
    of this workload (profiles/r01_v3_pmc.json for Sioux Falls,
    profiles/r01_ana_pmc.json for the Anaheim-size network; separate
    FETCH_SIZE / WRITE_SIZE passes, see tools/pmc_summary.py)."""
    name = {"sf": "r01_v3_pmc.json", "anaheim": "r01_ana_pmc.json"}[network]
    path = os.path.join(ROOT, "profiles", name)
    try:
        d = json.load(open(path))
        return d.get("hbm_bytes_per_launch_raw"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=66)
    ap.add_argument("--warmup", type=int, default=22)
    ap.add_argument("--network", default="sf", choices=sorted(NETWORKS),
                    help="sf = Sioux Falls (configs #1-#4); anaheim = config #5's 416-node network (env workload, "
                         "1024 envs, FW by default)")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default 4096 sf / 1024 anaheim)")
    ap.add_argument("--method", default=None, choices=["msa", "fw", "cfw"], help="default msa (sf) / fw (anaheim)")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--no-observe", action="store_true", help="skip get_state (assignment-only steps)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workload", default=None, choices=["train", "env"], help="default train (sf) / env (anaheim)")
    args = ap.parse_args()
    big = args.network != "sf"
    if args.envs is None:
        args.envs = 1024 if big else 4096
    if args.method is None:
        args.method = "fw" if big else "msa"
    if args.workload is None:
        args.workload = "env" if big else "train"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU; TRX_DIST_BACKEND=gloo rehearses the multi-rank path on
    # fewer GPUs than ranks (ranks then share devices: local % device_count)
    backend = os.environ.get("TRX_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()) if world > 1 else 0)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)

    from trafficrl.env import VecRepairEnv

    B = args.envs
    gd = load_network(args.network)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    observe = not args.no_observe
    ev_pairs = []      # env_kernel launches (HIP events on the launch stream)
    phase_ev = {}      # per-phase events (train workload)

    def timed(fn, bucket):
        s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s_.record()
        out = fn()
        e_.record()
        bucket.append((s_, e_))
        return out

    if args.workload == "train":
        from trafficrl.train import Trainer, load_config
        cfg = load_config(None)
        cfg.update(num_envs=B, assignment_iters=args.iters, assignment_method=args.method, batch_start=256,
                   batch_size=256, update_every=4, updates_per_step=1, eval_every=0, episodes=10 ** 9,
                   output_dir=os.path.join("/tmp", f"trx_bench_{os.getpid()}"), amp="bf16")
        tr = Trainer(cfg, device=dev, rank=rank, world=world, log=False)
        env = tr.env
        raw_step, raw_act, raw_update = env.step, tr.act, tr.update

        def step_w(actions, observe=True, check=True):
            _, rew, done, info = timed(lambda: raw_step(actions, observe=False, check=check), ev_pairs)
            return (env.observe() if observe else None), rew, done, info

        env.step = step_w
        tr.act = lambda *a, **k: timed(lambda: raw_act(*a, **k), phase_ev.setdefault("act", []))
        tr.update = lambda *a, **k: timed(lambda: raw_update(*a, **k), phase_ev.setdefault("update", []))
        tr._reset_envs(None)
        E, N = env.num_edges, env.num_nodes
        dmg_all = tr.fixed_mask.expand(B, E).contiguous()
        ep_len = int(tr.fixed_mask.sum().item())
        all_true = torch.ones(B, dtype=torch.bool, device=dev)
        st = {"obs": env.observe(), "it": 0, "t": 0}

        def reset():
            timed(lambda: env.reset_where(all_true, dmg_all), ev_pairs)
            st["obs"] = env.observe()
            st["t"] = 0
            for acc in (tr.ep_reward, tr.ep_tstt_sum, tr.ep_auc, tr.ep_len):
                acc.zero_()
            tr.ep_prev_tstt.copy_(env.tstt)

        def one_step():
            st["obs"], _ = tr.iteration(st["obs"], st["it"])
            st["it"] += 1
            st["t"] += 1
            if st["t"] == ep_len:
                reset()
    else:
        env = VecRepairEnv(gd, B, device=dev, assignment_method=args.method, assignment_iters=args.iters,
                           reward_mode="rel_improve", reward_alpha=1.0, reward_beta=0.0, reward_gamma=0.0,
                           reward_clip=2.0, capacity_damage=1e-3, unassigned_penalty=1e4, reset=False)
        E, N = env.num_edges, env.num_nodes
        dmg0 = torch.from_numpy(fixed_damage_mask(gd)).to(dev)
        dmg_all = dmg0[None].expand(B, E).contiguous()
        ep_len = int(dmg0.sum().item())
        st = {"t": 0}

        def reset():
            timed(lambda: env.reset(damaged=dmg_all, observe=False), ev_pairs)
            if observe:
                env.observe()
            st["t"] = 0

        def one_step():
            scores = torch.rand(B, E, device=dev, generator=gen) * env.damaged
            actions = scores.argmax(dim=1).to(torch.int32)
            timed(lambda: env.step(actions, observe=False, check=False), ev_pairs)
            if observe:
                env.observe()
            st["t"] += 1
            if st["t"] == ep_len:
                reset()

        reset()
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    ev_pairs.clear()
    for v in phase_ev.values():
        v.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    breakdown = {k: float(np.sum([s_.elapsed_time(e_) for s_, e_ in v])) / args.steps for k, v in phase_ev.items()}
    kern_ms = [s.elapsed_time(e) for s, e in ev_pairs]
    mean_kernel_s = float(np.mean(kern_ms)) / 1e3 if kern_ms else float("nan")
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        k = torch.tensor([mean_kernel_s], device=dev, dtype=torch.float64)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        mean_kernel_s = float(k.item())

    total_steps = args.steps * B * world
    value = total_steps / elapsed
    Z = env.graph.num_origins
    P = len(env.graph.od_o)
    bpa = bytes_per_assign(N, E, Z, P, args.iters)
    achieved = bpa * B / mean_kernel_s
    traffic, traffic_src = measured_traffic(args.network)
    if (args.envs, args.iters, args.method) != ((1024, 30, "fw") if big else (4096, 30, "msa")):
        traffic, traffic_src = None, None  # the committed PMC passes are for the default workloads
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(args.network, args.method, args.iters, args.cpu_seconds)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (link flows/costs) + f64 (path labels)" + (
                "; bf16 autocast GAT-SAC" if args.workload == "train" else ""),
            "data": (f"synthetic: {'Sioux Falls TNTP' if not big else 'seeded AnaheimSynth TNTP'}, "
                     "fixed_damage_seed=42, " + ("random-init GAT-SAC (hidden 256, 4 heads, embed 256)"
                                                 if args.workload == "train" else "uniform random valid repair actions")),
            "config": {
                "workload": (f"{'SF' if not big else 'AnaheimSynth'} {B} vectorised envs/GPU, {args.method.upper()}-{args.iters} assignment + get_state per"
                             " step" + (", GAT-SAC bf16 acting every step + 1 PER update (batch 256) every 4 steps"
                                        if args.workload == "train" else ", uniform random valid actions")),
                "workload_kind": args.workload,
                "envs_per_gpu": B, "global_envs": B * world, "network": NETWORKS[args.network][2],
                "method": args.method, "assignment_iters": args.iters, "episode_len": ep_len,
                "parallelism": f"env-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": traffic,
                "traffic_note": (f"rocprofv3 FETCH_SIZE+WRITE_SIZE per launch, {traffic_src} "
                                 "(raw; 4-byte loads, gfx950 x2 fetch correction not applied)") if traffic else None,
                "kernel": "trx::env_kernel_big" if big else "trx::env_kernel_q<24>", "kernel_mean_ms": mean_kernel_s * 1e3,
                "bytes_per_assign": bpa, "assigns_per_launch": B,
            },
            "cpu_baseline": cpu,
            "breakdown_ms_per_step": dict(breakdown, env_kernel=mean_kernel_s * 1e3 * len(kern_ms) / args.steps),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

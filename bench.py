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


def host_cores():
    """(cores this job may use, CPUs visible).  Usable = the CPU affinity set,
    capped by the cgroup CPU quota and by OMP_NUM_THREADS when the launcher
    sets it: a GPU box hands each 1-GPU job a 16-core share of a larger host
    (nproc shows the whole host there), and the baseline uses all of that share."""
    try:
        vis = len(os.sched_getaffinity(0))
    except AttributeError:
        vis = os.cpu_count() or 1
    n = vis
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n), vis


def sac_update_flops(bs, N, E, hidden=256, heads=4, embed=256, edge_in=6):
    """Dense GEMM FLOPs of one SAC update (src/rl/sac.py:157-243) at batch bs
    with this build's per-node factoring of the edge MLP: per graph forward the
    GAT lin layers (4 -> H*C is negligible), the edge head's node projection
    and context product, the link-feature product; 6 forwards (next actor, 2
    targets, 2 critics, actor) + 3 backwards at 2x their forward."""
    hc = heads * hidden
    per_graph = 2 * N * (hc * hc + hc * embed + embed * 2 * hidden) + 2 * (2 * embed * hidden) + 2 * E * edge_in * hidden
    return float(bs * per_graph * (6 + 3 * 2))


def cpu_baseline(network, method, iters, seconds=12.0, sp="scipy"):
    """Time the oracle's C restatement (same algorithm as the reference:
    scipy-order Dijkstra or the torch rule's Floyd-Warshall, predecessor /
    next-hop path walk, fp32 MSA/FW, then get_state with networkx-order
    Brandes betweenness) on all host cores available to this process
    (OpenMP over envs): warm-started env steps of the fixed-damage env, one
    assignment + one observation each -- the same per-step env work as the
    GPU env kernel + observe kernel.  The assignment-only rate is reported
    beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only

    npz = os.path.join(ROOT, "tests", "golden", NETWORKS[network][1])
    og = O.OracleGraph.from_npz(npz)
    gr = np.load(npz)
    E = og.E
    dmg = fixed_damage_mask(load_network(network))
    cap = np.where(dmg > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)
    f0, _, _, _ = og.assign(cap, dmg, np.zeros(E, np.float32), method=method, iters=iters, sp=sp)
    threads, visible = host_cores()
    # repair one random damaged link per row, warm start from the reset flow
    rng = np.random.default_rng(7)
    B = (64 if network == "sf" else 4) * threads
    cand = np.where(dmg > 0)[0]
    C = np.repeat(cap[None], B, 0)
    D = np.repeat(dmg[None], B, 0)
    G = D.copy()
    a = rng.choice(cand, B)
    C[np.arange(B), a] = gr["cap0"][a]
    D[np.arange(B), a] = 0.0
    F = np.repeat(f0[None], B, 0)
    done = 0
    t_assign = t_obs = 0.0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ta = time.perf_counter()
        fo, _, ts, _ = og.assign(C, D, F, method=method, iters=iters, nthreads=threads, sp=sp)
        tb = time.perf_counter()
        og.observe(C, D, G, fo, ts, nthreads=threads)
        t_obs += time.perf_counter() - tb
        t_assign += tb - ta
        done += B
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "env steps/s", "cores": threads, "kind": "port",
            "assign_only": done / t_assign, "host_cpus_visible": visible,
            "sample": f"{done} warm-started {method.upper()}-{iters} env steps ({network}, {sp} shortest-path rule, "
                      f"fixed damage seed 42, one repaired link each): assignment + get_state, in {dt:.1f}s on "
                      f"{threads} host threads (all cores available to the process); assignment alone "
                      f"{t_assign:.1f}s, get_state {t_obs:.1f}s; oracle/trx_oracle.c"}


MFMA_PEAK_BF16 = 2.5e15  # MI355X_MICROARCH.md: dense bf16 MFMA peak (no sparsity)


def gemm_mfma(rows, graphs, hidden=256, heads=4, embed=256, reps=20):
    """MFMA utilisation of the acting pass's dense GEMMs:
    the same bf16 torch.mm shapes trafficrl/models/fused.py issues per 4096-graph
    forward -- layer-1 lin [rows, H*C] x [H*C, H*C]^T, layer-2 lin
    [rows, H*C] x [embed, H*C]^T, the edge head's per-node projection
    [rows, embed] x [2*hidden, embed]^T and the context product
    [graphs, 2*embed] x [2*embed, hidden] -- timed with HIP events on the
    current stream; FLOPs (2mnk) / time vs the dense bf16 MFMA peak."""
    dev = torch.device("cuda", torch.cuda.current_device())
    bf = dict(dtype=torch.bfloat16, device=dev)
    hc = heads * hidden
    shapes = [(rows, hc, hc), (rows, hc, embed), (rows, embed, 2 * hidden), (graphs, 2 * embed, hidden)]
    ops = []
    for m, k, n in shapes:
        a, w = torch.randn(m, k, **bf), torch.randn(n, k, **bf)
        ops.append((a, w, 2.0 * m * n * k))
    for a, w, _ in ops:
        torch.mm(a, w.t())
    torch.cuda.synchronize()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    for _ in range(reps):
        for a, w, _ in ops:
            torch.mm(a, w.t())
    e_.record()
    torch.cuda.synchronize()
    sec = s_.elapsed_time(e_) / 1e3 / reps
    flops = sum(f for _, _, f in ops)
    return {"gemms": "act-pass lin GEMMs, bf16 hipBLASLt: " + ", ".join(f"{m}x{k}x{n}" for m, k, n in shapes),
            "flops_per_pass": flops, "ms_per_pass": sec * 1e3, "achieved": flops / sec / 1e12,
            "peak": MFMA_PEAK_BF16 / 1e12, "unit": "TFLOP/s", "frac": flops / sec / MFMA_PEAK_BF16}


def lib_sha16():
    """First 16 hex digits of sha256(libtrafficrl.so) -- the binary this process loads."""
    import hashlib
    from trafficrl import _lib
    with open(_lib.LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


PMC_SUMMARIES = {"sf": "r06_sf_pmc.json", "anaheim": "r05_ana_pmc.json"}


def measured_traffic(network, kname):
    """HBM bytes per env-kernel launch and the VALU / LDS-conflict shares from
    the committed rocprofv3 PMC summary of this workload (tools/pmc_summary.py:
    separate FETCH_SIZE / WRITE_SIZE / SQ passes, one record per kernel and
    grid).  Used only when the summary's record of this kernel was captured
    on the same machine code as the kernel this process launches
    (trafficrl.codeobj.kernel_code_hash of the loaded library: the kernel's
    code bytes and descriptor), whatever else in the library changed since;
    otherwise (None, reason)."""
    from trafficrl import _lib, codeobj
    path = os.path.join(ROOT, "profiles", PMC_SUMMARIES[network])
    rel = os.path.relpath(path, ROOT)
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, f"no PMC summary {rel}"
    recs = [r for r in d.get("kernels", {}).values() if r.get("kernel") == kname]
    if not recs:
        return None, f"{rel} holds no record of {kname}"
    # the workload's launches (the passes run the default workload only; bench checks that)
    rec = max(recs, key=lambda r: max(r["dispatches"].values()))
    live = codeobj.kernel_code_hash(_lib.LIB_PATH, rec["mangled_key"])
    if live != rec.get("code_sha16"):
        return None, (f"{rel} was captured on {kname} code {rec.get('code_sha16')}, this run launches code "
                      f"{live}: counters omitted")
    return rec, f"{rel} (kernel code {live})"


def env_kernel_name(env, big):
    """The env kernel trx_step launches for this workload (trx_env_kernel_name),
    with the template arguments of the Sioux Falls instantiation."""
    k = env.kernel_name
    if k == "env_kernel_pair" and env.num_nodes == 24:
        return "trx::env_kernel_pair<24, 3, true>"   # pair-per-tree Dijkstra (SF: max out-degree 5, every node reachable)
    if k == "env_kernel_s" and env.num_nodes == 24:
        return "trx::env_kernel_s<24, 2>"   # sparse-relaxation Dijkstra (SF: max out-degree 5)
    if k in ("env_kernel_t", "env_kernel_q") and env.num_nodes == 24:
        return f"trx::{k}<24>"
    return f"trx::{k}"


def cpu_greedy_episode(method, iters, nthreads):
    """The greedy one-step episode (src/baselines/__init__.py:35-69 driven by
    run_episode 72-101) on the oracle's C restatement: per decision one
    warm-started assignment per damaged candidate (a batch over the host
    threads), the first strict TSTT minimum, then the step's own assignment.
    Returns (seconds, actions, tstt curve)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only

    npz = os.path.join(ROOT, "tests", "golden", NETWORKS["sf"][1])
    og = O.OracleGraph.from_npz(npz)
    cap0 = np.load(npz)["cap0"].astype(np.float32)
    dmg = fixed_damage_mask(load_network("sf"))
    t0 = time.perf_counter()
    cap = np.where(dmg > 0, np.float32(1e-3), cap0).astype(np.float32)
    flow, _, _, _ = og.assign(cap, dmg, np.zeros_like(dmg), method=method, iters=iters)
    actions, curve = [], []
    while dmg.sum() > 0:
        cand = np.flatnonzero(dmg)
        C, D = np.repeat(cap[None], len(cand), 0), np.repeat(dmg[None], len(cand), 0)
        C[np.arange(len(cand)), cand] = cap0[cand]
        D[np.arange(len(cand)), cand] = 0.0
        _, _, ts, _ = og.assign(C, D, np.repeat(flow[None], len(cand), 0), method=method, iters=iters,
                                nthreads=nthreads)
        a = int(cand[int(np.argmin(ts))])
        cap[a], dmg[a] = cap0[a], 0.0
        flow, _, tstt, _ = og.assign(cap, dmg, flow, method=method, iters=iters)
        actions.append(a)
        curve.append(float(tstt))
    return time.perf_counter() - t0, actions, curve


def run_greedy(args):
    """Config #1 (configs/sioux_falls.yaml via run_greedy.py:47-121): one Sioux
    Falls env, fixed_damage_seed=42, the greedy one-step baseline through the
    drop-in RepairEnv facade (trafficrl/baselines: one batched trx_assign per
    decision over the damaged candidates, then RepairEnv.step).  A step =
    one greedy decision + the env step.  Timed: whole episodes (reset + 22
    decisions = 276 assignments) after one warm-up episode; the actions and
    TSTT curve are checked against the reference's own episode
    (tests/golden/sf_greedy_<method><K>_crpow.npz)."""
    from trafficrl.baselines import run_episode, select_greedy_one_step
    from trafficrl.env import RepairEnv
    method, K = args.method, args.iters
    env = RepairEnv(load_network("sf"), assignment_iters=K, assignment_method=method, fixed_damage=True,
                    fixed_damage_seed=42, seed=42, reward_mode="rel_improve", reward_alpha=1.0, reward_beta=0.0,
                    reward_gamma=0.0, reward_clip=2.0, unassigned_penalty=1e4, sp_backend=args.sp)
    acts = []

    def pol(s):
        a = select_greedy_one_step(env, s)
        acts.append(a)
        return a

    out = run_episode(env, pol)           # warm-up episode (and the trajectory checked below)
    torch.cuda.synchronize()
    ref = os.path.join(ROOT, "tests", "golden", f"sf_greedy_{method}{K}_crpow.npz")
    check = None
    if os.path.exists(ref) and args.sp == "scipy":
        z = np.load(ref)
        check = bool(acts == z["actions"].tolist() and np.array_equal(np.array(out["tstt_curve"]), z["tstt"]))
    episodes = max(1, -(-args.steps // len(acts)))
    t0 = time.perf_counter()
    for _ in range(episodes):
        run_episode(env, lambda s: select_greedy_one_step(env, s))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = episodes * len(acts)
    assigns = episodes * (1 + sum(int(env.num_edges * 0.3) - i + 1 for i in range(len(acts))))
    cpu = None
    if not args.no_cpu:
        threads, visible = host_cores()
        cs, cacts, ccurve = cpu_greedy_episode(method, K, threads)
        cpu = {"value": len(cacts) / cs, "unit": "env steps/s", "cores": threads, "kind": "port",
               "episode_s": cs, "decision_s": cs / len(cacts), "host_cpus_visible": visible,
               "same_trajectory": bool(cacts == acts),
               "sample": f"one greedy {method.upper()}-{K} episode (reset + {len(cacts)} decisions) on the C "
                         f"restatement, candidates batched over {threads} host threads; oracle/trx_oracle.c"}
    return {
        "metric": METRIC, "value": steps / dt, "unit": "env steps/s", "n_gpus": 1, "steps": steps,
        "warmup": len(acts), "ms_per_step": dt / steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32 (link flows/costs) + f64 (path labels)",
        "data": "synthetic: Sioux Falls TNTP, fixed_damage_seed=42",
        "config": {"workload": f"config #1: SF 1 env, greedy one-step baseline, {method.upper()}-{K} "
                               f"({args.sp} shortest-path rule), drop-in RepairEnv facade",
                   "workload_kind": "greedy", "envs_per_gpu": 1, "method": method, "assignment_iters": K,
                   "network": NETWORKS["sf"][2], "parallelism": "single env"},
        "greedy": {"episode_s": dt / episodes, "decision_s": dt / steps, "decisions_per_s": steps / dt,
                   "assigns_per_s": assigns / dt, "assigns_per_episode": assigns // episodes,
                   "episodes_timed": episodes, "matches_reference_episode": check,
                   "reference_cpu_decision_s": 1.63, "reference_cpu_episode_s": 21.52,
                   "reference_note": "SURVEY.md §6 / BASELINE.md: the reference's greedy MSA-30 episode on 1 core "
                                     "of this container (scipy rule)"},
        "cpu_baseline": cpu,
    }


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
    ap.add_argument("--sp", default="scipy", choices=["scipy", "torch"],
                    help="shortest-path rule: scipy = the reference's CPU Dijkstra (default; the bit-exact pinned "
                         "path), torch = its sp_backend='torch' Floyd-Warshall")
    ap.add_argument("--no-observe", action="store_true", help="skip get_state (assignment-only steps)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gemm-tuning", action="store_true",
                    help="train workload: torch's default GEMM kernels instead of the shipped TunableOp "
                         "selection (trafficrl/gemm_tuning_gfx950.csv)")
    ap.add_argument("--workload", default=None, choices=["train", "env", "greedy"],
                    help="default train (sf) / env (anaheim); greedy = config #1 (one env, greedy baseline; "
                         "--iters 60 is configs/sioux_falls.yaml's K)")
    ap.add_argument("--damage", default="fixed", choices=["fixed", "random"],
                    help="env workload: fixed = fixed_damage_seed=42 for every env; random = per-env "
                         "default_rng(1000 + global env id) draws at every reset (host-side, repair_env.py:167-192; "
                         "the resets are inside the timed region)")
    args = ap.parse_args()
    big = args.network != "sf"
    if args.envs is None:
        args.envs = 1024 if big else 4096
    if args.method is None:
        args.method = "fw" if big else "msa"
    if args.workload is None:
        args.workload = "env" if big else "train"

    if args.workload == "greedy":
        torch.cuda.set_device(0)
        print(json.dumps(run_greedy(args)), flush=True)
        return

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
    ev_pairs = []      # env_kernel step launches (HIP events on the launch stream)
    reset_ev = []      # env_kernel reset launches (whole-batch cold resets, once per episode)
    phase_ev = {}      # per-phase events (train workload)
    phase_on = [False]  # recording them (the instrumented steps after the timed loop)
    PHASE_STEPS = 64    # instrumented steps: sixteen updates at update_every 4

    def timed(fn, bucket):
        s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s_.record()
        out = fn()
        e_.record()
        bucket.append((s_, e_))
        return out

    if args.workload == "train":
        from trafficrl.train import GEMM_TUNING_GFX950, Trainer, sf_config
        cfg = sf_config()
        cfg.update(num_envs=B, assignment_iters=args.iters, assignment_method=args.method, sp_backend=args.sp,
                   batch_start=256,
                   batch_size=256, update_every=4, updates_per_step=1, update_unit="iterations", eval_every=0, episodes=10 ** 9,
                   output_dir=os.path.join("/tmp", f"trx_bench_{os.getpid()}"), amp="bf16",
                   gemm_tuning=None if args.no_gemm_tuning else GEMM_TUNING_GFX950)
        tr = Trainer(cfg, device=dev, rank=rank, world=world, log=False)
        env = tr.env
        raw_step, raw_act, raw_update = env.step, tr.act, tr.update

        def step_w(actions, observe=True, check=True):
            _, rew, done, info = timed(lambda: raw_step(actions, observe=False, check=check), ev_pairs)
            return (env.observe() if observe else None), rew, done, info

        env.step = step_w
        # act / update phase events only in the instrumented steps after the timed
        # loop: inside it they cost ~1 % of the step (measured)
        tr.act = lambda *a, **k: (timed(lambda: raw_act(*a, **k), phase_ev.setdefault("act", [])) if phase_on[0]
                                  else raw_act(*a, **k))
        tr.update = lambda *a, **k: (timed(lambda: raw_update(*a, **k), phase_ev.setdefault("update", []))
                                     if phase_on[0] else raw_update(*a, **k))
        tr._reset_envs(None)
        E, N = env.num_edges, env.num_nodes
        dmg_all = tr.fixed_mask.expand(B, E).contiguous()
        ep_len = int(tr.fixed_mask.sum().item())
        all_true = torch.ones(B, dtype=torch.bool, device=dev)
        st = {"obs": env.observe(), "it": 0, "t": 0}

        def reset():
            timed(lambda: env.reset_where(all_true, dmg_all), reset_ev)
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
                           reward_clip=2.0, capacity_damage=1e-3, unassigned_penalty=1e4, reset=False,
                           sp_backend=args.sp, seeds=[1000 + rank * B + i for i in range(B)])
        E, N = env.num_edges, env.num_nodes
        dmg0 = torch.from_numpy(fixed_damage_mask(gd)).to(dev)
        dmg_all = None if args.damage == "random" else dmg0[None].expand(B, E).contiguous()
        ep_len = int(dmg0.sum().item())     # max(1, int(E * 0.3)) damaged links either way
        st = {"t": 0}

        if dmg_all is None:
            # random damage: every env's next mask is drawn on a host thread while the
            # device steps the current episode (pinned, copied asynchronously at reset)
            env.enable_damage_prefetch(True)

        def reset():
            if dmg_all is None:
                timed(lambda: env.reset(observe=False), reset_ev)
            else:
                timed(lambda: env.reset(damaged=dmg_all, observe=False), reset_ev)
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
    if args.workload == "train":
        # steady state whatever --warmup is: the eager warm-up updates and the
        # HIP-graph capture of the SAC update happen here, never in the timed loop
        while tr.replay.size <= int(cfg["batch_start"]):
            one_step()
        tr.prime_update()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    ev_pairs.clear()
    reset_ev.clear()
    for v in phase_ev.values():
        v.clear()
    torch.cuda.synchronize()
    upd0 = tr.updates_done if args.workload == "train" else 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    upd_in_loop = (tr.updates_done - upd0) if args.workload == "train" else 0
    step_ms = [s.elapsed_time(e) for s, e in ev_pairs]
    reset_ms = [s.elapsed_time(e) for s, e in reset_ev]
    if args.workload == "train":   # the per-phase breakdown, from instrumented steps after the timed loop
        phase_on[0] = True
        for _ in range(PHASE_STEPS):
            one_step()
        torch.cuda.synchronize()
        phase_on[0] = False
    breakdown = {k: float(np.sum([s_.elapsed_time(e_) for s_, e_ in v])) / PHASE_STEPS for k, v in phase_ev.items()}
    kern_ms = step_ms + reset_ms     # every assignment launch of the timed region
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
    kname = env_kernel_name(env, big)
    sha = lib_sha16()
    pmc, pmc_src = measured_traffic(args.network, kname)
    if pmc is not None and (args.envs, args.iters, args.method) != ((1024, 30, "fw") if big else (4096, 30, "msa")):
        pmc, pmc_src = None, "committed PMC passes cover the default workloads only"
    traffic = pmc.get("hbm_bytes_per_launch_raw") if pmc else None
    valu_frac = pmc.get("valu_busy_frac") if pmc else None
    lds_conf = pmc.get("lds_bank_conflict_frac") if pmc else None
    mfma = gemm_mfma(B * N, B) if (args.workload == "train" and rank == 0) else None
    if mfma is not None and breakdown.get("act"):
        # the live acting pass (one per step, HIP events around it in the instrumented steps):
        # its GEMM FLOPs over its whole wall time -- GAT layer kernels, edge scorer,
        # prologue included -- beside the GEMM-only figure above
        act_ms = breakdown["act"]
        mfma.update(act_pass_ms=act_ms, act_pass_achieved=mfma["flops_per_pass"] / (act_ms / 1e3) / 1e12,
                    act_pass_frac=mfma["flops_per_pass"] / (act_ms / 1e3) / MFMA_PEAK_BF16,
                    act_pass_note="frac / achieved: the acting GEMMs' shapes timed alone (torch.mm, HIP events); "
                                  "act_pass_*: the same FLOPs over the acting pass of this run (HIP events, "
                                  "instrumented steps after the timed loop)")
    upd_stats = None
    if args.workload == "train" and phase_ev.get("update"):
        # SAC update throughput (the timed updates are graph replays), and the env
        # steps/s this GPU would sustain at the reference's update-to-data ratio
        # (configs/sioux_falls.yaml:17-18 update_every 4, updates_per_step 1: one
        # update per 4 transitions, src/train.py:954-955) instead of the bench's 1/(4B)
        upd_ms = [s_.elapsed_time(e_) for s_, e_ in phase_ev["update"]]
        ms_upd = float(np.mean(upd_ms))
        # one iteration without its updates: the timed loop's own update count times the
        # instrumented mean update time (update_unit "transitions" runs a varying number)
        ms_rest = elapsed / args.steps * 1e3 - upd_in_loop * ms_upd / args.steps
        flops = sac_update_flops(int(cfg["batch_size"]), N, E)
        upd_stats = {"ms_per_update": ms_upd, "updates_per_s": 1e3 / ms_upd, "updates_timed": len(upd_ms),
                     "updates_in_timed_loop": upd_in_loop,
                     "flops_per_update": flops, "mfma_frac": flops / (ms_upd / 1e3) / MFMA_PEAK_BF16,
                     "env_steps_per_s_at_reference_utd": 1e3 / (ms_rest / B + ms_upd / 4.0),
                     "note": "mfma_frac: GEMM FLOPs of 3 no-grad + 3 training forwards and 3 backwards "
                             "(2x forward) at batch 256 / the update's wall time / 2.5 PF dense bf16"}
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(args.network, args.method, args.iters, args.cpu_seconds, args.sp)
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
                     + ("fixed_damage_seed=42, " if args.damage == "fixed" or args.workload == "train" else
                        "random damage per env (default_rng(1000 + env id), redrawn at every reset), ") + ("random-init GAT-SAC (hidden 256, 4 heads, embed 256)"
                                                 if args.workload == "train" else "uniform random valid repair actions")),
            "config": {
                "workload": (f"{'SF' if not big else 'AnaheimSynth'} {B} vectorised envs/GPU, {args.method.upper()}-{args.iters} assignment"
                             f" ({args.sp} shortest-path rule) + get_state per step"
                             + (f", GAT-SAC bf16 acting every step + 1 PER update (batch 256) every 4 steps (update-to-data "
                                f"ratio 1/{4 * B} per transition)" if args.workload == "train" else ", uniform random valid actions")),
                "sp_backend": args.sp,
                "workload_kind": args.workload,
                "damage": "fixed" if args.workload == "train" else args.damage,
                "envs_per_gpu": B, "global_envs": B * world, "network": NETWORKS[args.network][2],
                "method": args.method, "assignment_iters": args.iters, "episode_len": ep_len,
                "parallelism": f"env-sharded x{world}",
                **({"gemm_kernels": ("TunableOp selection trafficrl/gemm_tuning_gfx950.csv (lookup only)"
                                     if tr.tuned_gemms else "torch default"),
                    "update_precision": ("critics bf16 autocast; actor training pass float32 (exact kernels, "
                                         "three-product split-bf16 GEMMs)" if tr.agent.fp32_actor
                                         else "bf16 autocast")} if args.workload == "train" else {}),
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": traffic,
                "traffic_note": (f"rocprofv3 FETCH_SIZE+WRITE_SIZE per launch, {pmc_src}; raw: 4-byte loads, "
                                 f"gfx950 x2 wide-read fetch correction not applied") if traffic
                else pmc_src,
                "lib_sha16": sha,
                "kernel": kname, "kernel_mean_ms": mean_kernel_s * 1e3,
                "valu_busy_frac": valu_frac,
                "lds_bank_conflict_frac": lds_conf,
                "valu_note": ("SIMD VALU issue share of the same kernel from the committed PMC passes "
                              "(4 x SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)); the kernel is issue-bound, "
                              "not HBM-bound; lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS") if valu_frac else None,
                "bytes_per_assign": bpa, "assigns_per_launch": B,
                "mfma": mfma,
            },
            "cpu_baseline": cpu,
            "breakdown_note": (f"act / update: HIP events over {PHASE_STEPS} instrumented steps after the timed "
                               f"loop ({len(phase_ev.get('update', []))} updates); env_*: events around every env "
                               "launch of the timed loop")
            if args.workload == "train" else None,
            "breakdown_ms_per_step": dict(breakdown, env_kernel=float(np.sum(kern_ms)) / args.steps,
                                          env_step_kernel=float(np.sum(step_ms)) / args.steps,
                                          env_reset_kernel=float(np.sum(reset_ms)) / args.steps),
            "env_launches": {"step_mean_ms": float(np.mean(step_ms)) if step_ms else None,
                             "reset_mean_ms": float(np.mean(reset_ms)) if reset_ms else None,
                             "resets_timed": len(reset_ms), "steps_timed": len(step_ms),
                             "note": "HIP events around trx_step / trx_reset (the reset's events include the "
                                     "asynchronous copy of the prefetched damage masks when damage is random)"},
        }
        if args.workload == "train" and upd_stats is not None:
            out["sac_update"] = upd_stats
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

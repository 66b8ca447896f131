"""Host submission cost vs GPU time of the replayed graphs (the SAC update and the
acting pass, bench shapes).  For each graph: the host time of `replay()` alone (the
runtime enqueues every node's packet from the calling thread), the GPU time of one
isolated replay (HIP events around it, after a synchronize), and the GPU time per
replay of K back-to-back replays.  If the host time of one replay approaches its GPU
time, the replay is submission-bound: the GPU waits for packets.

usage: python tools/graph_launch_probe.py [K]"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def probe(name, replay, K):
    host, iso = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        replay()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        host.append((t1 - t0) * 1e3)
        iso.append(e0.elapsed_time(e1))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(K):
        replay()
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: host replay() {statistics.median(host):.3f} ms, GPU isolated {statistics.median(iso):.3f} ms, "
          f"GPU back-to-back {e0.elapsed_time(e1) / K:.3f} ms/replay (host {(t1 - t0) * 1e3 / K:.3f} ms/replay)",
          flush=True)


def main():
    from trafficrl.train import Trainer, sf_config
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    cfg = sf_config()
    cfg.update(num_envs=4096, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_glp",
               buffer_size=65536)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(4):
        obs, _ = tr.iteration(obs, it)
    tr.prime_update()
    tr.update()
    gu = tr._graphed
    probe("update graph", gu._replay, K)
    tr.act(obs)
    tr.act(obs)
    ga = tr._graphed_act
    probe("act graph", ga.g.replay, K)


if __name__ == "__main__":
    main()

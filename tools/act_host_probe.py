"""Is the acting pass host-bound?  Times one 4096-env actor pass three ways:
host enqueue time (no sync), GPU time (HIP events), wall per call (synced);
and the same pass replayed from a HIP graph (train.GraphedAct).
Usage: python tools/act_host_probe.py [B]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def main():
    from trafficrl.train import Trainer, sf_config
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    cfg = sf_config()
    cfg.update(num_envs=B, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_probe",
               buffer_size=65536, sp_backend="scipy", amp="bf16")
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    for _ in range(5):
        tr._act(obs)
    torch.cuda.synchronize()
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        tr._act(obs)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        tr._act(obs)
    e.record()
    torch.cuda.synchronize()
    print(f"eager: host enqueue {(t1 - t0) / n * 1e3:.3f} ms/call, wall {(t2 - t0) / n * 1e3:.3f} ms/call, "
          f"GPU span {s.elapsed_time(e) / n:.3f} ms/call")
    if tr._graphed_act is not None:
        for _ in range(3):
            tr.act(obs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            tr.act(obs)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"graph: host enqueue {(t1 - t0) / n * 1e3:.3f} ms/call, wall {(t2 - t0) / n * 1e3:.3f} ms/call")


if __name__ == "__main__":
    main()

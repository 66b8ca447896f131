"""Steady-state time of one graphed SAC update (the bench's update: batch 256,
Sioux Falls, float32 actor): prime (eager warm-ups + capture), then R rounds
of K back-to-back updates timed with HIP events; prints each round and the
median.  Environment knobs are read by the callers (GPU_MAX_HW_QUEUES, ...).

usage: python tools/upd_time.py [K] [R]"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def main():
    if os.environ.get("TRX_LIB"):
        from trafficrl import _lib
        _lib.LIB_PATH = os.path.abspath(os.environ["TRX_LIB"])
    from trafficrl.train import Trainer, sf_config
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cfg = sf_config()
    cfg.update(num_envs=1024, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_upd",
               buffer_size=65536)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(4):
        obs, _ = tr.iteration(obs, it)
    tr.prime_update()
    ms = []
    for r in range(R):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(K):
            tr.update()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1) / K)
        print(f"round {r}: {ms[-1]:.3f} ms/update", flush=True)
    print(f"update median {statistics.median(ms):.3f} ms/update ({K} x {R})", flush=True)


if __name__ == "__main__":
    main()

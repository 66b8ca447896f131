"""Is the train loop host-bound?  Times the host side of each trainer
iteration (enqueue only, no sync) against the device time of the same
iteration (events), at the bench's default workload."""
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
    cfg.update(num_envs=B, batch_start=256, batch_size=256, update_every=4, update_unit="iterations", eval_every=0,
               output_dir="/tmp/trx_probe", amp="bf16", fixed_damage=True)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    E = tr.env.num_edges
    ep_len = int(tr.fixed_mask.sum().item())
    every = torch.ones(B, dtype=torch.bool, device="cuda")

    def step(obs, it):  # auto-reset every episode, like bench.py
        obs, _ = tr.iteration(obs, it)
        if (it + 1) % ep_len == 0:
            tr.env.reset_where(every, tr.fixed_mask.expand(B, E))
            obs = tr.env.observe()
        return obs

    for it in range(44):
        obs = step(obs, it)
    torch.cuda.synchronize()
    host, dev = [], []
    for it in range(44, 88):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        t0 = time.perf_counter()
        obs = step(obs, it)
        host.append((time.perf_counter() - t0) * 1e3)
        e.record()
        dev.append((s, e))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(88, 132):
        obs = step(obs, it)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 44 * 1e3
    d = [a.elapsed_time(b) for a, b in dev]
    print(f"host enqueue {sum(host) / len(host):.3f} ms/iter, device {sum(d) / len(d):.3f} ms/iter, "
          f"wall {wall:.3f} ms/iter")


if __name__ == "__main__":
    main()

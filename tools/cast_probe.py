#!/usr/bin/env python3
"""Where the update's dtype casts come from: one eager SAC update
(compute_gradients) under torch.profiler with shapes and Python stacks; prints
every aten::_to_copy / aten::copy_ / aten::cat / elementwise op with its shape
and the innermost trafficrl frame.  Usage: python tools/cast_probe.py"""
import os
import sys
from collections import Counter

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def main():
    from torch.profiler import ProfilerActivity, profile
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    cfg.update(num_envs=512, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_cast",
               buffer_size=65536, graph_update=False)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(2):
        obs, _ = tr.iteration(obs, it)
    tr.update()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        tr.update()
        torch.cuda.synchronize()
    counts = Counter()
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        if ev.name not in ("aten::_to_copy", "aten::copy_", "aten::cat", "aten::add", "aten::add_", "aten::fill_",
                           "aten::zero_", "aten::sum", "aten::index", "aten::mul", "aten::clone", "aten::contiguous"):
            continue
        frames = [f for f in (ev.stack or []) if "trafficrl" in f or "torch/autograd" in f]
        where = frames[0] if frames else "?"
        key = (ev.name, str(ev.input_shapes)[:70], where[-90:])
        counts[key] += 1
    for (name, shp, where), n in sorted(counts.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d} {name:16s} {shp:70s} {where}")


if __name__ == "__main__":
    main()

"""Op-level profile of ONE eager SAC update (batch 256) of the GAT-SAC
trainer: torch.profiler with input shapes, sorted by device time, so the
kernels of the graphed update can be attributed to aten ops.
Usage: python tools/update_profile.py [rows]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def main():
    from torch.profiler import ProfilerActivity, profile

    from trafficrl.train import Trainer, sf_config
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    cfg = sf_config()
    cfg.update(num_envs=512, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_prof", buffer_size=65536)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr.use_graphs = False
    tr._graphed = None
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(6):
        obs, _ = tr.iteration(obs, it)
    for _ in range(3):
        u, her_u = tr._draw_update_randoms()
        tr._update_once(u, her_u)
    torch.cuda.synchronize()
    copies = len(sys.argv) > 2 and sys.argv[2] == "copies"
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=copies) as prof:
        u, her_u = tr._draw_update_randoms()
        tr._update_once(u, her_u)
        torch.cuda.synchronize()
    if copies:  # dtype conversions attributed to the trafficrl source line that issued them
        ka = prof.key_averages(group_by_input_shape=True, group_by_stack_n=6)
        evs = [e for e in ka if e.key in ("aten::_to_copy", "aten::copy_") and e.device_time_total > 0]
        evs.sort(key=lambda e: -e.device_time_total)
        for e in evs[:rows]:
            stack = [f for f in (e.stack or []) if "trafficrl" in f][:2]
            print(f"{e.device_time_total / 1e3:7.3f} ms x{e.count:<3d} {e.key:15s} {str(e.input_shapes)[:60]:60s} "
                  f"{' <- '.join(x.split('/')[-1] for x in stack)}")
        return
    ka = prof.key_averages(group_by_input_shape=True)
    evs = [e for e in ka if not e.key.startswith(("autograd::", "Cijk", "void ", "trx::", "Custom_", "__amd"))]
    evs.sort(key=lambda e: -e.device_time_total)
    for e in evs[:rows]:
        print(f"{e.device_time_total / 1e3:8.3f} ms total {e.self_device_time_total / 1e3:8.3f} self  x{e.count:<4d} "
              f"{e.key[:38]:38s} {str(e.input_shapes)[:110]}")
    tot = sum(e.self_device_time_total for e in prof.key_averages())
    n = sum(e.count for e in prof.key_averages() if e.self_device_time_total > 0)
    print(f"self device total {tot / 1e3:.3f} ms")


if __name__ == "__main__":
    main()

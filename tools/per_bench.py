#!/usr/bin/env python3
"""Time the device PER sum tree (float32 reference tree vs float64) at the
reference's buffer_size 1e6: a 4096-transition ring add per env step and a
256-draw sample + update_priorities per SAC update.
Usage: python tools/per_bench.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
import torch  # noqa: E402

from trafficrl.rl.replay import DeviceReplay  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    d = torch.device("cuda", 0)
    for dt in ("float32", "float64"):
        rb = DeviceReplay(1_000_000, 1, 1, node_dim=1, edge_dim=1, device=d, tree_dtype=dt)
        B = 4096
        z = lambda *s, **kw: torch.zeros(*s, device=d, **kw)  # noqa: E731
        args = (z(B, 1, 1), z(B, 1, 1), z(B, 1), torch.zeros(B, dtype=torch.int64, device=d), z(B), z(B, 1, 1),
                z(B, 1, 1), z(B, 1), z(B), z(B, 1), z(B, dtype=torch.float64), z(B, dtype=torch.float64),
                z(B, dtype=torch.float64))
        for _ in range(20):
            rb.add_batch(*args)
        u = torch.rand(256, dtype=torch.float64, device=d)
        td = torch.randn(256, device=d)
        res = {}
        for name, fn in (("add4096", lambda: rb._priorities_for_new(None, B)),
                         ("sample256", lambda: rb.sample(256, u=u)),
                         ("update256", lambda: rb.update_priorities(rb.sample(256, u=u).idx, td))):
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[name] = s.elapsed_time(e) / reps * 1e3
        print(dt, " ".join(f"{k}={v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()

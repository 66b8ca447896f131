"""Per-phase op profile of the GAT-SAC trainer (acting at B envs, one SAC
update at batch 256) with torch.profiler; prints the top device-time ops of
each phase and the wall time per call.  Usage: python tools/agent_profile.py [B] [act|update]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def main():
    from torch.profiler import ProfilerActivity, profile

    if os.environ.get("TRX_LIB"):   # A/B a second build of libtrafficrl.so
        from trafficrl import _lib
        _lib.LIB_PATH = os.path.abspath(os.environ["TRX_LIB"])
    from trafficrl.train import Trainer, sf_config
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    cfg = sf_config()
    cfg.update(num_envs=B, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_prof", buffer_size=65536)
    if os.environ.get("TRX_FP32_ACTOR"):   # A/B the float32 actor of the fused update
        cfg.update(fp32_actor=os.environ["TRX_FP32_ACTOR"] == "1")
    tr = Trainer(cfg, device="cuda:0", log=False)
    serial = os.environ.get("TRX_UPD_SERIAL", "")   # fwd | bwd: that phase of the fused update on one stream
    if serial in ("fwd", "bwd"):
        conc, n_serial = tr.agent._concurrent, (6 if serial == "fwd" else 3)
        tr.agent._concurrent = lambda fns, streams=None: ([fn() for fn in fns] if len(fns) == n_serial
                                                         else conc(fns, streams))
    if os.environ.get("TRX_UPD_STREAMS"):   # concurrent side streams of the update (A/B)
        tr.agent.max_streams = int(os.environ["TRX_UPD_STREAMS"])
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(8):
        obs, _ = tr.iteration(obs, it)
    torch.cuda.synchronize()

    def timeit(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    only = sys.argv[2] if len(sys.argv) > 2 else None
    if only == "update":   # for rocprofv3: only SAC updates (graph replays after 3 eager warm-ups)
        print(f"update wall {timeit(tr.update, 30):8.3f} ms/call")
        return
    if only == "act":
        print(f"act    wall {timeit(lambda: tr.act(obs), 30):8.3f} ms/call")
        return
    print(f"act    wall {timeit(lambda: tr.act(obs), 10):8.3f} ms/call")
    print(f"update wall {timeit(tr.update, 10):8.3f} ms/call")
    for name, fn in (("act", lambda: tr.act(obs)), ("update", tr.update)):
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
        print(f"===== {name} (5 calls)")
        print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=40, max_name_column_width=70))


if __name__ == "__main__":
    main()

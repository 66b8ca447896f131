"""Probe: how much of one graphed SAC update hides behind an env step (and an
acting pass) when the two run on different HIP streams.  Prints the
sequential and the overlapped wall time per (step [+ act] + update)."""
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
    cfg.update(num_envs=B, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_ov", buffer_size=65536)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(12):
        obs, fin = tr.iteration(obs, it)
        tr._reset_envs(fin)
    for _ in range(4):
        tr.update()
    torch.cuda.synchronize()
    acts = tr.act(obs).to(torch.int32)
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def env_part(with_act):
        if with_act:
            tr.act(obs)
        tr.env.step(acts, check=False)

    def timeit(fn, reps=20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    for with_act in (False, True):
        tag = "step+act" if with_act else "step"
        t_env = timeit(lambda: env_part(with_act))
        t_upd = timeit(tr.update)
        t_seq = timeit(lambda: (env_part(with_act), tr.update()))

        def ovl():
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                tr.update()
            env_part(with_act)
            main_s.wait_stream(side)
        t_ovl = timeit(ovl)
        print(f"{tag:>9}: alone {t_env:6.2f} ms, update alone {t_upd:6.2f} ms, sequential {t_seq:6.2f} ms, "
              f"overlapped {t_ovl:6.2f} ms")


if __name__ == "__main__":
    main()

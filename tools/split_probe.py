"""Probe: does splitting the vector env into two halves on two HIP streams, with
the acting pass of one half overlapping the env kernel of the other, beat the
serial act -> step -> observe chain at the same total env count?

  python tools/split_probe.py [--envs 4096] [--steps 44]

Prints ms per vector step (all envs) for: serial (one Trainer of B envs), split
(two Trainers of B/2 envs, acts ordered A, B, A, ... by events, each half's env
step free to overlap the other half's act) and free (two streams, no ordering).
Acting only (no replay, no update): the part of the train step the split changes."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

import torch  # noqa: E402

from trafficrl.train import GEMM_TUNING_GFX950, Trainer, sf_config  # noqa: E402


def make(B):
    cfg = sf_config()
    cfg.update(num_envs=B, batch_start=256, batch_size=256, buffer_size=4096, eval_every=0,
               output_dir=f"/tmp/trx_probe_{os.getpid()}", amp="bf16", gemm_tuning=GEMM_TUNING_GFX950)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    return tr


class Half:
    def __init__(self, tr):
        self.tr, self.env = tr, tr.env
        self.obs = self.env.observe()
        self.t = 0
        self.len = int(tr.fixed_mask.sum().item())
        self.all = torch.ones(tr.B, dtype=torch.bool, device=tr.device)
        self.dmg = tr.fixed_mask.expand(tr.B, -1).contiguous()

    def act(self):
        return self.tr.act(self.obs)

    def env_step(self, a):
        self.env.step(a.to(torch.int32), observe=False, check=False)
        self.t += 1
        if self.t == self.len:
            self.env.reset_where(self.all, self.dmg)
            self.t = 0
        self.obs = self.env.observe()


def run_serial(h, steps):
    for _ in range(steps):
        h.env_step(h.act())


def run_split(hA, hB, sA, sB, steps, ordered):
    evA, evB = torch.cuda.Event(), torch.cuda.Event()
    first = True
    for _ in range(steps):
        with torch.cuda.stream(sA):
            if ordered and not first:
                sA.wait_event(evB)
            a = hA.act()
            evA.record(sA)
            hA.env_step(a)
        with torch.cuda.stream(sB):
            if ordered:
                sB.wait_event(evA)
            b = hB.act()
            evB.record(sB)
            hB.env_step(b)
        first = False


def timeit(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(steps)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=44)
    args = ap.parse_args()
    B = args.envs
    full = Half(make(B))
    run_serial(full, 24)
    ms_serial = timeit(lambda k: run_serial(full, k), args.steps)
    print(f"serial B={B}: {ms_serial:.3f} ms/step", flush=True)
    del full
    hA, hB = Half(make(B // 2)), Half(make(B // 2))
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    for ordered in (True, False):
        run_split(hA, hB, sA, sB, 24, ordered)
        ms = timeit(lambda k: run_split(hA, hB, sA, sB, k, ordered), args.steps)
        print(f"split {'ordered' if ordered else 'free'} 2x{B // 2}: {ms:.3f} ms/step "
              f"({ms_serial / ms:.3f}x serial)", flush=True)
    run_serial(hA, 24)
    ms_half = timeit(lambda k: run_serial(hA, k), args.steps)
    print(f"serial B={B // 2}: {ms_half:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()

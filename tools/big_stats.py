"""Diagnostic: trees / label sweeps / exact replays and the launch time of the
large-graph assignment kernel (bigstats build: make bigstats), for the
register-entry path (default) and, with TRX_BIG_KM=0, the LDS-entry path.

Usage: python tools/big_stats.py [B] [method]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
import torch  # noqa: E402
from trafficrl import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "sac-gat-her_transportationrl_amd", "trafficrl", "libtrafficrl_bigstats.so")
L = _lib.load()
L.trx_debug_big_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
from trafficrl.data import anaheim_synthetic  # noqa: E402
from trafficrl.env import VecRepairEnv  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
method = sys.argv[2] if len(sys.argv) > 2 else "fw"
env = VecRepairEnv(anaheim_synthetic(), B, assignment_iters=30, assignment_method=method, fixed_damage=True,
                   fixed_damage_seed=42)
buf = (ctypes.c_ulonglong * 8)()
gen = torch.Generator(device="cuda").manual_seed(0)
acts = [(torch.rand(B, env.num_edges, device="cuda", generator=gen) * env.damaged).argmax(1).to(torch.int32)
        for _ in range(4)]
env.step(acts[0], observe=False)
torch.cuda.synchronize()
L.trx_debug_big_stats(buf, 1)
t0 = time.perf_counter()
for a in acts[1:]:
    env.step(a, observe=False)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 3
L.trx_debug_big_stats(buf, 1)
trees = buf[0]
print(f"{dt * 1e3:.2f} ms/step  trees/step {trees / 3:.0f}  "
      f"sweeps/tree {buf[1] / max(trees, 1):.2f}  exact replays {buf[2]}")
print(f"per tree (s_memtime ticks, 100 MHz): sweeps {buf[3] / max(trees, 1):.0f}  preds {buf[4] / max(trees, 1):.0f}  "
      f"walks {buf[5] / max(trees, 1):.0f}")

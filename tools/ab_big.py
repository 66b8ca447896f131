"""A/B of the large-graph env kernel: one library (by path) per process.
AnaheimSynth, B envs, FW-30, fixed damage, 8 timed steps of one repaired link
each (HIP events around env.step) + a checksum of flows / TSTT so variants are
compared bit for bit.  Usage: python tools/ab_big.py LIB [B]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
import torch  # noqa: E402
from trafficrl import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
from trafficrl.data import anaheim_synthetic  # noqa: E402
from trafficrl.env import VecRepairEnv  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
env = VecRepairEnv(anaheim_synthetic(), B, assignment_iters=30, assignment_method="fw", fixed_damage=True,
                   fixed_damage_seed=42)
gen = torch.Generator(device="cuda").manual_seed(0)
acts = [(torch.rand(B, env.num_edges, device="cuda", generator=gen) * env.damaged).argmax(1).to(torch.int32)
        for _ in range(11)]
for a in acts[:3]:
    env.step(a, observe=False)
torch.cuda.synchronize()
ts = []
for a in acts[3:]:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    env.step(a, observe=False)
    e.record()
    ts.append((s, e))
torch.cuda.synchronize()
ms = sorted(s.elapsed_time(e) for s, e in ts)
h = hashlib.sha256(env.flow.cpu().numpy().tobytes() + env.tstt.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"{os.path.basename(sys.argv[1])}: step kernel median {ms[len(ms) // 2]:.2f} ms (min {ms[0]:.2f})  sha {h}")

"""A/B timing of the env kernel from two builds of libtrafficrl.so in one
process each: python tools/ab_env.py <lib.so> [B] [reps] [scipy|torch|obs]
("obs" times trx_observe after one step instead of the step kernel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
import torch  # noqa: E402
from trafficrl import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
from trafficrl.data import sioux_falls  # noqa: E402
from trafficrl.env import VecRepairEnv  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
sp = sys.argv[4] if len(sys.argv) > 4 else "scipy"
env = VecRepairEnv(sioux_falls(), B, assignment_iters=30, fixed_damage=True, fixed_damage_seed=42,
                   sp_backend="scipy" if sp == "obs" else sp)
gen = torch.Generator(device="cuda").manual_seed(0)
acts = [(torch.rand(B, 76, device="cuda", generator=gen) * env.damaged).argmax(1).to(torch.int32) for _ in range(2)]
flow0, cap0, dmg0 = env.flow.clone(), env.capacity.clone(), env.damaged.clone()
ms = []
if sp == "obs":
    env.step(acts[0], observe=False, check=False)
    for r in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        env.observe()
        e.record()
        torch.cuda.synchronize()
        ms.append(s.elapsed_time(e))
    ms = sorted(ms)[2:-2]
    print(f"{os.path.basename(sys.argv[1])}: observe {sum(ms) / len(ms) * 1e3:.1f} us (B={B})")
    sys.exit(0)
for r in range(reps):
    env.flow.copy_(flow0); env.capacity.copy_(cap0); env.damaged.copy_(dmg0)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    env.step(acts[0], observe=False, check=False)
    e.record()
    torch.cuda.synchronize()
    ms.append(s.elapsed_time(e))
ms = sorted(ms)[2:-2]
# result checksum (variants must agree bit for bit): the timed step's state, then a
# cold reset with per-env random damage (tie-heavy: exercises the exact-heap replays)
import hashlib  # noqa: E402
import numpy as np  # noqa: E402
h = hashlib.sha1(env.flow.cpu().numpy().tobytes() + env.tstt.cpu().numpy().tobytes())
rng = np.random.default_rng(5)
dmg = np.zeros((B, 76), np.float32)
for b in range(B):
    dmg[b, rng.choice(76, 22, replace=False)] = 1.0
dmg_t = torch.from_numpy(dmg).cuda()
rs = []
for r in range(3):   # cold resets: per-env random damage, then the fixed damage of the timed steps
    for dm in (dmg_t, dmg0):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        env.reset(damaged=dm, observe=False)
        e.record()
        torch.cuda.synchronize()
        rs.append(s.elapsed_time(e))
env.reset(damaged=dmg_t, observe=False)
h.update(env.flow.cpu().numpy().tobytes() + env.tstt.cpu().numpy().tobytes())
print(f"{os.path.basename(sys.argv[1])} [{sp}]: step kernel {sum(ms) / len(ms):.4f} ms (B={B}) sha {h.hexdigest()[:12]}"
      f"  reset random {min(rs[0::2]):.2f} ms, fixed {min(rs[1::2]):.2f} ms")

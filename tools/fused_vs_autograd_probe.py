"""Probe: worst per-tensor gradient difference between the fused update and
the autograd path (tests/test_fused_update.py::test_fused_update_vs_autograd_path),
after the optimizer-step test's agents have run in the same process, with the
autograd path's side-stream concurrency on and off, repeated.
Usage: python tools/fused_vs_autograd_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "sac-gat-her_transportationrl_amd")]

import torch  # noqa: E402

import test_flat_adam as FA  # noqa: E402
import test_fused_update as T  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False


def run(tag, concurrent):
    B = 256
    batch = T._update_batch(B)
    agent = T.make_agent(hidden=256, embed=256)
    agent.concurrent = concurrent
    w = torch.rand(B, device="cuda") * 0.5 + 0.5
    agent.compute_gradients(batch, weights=w)
    got = T._grads(agent)
    ref, _, _ = T._autograd_grads(agent, batch, w)
    for m in T.MODS:
        sub = {k: v for k, v in ref.items() if k.startswith(m + ".")}
        print(tag, m, T._worst({k: got[k] for k in sub}, sub), flush=True)
    return got, ref


g0, r0 = run("fresh concurrent", True)
FA.test_flat_adam_vs_torch_optimizers()
FA.test_flat_adam_handoff_to_torch_and_back()
g1, r1 = run("after-flat-adam concurrent", True)
g2, r2 = run("after-flat-adam sequential", False)
g3, r3 = run("after-flat-adam concurrent again", True)
for name, a, b in (("fused 0 vs 1", g0, g1), ("fused 1 vs 2", g1, g2), ("autograd 0 vs 1", r0, r1),
                   ("autograd 1 vs 2", r1, r2), ("autograd 2 vs 3", r2, r3)):
    d = max(float((a[k] - b[k]).abs().max()) for k in a)
    print(f"{name}: max abs diff {d:.3e}", flush=True)

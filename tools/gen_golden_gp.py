#!/usr/bin/env python3
"""Golden fixtures for the path-based (GP) assignment
(src/env/repair_env.py:351-419, assignment_method="gp") on Sioux Falls,
produced by running the REFERENCE env read-only in this container (same
procedure and 'crpow' variant as tools/gen_golden.py).

Writes tests/golden/sf_gp_crpow.npz:
  reset_<tag>_{damaged,flow,t,tstt,unassigned}   fixed_damage_seed=42 resets
  steps_<tag>_{damaged,flow,tstt,actions,step_flow,step_tstt,step_reward,step_done}
     4 random-seed envs: reset + 3 steps (the 2nd repeats a repaired link)
  tags: s1k2i30 (gp_step 1, keep 2, 30 iters: configs/sioux_falls.yaml),
        s1k3i10 (reference defaults), s0k3i10 (step 1/(it+1): fractional path
        flows, order-dependent float32 loading), s05k2i8 (step 0.5)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_gp.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402

CASES = {"s1k2i30": (1.0, 2, 30), "s1k3i10": (1.0, 3, 10), "s0k3i10": (0.0, 3, 10), "s05k2i8": (0.5, 2, 8)}


def main():
    t0 = time.time()
    out = {}
    for tag, (step, keep, iters) in CASES.items():
        env = G.make_env(G.CRPowEnv, assignment_method="gp", assignment_iters=iters, gp_step=step,
                         gp_keep_paths=keep, fixed_damage=True, fixed_damage_seed=42, seed=42)
        out[f"reset_{tag}_damaged"] = env.is_damaged.copy()
        out[f"reset_{tag}_flow"] = env.flow.copy()
        out[f"reset_{tag}_t"] = env.compute_travel_time(env.flow)
        out[f"reset_{tag}_tstt"] = np.float64(env.tstt)
        out[f"reset_{tag}_unassigned"] = np.float64(env.unassigned_demand)
        seeds = [0, 1, 2, 3]
        rec = {k: [] for k in ("damaged", "flow", "tstt", "actions", "step_flow", "step_tstt", "step_reward",
                               "step_done")}
        for s in seeds:
            env = G.make_env(G.CRPowEnv, assignment_method="gp", assignment_iters=iters, gp_step=step,
                             gp_keep_paths=keep, seed=s)
            rec["damaged"].append(env.is_damaged.copy())
            rec["flow"].append(env.flow.copy())
            rec["tstt"].append(env.tstt)
            rng = np.random.default_rng(7 + s)
            acts, fl, ts, rw, dn = [], [], [], [], []
            first = None
            for j in range(3):
                if j == 1:
                    a = first
                else:
                    a = int(rng.choice(np.where(env.is_damaged > 0)[0]))
                    first = a if first is None else first
                _, r, d, info = env.step(a)
                acts.append(a); fl.append(env.flow.copy()); ts.append(info["tstt"]); rw.append(r); dn.append(d)
            rec["actions"].append(acts); rec["step_flow"].append(fl); rec["step_tstt"].append(ts)
            rec["step_reward"].append(rw); rec["step_done"].append(dn)
        for k, v in rec.items():
            out[f"steps_{tag}_{k}"] = np.array(v)
        print(f"  {tag}: {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(G.OUT, "sf_gp_crpow.npz"), **out)
    print(f"GP fixtures written in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()

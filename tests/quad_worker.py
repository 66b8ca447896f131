"""Subprocess body of tests/test_gpu_fallback.py::test_forced_quad_on_sf_fixtures
and tests/test_gpu_sparse.py::test_quad_sparse_kernel_on_pair_cases: runs with
TRX_KERNEL=quad or TRX_KERNEL=sparse in its environment (the switch is read
once per process by csrc/capi.hip).  quad: every Sioux Falls env call goes
through the general quad kernel (csrc/assign_quad.hip, env_kernel_q) for both
shortest-path rules.  sparse: the scipy rule goes through the quad-per-tree
sparse kernel (csrc/assign_sparse.hip, env_kernel_s) instead of the pair
kernel, on the Sioux Falls fixtures and on test_gpu_sparse.py's random
networks (against the C oracle).  Checks bit for bit and exits 0, or raises
(non-zero exit) on the first mismatch.

Fixtures: tests/golden/sf_reset_seed42_crpow.npz (msa/fw resets),
sf_random_resets_crpow.npz (32 random resets + 4 steps, scipy rule),
sf_torchsp_crpow.npz (torch rule resets + random resets + steps), all
generated from the reference (tools/gen_golden*.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def golden(name):
    return os.path.join(ROOT, "tests", "golden", name)


def make(gd, tg, B, method, iters, sp):
    from trafficrl.env import VecRepairEnv
    return VecRepairEnv(gd, B, device="cuda", assignment_method=method, assignment_iters=iters, graph=tg,
                        reset=False, reward_mode="rel_improve", reward_beta=0.0, reward_gamma=0.0, reward_clip=2.0,
                        unassigned_penalty=1e4, sp_backend=sp)


def main():
    kind = os.environ.get("TRX_KERNEL")
    assert kind in ("quad", "sparse"), kind
    scipy_k = "env_kernel_q" if kind == "quad" else "env_kernel_s"
    torch_k = "env_kernel_q" if kind == "quad" else "env_kernel_t"
    from trafficrl.data import sioux_falls
    from trafficrl.graph import TrafficGraph
    gd = sioux_falls()
    tg = TrafficGraph(gd)
    eq = np.testing.assert_array_equal
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    for key, m, k in (("msa30", "msa", 30), ("fw30", "fw", 30), ("msa60", "msa", 60), ("fw2", "fw", 2)):
        env = make(gd, tg, 2, m, k, "scipy")
        assert env.kernel_name == scipy_k, env.kernel_name
        env.reset(damaged=torch.from_numpy(np.repeat(r[key + "_damaged"][None], 2, 0)), observe=False)
        for b in range(2):
            eq(env.flow[b].cpu().numpy(), r[key + "_flow"])
            eq(env.t[b].cpu().numpy(), r[key + "_t"])
            assert float(env.tstt[b]) == float(r[key + "_tstt"])
    z = np.load(golden("sf_random_resets_crpow.npz"))
    env = make(gd, tg, len(z["seeds"]), "msa", 30, "scipy")
    env.reset(damaged=torch.from_numpy(z["damaged"]), observe=False)
    eq(env.flow.cpu().numpy(), z["flow"])
    eq(env.tstt.cpu().numpy(), z["tstt"])
    for j in range(4):
        _, rew, done, _ = env.step(torch.from_numpy(z["step_actions"][:, j]), observe=False)
        eq(env.flow.cpu().numpy(), z["step_flow"][:, j])
        eq(env.tstt.cpu().numpy(), z["step_tstt"][:, j])
        eq(rew.cpu().numpy(), z["step_reward"][:, j])
    t = np.load(golden("sf_torchsp_crpow.npz"))
    for key, m, k in (("msa30", "msa", 30), ("fw30", "fw", 30)):
        env = make(gd, tg, 2, m, k, "torch")
        assert env.kernel_name == torch_k, env.kernel_name
        env.reset(damaged=torch.from_numpy(np.repeat(t[key + "_damaged"][None], 2, 0)), observe=False)
        for b in range(2):
            eq(env.flow[b].cpu().numpy(), t[key + "_flow"])
            assert float(env.tstt[b]) == float(t[key + "_tstt"])
    env = make(gd, tg, len(t["rand_seeds"]), "msa", 30, "torch")
    env.reset(damaged=torch.from_numpy(t["rand_damaged"]), observe=False)
    eq(env.flow.cpu().numpy(), t["rand_flow"])
    eq(env.tstt.cpu().numpy(), t["rand_tstt"])
    for j in range(4):
        _, rew, _, _ = env.step(torch.from_numpy(t["rand_step_actions"][:, j]), observe=False)
        eq(env.flow.cpu().numpy(), t["rand_step_flow"][:, j])
        eq(env.tstt.cpu().numpy(), t["rand_step_tstt"][:, j])
        eq(rew.cpu().numpy(), t["rand_step_reward"][:, j])
    if kind == "sparse":
        sparse_cases()
    torch.cuda.synchronize()
    print(f"{kind} worker ok")


def sparse_cases():
    """test_gpu_sparse.py's random networks that the pair kernel takes by default,
    through env_kernel_s, against the C oracle."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from test_gpu_sparse import CASES, case_network
    from trafficrl.env import VecRepairEnv
    from trafficrl.graph import TrafficGraph
    for case in CASES:
        if case[7] != "env_kernel_pair":
            continue
        gd = case_network(case)
        tg = TrafficGraph(gd)
        og = O.OracleGraph(case[0], tg.src, tg.dst, tg.t0, tg.cap0, tg.od_o, tg.od_d, tg.od_v)
        E = tg.num_edges
        rng = np.random.default_rng(100 + case[3])
        B = 96
        dmg = (rng.random((B, E)) < 0.25).astype(np.float32)
        cap = np.where(dmg > 0, np.float32(1e-3), tg.cap0).astype(np.float32)
        flow0 = np.zeros((B, E), np.float32)
        flow0[B // 2:] = (rng.random((B - B // 2, E)) * 3000).astype(np.float32)
        for method in ("msa", "fw", "cfw"):
            f_o, t_o, ts_o, _ = og.assign(cap, dmg, flow0, method=method, iters=8, nthreads=8, penalty=2e7)
            env = VecRepairEnv(gd, B, device="cuda", assignment_method=method, assignment_iters=8, graph=tg,
                               reset=False)
            assert env.kernel_name == "env_kernel_s", env.kernel_name
            env.capacity.copy_(torch.from_numpy(cap))
            env.damaged.copy_(torch.from_numpy(dmg))
            env.flow.copy_(torch.from_numpy(flow0))
            env.assign()
            np.testing.assert_array_equal(env.flow.cpu().numpy(), f_o)
            np.testing.assert_array_equal(env.tstt.cpu().numpy(), ts_o)


if __name__ == "__main__":
    main()

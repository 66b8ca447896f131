"""Env rows after training vs the C oracle, every row (diagnostic for the 8-rank
rehearsal's oracle check, tests/test_dist_gpu.py): one process trains the Trainer
(4096 envs, random damage, MSA-30, hidden 32) for a few iterations, then runs one
warm-started assignment (trx_assign) of the whole batch from its state and
compares every row with oracle/trx_oracle.c.  Mismatching rows' inputs and both
results go to gpurun_out/trainer_mismatch_<kernel>.npz.

usage: python tools/trainer_oracle_check.py [iters] [envs]   (TRX_KERNEL=sparse: the quad kernel;
TRX_CHECK_SP=scipy|torch: the shortest-path rule, default the trainer config's)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    envs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    import oracle as O
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    cfg.update(sp_backend=os.environ.get("TRX_CHECK_SP", cfg["sp_backend"]), num_envs=envs, batch_start=64, batch_size=32, hidden_dim=32, embed_dim=32, eval_every=0,
               output_dir="/tmp/trx_oracle_check", update_every=4, update_unit="iterations", her_ratio=0.5,
               assignment_method="msa", assignment_iters=30, fixed_damage=False, early_stop_patience=10 ** 6,
               episodes=10 ** 6, max_steps=0)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr.run(max_iters=iters)
    env = tr.env
    kname = env.kernel_name
    torch.cuda.synchronize()
    cap = env.capacity.cpu().numpy()
    dmg = env.damaged.cpu().numpy()
    flow0 = env.flow.cpu().numpy()
    env.assign()
    torch.cuda.synchronize()
    f_d, t_d, ts_d = env.flow.cpu().numpy(), env.t.cpu().numpy(), env.tstt.cpu().numpy()
    og = O.OracleGraph.from_npz(os.path.join(ROOT, "tests", "golden", "sf_graph.npz"))
    from trafficrl import _lib
    sp = "torch" if env.params.sp_rule == _lib.SP_TORCH else "scipy"   # the env's own rule
    f_o, t_o, ts_o, _ = og.assign(cap, dmg, flow0, method="msa", iters=30, nthreads=16,
                                  penalty=float(env.params.unassigned_penalty), sp=sp)
    bad = np.nonzero(np.any(f_d != f_o, axis=1) | (ts_d != ts_o))[0]
    print(f"{kname}: {len(bad)} of {envs} rows differ from the oracle after {iters} training iterations"
          f"{' (first: ' + str(bad[:8].tolist()) + ')' if len(bad) else ''}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"trainer_state_{kname}.npz"), cap=cap, dmg=dmg,
                        flow0=flow0, flow_dev=f_d, tstt_dev=ts_d)
    if len(bad):
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"trainer_mismatch_{kname}.npz"), rows=bad,
                            cap=cap[bad], dmg=dmg[bad], flow0=flow0[bad], flow_dev=f_d[bad], flow_oracle=f_o[bad],
                            t_dev=t_d[bad], t_oracle=t_o[bad], tstt_dev=ts_d[bad], tstt_oracle=ts_o[bad])
    return 1 if len(bad) else 0


if __name__ == "__main__":
    sys.exit(main())

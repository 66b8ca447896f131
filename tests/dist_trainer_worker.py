"""Worker for tests/test_dist_gpu.py: one rank of a data-parallel Trainer run
on a shared GPU over gloo (TRX_DIST_BACKEND rehearsal of the RCCL path), or a
single rank over nccl (RCCL) itself.  TRX_WORKER_HIDDEN sets hidden = embed
(32: the autograd update path; 256: the fused update and its flat buffer);
TRX_WORKER_UNIT / TRX_WORKER_EVERY set update_unit / update_every
("transitions" with random damage: per-env episode lengths differ, so the
ranks' due-update counts differ and train.updates_due must deal them out).
TRX_WORKER_ENVS / TRX_WORKER_BATCH / TRX_WORKER_BUFFER / TRX_WORKER_AMP /
TRX_WORKER_ITERS / TRX_WORKER_SP set envs per rank, SAC batch, replay capacity,
autocast dtype, assignment iterations and shortest-path rule (config #4's shard:
4096 envs, batch 256, bf16, MSA-30, the bench's scipy rule; the trainer's own
default is the reference config's torch rule); TRX_WORKER_ORACLE=1 re-runs one warm-started assignment of the whole
shard after training and checks sampled rows against the C oracle
(oracle/trx_oracle.c) bit for bit.

Each rank trains `iters` vector iterations with HIP-graph updates (3 eager
warm-ups, then the update captured as two graphs around the eager gradient
all-reduce) and writes its parameters to <out>/rank<r>.pt.
Usage (env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT):
    python dist_trainer_worker.py <out_dir> <iters> <sync 0|1> <method>
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out, iters, sync, method = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    backend = os.environ.get("TRX_DIST_BACKEND", "gloo")
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend)
    hid = int(os.environ.get("TRX_WORKER_HIDDEN", "32"))
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    nenv = int(os.environ.get("TRX_WORKER_ENVS", "64"))
    cfg.update(num_envs=nenv, batch_start=64, batch_size=int(os.environ.get("TRX_WORKER_BATCH", "32")),
               buffer_size=int(os.environ.get("TRX_WORKER_BUFFER", str(cfg["buffer_size"]))),
               amp=os.environ.get("TRX_WORKER_AMP") or None, hidden_dim=hid, embed_dim=hid, eval_every=0,
               output_dir=os.path.join(out, f"run{rank}"), update_every=int(os.environ.get("TRX_WORKER_EVERY", "1")),
               update_unit=os.environ.get("TRX_WORKER_UNIT", "iterations"),
               her_ratio=0.5, assignment_method=method,
               assignment_iters=int(os.environ.get("TRX_WORKER_ITERS", "10")), fixed_damage=False,
               sp_backend=os.environ.get("TRX_WORKER_SP", cfg["sp_backend"]),
               early_stop_patience=10 ** 6, episodes=10 ** 6, max_steps=0)
    tr = Trainer(cfg, device="cuda:0", rank=rank, world=world if sync else 1, log=False)
    if not sync:
        tr.agent.grad_sync = None
    elif world == 1:  # one rank: the all-reduce is the identity, but its code path (RCCL) runs
        from trafficrl.train import GradAllReduce
        tr.agent.grad_sync = GradAllReduce(1, tr.agent)
    hist = tr.run(max_iters=iters)
    identity = None
    if sync and world == 1 and tr.agent.grad_flat is not None:
        # one more reduce of the last update's flat gradient buffer: on one rank it
        # must hand every value back unchanged
        before = tr.agent.grad_flat.clone()
        tr.agent.grad_sync(tr.agent.gradients())
        torch.cuda.synchronize()
        identity = bool(torch.equal(before, tr.agent.grad_flat))
    oracle_rows = None
    if os.environ.get("TRX_WORKER_ORACLE") == "1":
        oracle_rows = check_rows_vs_oracle(tr.env, method, int(cfg["assignment_iters"]), rank)
    sd = {f"{m}.{k}": v.detach().cpu() for m in ("actor", "critic1", "critic2", "target1", "target2")
          for k, v in getattr(tr.agent, m).state_dict().items()}
    sd["log_alpha"] = tr.agent.log_alpha.detach().cpu()
    torch.save({"params": sd, "episodes": tr.episodes_done, "history": len(hist), "updates": tr.updates_done,
                "transitions": tr._transitions,
                "graphed": tr._graphed is not None and tr._graphed.g_grads is not None,
                "split": tr._graphed is not None and tr._graphed.g_apply is not None,
                "reduce_calls": dict(tr.agent.grad_sync.calls) if tr.agent.grad_sync is not None else None,
                "identity": identity, "oracle_rows": oracle_rows},
               os.path.join(out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def check_rows_vs_oracle(env, method, iters, rank):
    """One warm-started assignment (trx_assign) of the rank's whole shard from its
    state after training; sampled rows must equal the C oracle's bit for bit."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    og = O.OracleGraph.from_npz(os.path.join(ROOT, "tests", "golden", "sf_graph.npz"))
    B = env.flow.shape[0]
    rows = sorted({0, 1, B // 3, B // 2 + rank, B - 1})
    cap = env.capacity[rows].cpu().numpy()
    dmg = env.damaged[rows].cpu().numpy()
    flow0 = env.flow[rows].cpu().numpy()
    env.assign()
    torch.cuda.synchronize()
    from trafficrl import _lib
    sp = "torch" if env.params.sp_rule == _lib.SP_TORCH else "scipy"   # the env's own rule
    f_o, t_o, ts_o, _ = og.assign(cap, dmg, flow0, method=method, iters=iters, nthreads=4,
                                  penalty=float(env.params.unassigned_penalty), sp=sp)
    np.testing.assert_array_equal(env.flow[rows].cpu().numpy(), f_o)
    np.testing.assert_array_equal(env.t[rows].cpu().numpy(), t_o)
    np.testing.assert_array_equal(env.tstt[rows].cpu().numpy(), ts_o)
    return rows


if __name__ == "__main__":
    main()

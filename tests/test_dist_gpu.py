"""Multi-rank trainer on one GPU (config #4's data-parallel path, rehearsed).

Two ranks share the card over gloo (the RCCL path's collectives through
torch.distributed; TRX_DIST_BACKEND=gloo in bench.py), each with its own env
shard (random damage: the host-side reset path), replay shard and PER draws.
After several HIP-graph updates -- 3 eager warm-ups, then the update captured
as two graphs around the eager gradient all-reduce (train.GraphedUpdate) --
both ranks must hold bit-identical parameters (one bucketed all-reduce per
update, src/rl/sac.py:157-263 semantics), while the same run without the
all-reduce diverges.  Ranks are separate processes started with subprocess
(no exec from a GPU-initialised process).
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp, sync, method="fw", iters=12, world=2, extra=None, timeout=240):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0", **(extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_trainer_worker.py"), str(tmp),
                                       str(iters), str(int(sync)), method], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o.decode(errors="replace"))
    bad = [(r, o) for r, (p, o) in enumerate(zip(procs, outs)) if p.returncode != 0]
    # the rank that failed first, not its peers' "connection closed"
    bad.sort(key=lambda ro: "Connection closed" in ro[1])
    assert not bad, "\n".join(f"--- rank {r}:\n{o[-2500:]}" for r, o in bad[:2])
    return [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(world)]


def test_two_ranks_stay_identical_with_graphed_updates(tmp_path):
    res = _run(tmp_path, sync=True, iters=26)
    assert all(r["graphed"] and r["split"] for r in res), [(r["graphed"], r["split"]) for r in res]
    p0, p1 = res[0]["params"], res[1]["params"]
    assert set(p0) == set(p1)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k
    assert res[0]["episodes"] == res[1]["episodes"]   # episode bookkeeping is collective
    # and the updates did move the weights (vs a fresh agent with the same seed)
    from trafficrl.rl.sac import DiscreteSAC
    torch.manual_seed(42)
    fresh = DiscreteSAC(4, 6, 32, 32, num_layers=3, share_critic_encoder=False)
    moved = sum(not torch.equal(fresh.actor.state_dict()[k], p0["actor." + k]) for k in fresh.actor.state_dict())
    assert moved > 0


def test_two_ranks_transition_schedule_random_damage(tmp_path):
    """update_unit "transitions" (the reference's per-env schedule, update_every
    4) with random damage: the ranks' envs finish episodes at different steps,
    so their due-update counts differ every iteration; train.updates_due sums
    them over the ranks and deals them out evenly, so both ranks run the same
    number of updates (each one all-reduces) and end bit-identical."""
    extra = {"TRX_WORKER_UNIT": "transitions", "TRX_WORKER_EVERY": "4"}
    res = _run(tmp_path, sync=True, iters=14, extra=extra)
    assert res[0]["updates"] == res[1]["updates"] > 20, (res[0]["updates"], res[1]["updates"])
    assert all(r["graphed"] and r["split"] for r in res)
    for k in res[0]["params"]:
        assert torch.equal(res[0]["params"][k], res[1]["params"][k]), k
    assert res[0]["episodes"] == res[1]["episodes"]


def test_two_ranks_diverge_without_allreduce(tmp_path):
    res = _run(tmp_path, sync=False, iters=8)
    p0, p1 = res[0]["params"], res[1]["params"]
    assert any(not torch.equal(p0[k], p1[k]) for k in p0)


def test_rccl_single_rank_flat_all_reduce(tmp_path):
    """The nccl (RCCL) branch itself, which two ranks on one GPU cannot take: one
    rank trains with the fused update (hidden = embed = 256), its gradients
    reduced in place in the flat buffer by RCCL (GradAllReduce's flat path,
    never the bucket) between the two captured update graphs; a final reduce
    of the last flat buffer hands every value back unchanged (one rank: the
    identity)."""
    extra = {"TRX_DIST_BACKEND": "nccl", "TRX_WORKER_HIDDEN": "256"}
    a = _run(tmp_path, sync=True, iters=10, world=1, extra=extra)[0]
    assert a["graphed"] and a["split"], (a["graphed"], a["split"])
    assert a["reduce_calls"]["flat"] > 0 and a["reduce_calls"]["bucket"] == 0, a["reduce_calls"]
    assert a["identity"] is True
    for k, v in a["params"].items():
        assert bool(torch.isfinite(v.float()).all()), k


def test_eight_ranks_config4_sharding(tmp_path):
    """Config #4's sharding rehearsed on the one GPU: 8 ranks over gloo, 4096 envs
    each (32,768 in all), MSA-30, GAT-SAC at the bench's shapes (hidden = embed =
    256, batch 256, bf16 autocast: the fused update and its flat gradient buffer),
    random damage, one all-reduce per update, replay capacity split over the ranks.
    Every rank ends with bit-identical parameters and the same update and episode
    counts, and each rank's sampled env rows equal the C oracle after training.
    Unmeasured on hardware: RCCL over xGMI needs the 8-GPU node."""
    extra = {"TRX_WORKER_HIDDEN": "256", "TRX_WORKER_ENVS": "4096", "TRX_WORKER_BATCH": "256",
             "TRX_WORKER_BUFFER": "200000", "TRX_WORKER_AMP": "bf16", "TRX_WORKER_ITERS": "30",
             "TRX_WORKER_UNIT": "iterations", "TRX_WORKER_EVERY": "2", "TRX_WORKER_ORACLE": "1",
             "TRX_WORKER_SP": "scipy"}
    # 3 eager warm-up updates, then the captured graphs (every 2nd iteration: 10 updates)
    res = _run(tmp_path, sync=True, method="msa", iters=20, world=8, extra=extra, timeout=600)
    assert all(r["graphed"] and r["split"] for r in res), [(r["graphed"], r["split"]) for r in res]
    assert len({r["updates"] for r in res}) == 1 and res[0]["updates"] >= 6, [r["updates"] for r in res]
    assert len({r["episodes"] for r in res}) == 1
    assert all(r["reduce_calls"]["flat"] > 0 for r in res)
    assert all(r["oracle_rows"] for r in res)
    for r in res[1:]:
        for k in res[0]["params"]:
            assert torch.equal(res[0]["params"][k], r["params"][k]), k


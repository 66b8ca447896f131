"""N>1 path on CPU (gloo, world_size 2): the SAC gradient bucket all-reduce
(trafficrl.train.GradAllReduce, the only data-parallel collective) averages
every gradient and leaves ranks bit-identical -- both the concatenated bucket
and the zero-copy in-place reduction of the fused update's flat gradient
buffer; the bench's max-over-ranks timing reduction picks the slowest rank."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trafficrl.train import GradAllReduce
    torch.manual_seed(100 + rank)
    grads = [torch.randn(7, 3), torch.randn(11), torch.randn(2, 2, 2)]
    mine = [g.clone() for g in grads]
    GradAllReduce(world)(grads)
    gathered = [None] * world
    dist.all_gather_object(gathered, [g for g in mine])
    mean = [sum(x[i] for x in gathered) / world for i in range(len(mine))]
    ok = all(torch.allclose(a, b, atol=1e-6) for a, b in zip(grads, mean))
    # zero-copy path: gradients that are views of the agent's flat buffer (the
    # fused update's layout) are reduced in place, the buffer itself reduced once
    from types import SimpleNamespace
    flat = torch.randn(30)
    views = [flat[0:21].view(7, 3), flat[21:29], flat[29:30]]
    before = flat.clone()
    red = GradAllReduce(world, SimpleNamespace(grad_flat=flat))
    assert red._flat_of(views) is flat and red._flat_of([torch.zeros(3)]) is None
    red(views)
    allb = [None] * world
    dist.all_gather_object(allb, before)
    ok = ok and torch.allclose(flat, sum(allb) / world, atol=1e-6)
    ok = ok and views[1].data_ptr() == flat.data_ptr() + 21 * 4          # still views: nothing copied back
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, ok, float(t), [g.sum().item() for g in grads]))
    dist.destroy_process_group()


def test_grad_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] for r in res)
    assert res[0][2] == res[1][2] == 1.5
    assert res[0][3] == res[1][3]  # identical averaged gradients on both ranks

"""Diagnostic: run identical work twice and report the largest differences."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_sac import _batch  # noqa: E402
from trafficrl.models import GATConv  # noqa: E402
from trafficrl.rl.sac import DiscreteSAC  # noqa: E402

torch.manual_seed(0)
gen = torch.Generator().manual_seed(0)
batch = _batch(8, "cuda", gen)
node_x, ei, ea = batch[0], batch[1], batch[2]
conv = GATConv(4, 64, heads=4, edge_dim=6).cuda()
outs, grads = [], []
for r in range(5):
    x = node_x.clone().requires_grad_(True)
    o = conv(x, ei, ea)
    g = torch.autograd.grad(o.square().sum(), [x] + list(conv.parameters()))
    outs.append(o.detach())
    grads.append(g)
print("gatconv fwd max diff", max((outs[0] - o).abs().max().item() for o in outs))
for i, name in enumerate(["x"] + [n for n, _ in conv.named_parameters()]):
    print("  grad", name, max((grads[0][i] - g[i]).abs().max().item() for g in grads))
for share in (False, True):
    kw = dict(hidden=64, embed=64, lr=1e-3, grad_clip=1.0, share_critic_encoder=share, device="cuda")
    torch.manual_seed(3)
    a = DiscreteSAC(4, 6, **kw)
    init = {n: {k: v.clone() for k, v in m.state_dict().items()} for n, m in
            (("actor", a.actor), ("critic1", a.critic1), ("critic2", a.critic2))}
    res = []
    for r in range(3):
        torch.manual_seed(3)
        b = DiscreteSAC(4, 6, **kw)
        for n, m in (("actor", b.actor), ("critic1", b.critic1), ("critic2", b.critic2)):
            m.load_state_dict(init[n])
        for o in (b.actor_opt, b.critic_opt, b.alpha_opt):
            for g_ in o.param_groups:
                g_["lr"] = 1e-2
        b.actor_opt = torch.optim.SGD(b.actor.parameters(), lr=1e-2)
        b.critic_opt = torch.optim.SGD(b.critic_params, lr=1e-2)
        b.update(batch, weights=np.ones(8, np.float32), alpha_max=2.5)
        res.append({n: {k: v.clone() for k, v in m.state_dict().items()} for n, m in
                    (("actor", b.actor), ("critic1", b.critic1), ("critic2", b.critic2))})
    worst = max(((res[0][n][k] - r[n][k]).abs().max().item(), n + "." + k) for r in res for n in res[0]
                for k in res[0][n])
    print("share", share, "update run-to-run worst", worst)

"""Which bf16 rounding sites make the actor's gradient differ from fp32?

CPU experiment over the fp32 restatement of the Actor (tests/test_sac_e2e.py,
reference src/rl/sac.py:35-46 over gat_encoder.py:32-53) at the bench's
hidden = embed = 256, batch 256 Sioux Falls graphs (synthetic features):
each GEMM site of bf16 autocast -- operands rounded to bf16, output rounded to
bf16, gradients rounded likewise (autograd.Function R) -- switched on alone,
all together, or all but one group.  Printed: the largest per-tensor relative
actor-gradient error vs fp32 (the floor of tests/test_fused_update.py _worst).
Result (profiles/r04_precision_sites.txt): every site costs 1-2.5 %, all of
them 6 %; no single one dominates, hence fp32_actor (rl/fused_update.py).

usage: python tools/precision_sites.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from test_gat import batched_graph  # noqa: E402

torch.manual_seed(0)
ON = set()


class R(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return x.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return (g.bfloat16().float() if ctx.g else g), None


def rnd(x, site, grad=True):
    return R.apply(x, grad) if site in ON else x


def lin(site, x, w, b=None):
    # autocast: bf16 operands, fp32 accumulate, bf16 output; grads likewise
    y = F.linear(rnd(x, site), rnd(w, site), None)
    if b is not None:
        y = y + b   # addmm with bias in bf16 too; ignore
    return rnd(y, site + "_out")


def gat(conv, x, ei, ea, tag):
    H, C = conv.heads, conv.out_channels
    N = x.size(0)
    xh = lin(tag, x, conv.lin.weight).view(N, H, C)
    a_s = (xh * conv.att_src).sum(-1)
    a_d = (xh * conv.att_dst).sum(-1)
    cnt = torch.zeros(N).index_add_(0, ei[1], torch.ones(ei.size(1)))
    loop_attr = torch.zeros(N, ea.size(1)).index_add_(0, ei[1], ea) / cnt.clamp(min=1).unsqueeze(1)
    loops = torch.arange(N)
    ei = torch.cat([ei, torch.stack([loops, loops])], 1)
    ea = torch.cat([ea, loop_attr], 0)
    e = lin("edge", ea, conv.lin_edge.weight).view(-1, H, C)
    a_e = (e * conv.att_edge).sum(-1)
    logit = F.leaky_relu(a_s[ei[0]] + a_d[ei[1]] + a_e, conv.negative_slope)
    amax = torch.full((N, H), float("-inf")).scatter_reduce(0, ei[1].unsqueeze(1).expand(-1, H), logit,
                                                            reduce="amax", include_self=True)
    ex = torch.exp(logit - amax[ei[1]])
    ssum = torch.zeros(N, H).index_add_(0, ei[1], ex)
    alpha = ex / (ssum[ei[1]] + 1e-16)
    out = torch.zeros(N, H, C).index_add_(0, ei[1], alpha.unsqueeze(-1) * xh[ei[0]])
    return out.reshape(N, H * C) + conv.bias


def head(net, nx, ei, ex, batch, B):
    x = F.layer_norm(nx, net.node_norm.normalized_shape, net.node_norm.weight, net.node_norm.bias, net.node_norm.eps)
    ea = F.layer_norm(ex, net.edge_norm.normalized_shape, net.edge_norm.weight, net.edge_norm.bias, net.edge_norm.eps)
    enc = net.encoder
    h = x
    L = len(enc.layers)
    for i, conv in enumerate(enc.layers):
        out = gat(conv, h, ei, ea, f"gat{i}")
        norm = enc.norms[i]
        if i < L - 1:
            x_in = lin("inproj", h, enc.input_proj.weight, enc.input_proj.bias) if i == 0 else h
            h = torch.relu(F.layer_norm(out, norm.normalized_shape, norm.weight, norm.bias, norm.eps) + x_in)
        else:
            h = F.elu(F.layer_norm(out, norm.normalized_shape, norm.weight, norm.bias, norm.eps))
        h = rnd(h, f"act{i}")
    C = h.size(1)
    cnt = torch.zeros(B).index_add_(0, batch, torch.ones(batch.numel()))
    mean = torch.zeros(B, C).index_add_(0, batch, h) / cnt.unsqueeze(1)
    mx = torch.full((B, C), float("-inf")).scatter_reduce(0, batch.unsqueeze(1).expand(-1, C), h, reduce="amax",
                                                          include_self=True)
    ctx = torch.cat([mean, mx], 1)
    src, dst = ei
    eb = batch[src]
    z = torch.cat([h[src], h[dst], ea, ctx[eb]], 1)
    l0, l2 = net.edge_mlp[0], net.edge_mlp[2]
    hid = torch.relu(lin("mlp0", z, l0.weight, l0.bias))
    return lin("mlp2", hid, l2.weight, l2.bias).squeeze(-1), eb


def main():
    from trafficrl.rl.sac import DiscreteSAC
    B = 256
    ei, batch, N, E = batched_graph(B, "cpu")
    ag = DiscreteSAC(4, 6, 256, 256, num_layers=3, lr=1e-4, grad_clip=1.0, share_critic_encoder=False,
                     alpha_init=0.1, target_entropy_ratio=0.2, device="cpu", amp_dtype=None)
    g = torch.Generator().manual_seed(1)
    nx = torch.rand(B * N, 4, generator=g) * torch.tensor([1.0, 5.0, 1.0, 0.2])
    ex = torch.rand(B * E, 6, generator=g) * torch.tensor([1.0, 3.0, 1.0, 1.0, 0.5, 1.0])
    mask = (torch.rand(B * E, generator=g) < 0.3).float()
    mask.view(B, E)[:, 0] = 1
    with torch.no_grad():
        q = torch.min(head(ag.critic1, nx, ei, ex, batch, B)[0], head(ag.critic2, nx, ei, ex, batch, B)[0])

    def actor_grads():
        ag.actor.zero_grad(set_to_none=True)
        lg, eb = head(ag.actor, nx, ei, ex, batch, B)
        lg = lg.masked_fill(mask <= 0, -1e9)
        mx = torch.full((B,), float("-inf")).scatter_reduce(0, eb, lg, reduce="amax", include_self=True)
        e = (lg - mx[eb]).exp()
        p = e / (torch.zeros(B).index_add_(0, eb, e) + 1e-16)[eb]
        loss = torch.zeros(B).index_add_(0, eb, p * (0.1 * torch.log(p + 1e-8) - q)).mean()
        loss.backward()
        return {n: pp.grad.clone() for n, pp in ag.actor.named_parameters() if pp.grad is not None}

    ref = actor_grads()
    floor = 1e-2 * float(torch.stack([v.norm() for v in ref.values()]).pow(2).mean().sqrt())

    def worst(got):
        errs = sorted(((float((got[k] - ref[k]).norm()) / (float(ref[k].norm()) + floor), k) for k in ref),
                      reverse=True)
        return errs[0]

    allsites = ["gat0", "gat1", "gat2", "edge", "inproj", "mlp0", "mlp2"]
    outs = [s + "_out" for s in allsites]
    acts = ["act0", "act1", "act2"]
    full = set(allsites + outs + acts)
    configs = {"all": full}
    for grp, names in (("no_gat_lin", ["gat0", "gat1", "gat2", "gat0_out", "gat1_out", "gat2_out"]),
                       ("no_mlp", ["mlp0", "mlp2", "mlp0_out", "mlp2_out"]),
                       ("no_mlp0", ["mlp0", "mlp0_out"]), ("no_mlp2", ["mlp2", "mlp2_out"]),
                       ("no_acts", acts), ("no_outs", outs), ("no_inproj", ["inproj", "inproj_out"]),
                       ("no_edge", ["edge", "edge_out"])):
        configs[grp] = full - set(names)
    for s in sorted(full):
        configs["only_" + s] = {s}
    for name, on in configs.items():
        ON.clear()
        ON.update(on)
        print(f"{name:16s} {worst(actor_grads())}", flush=True)


main()

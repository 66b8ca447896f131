"""Fused GAT-SAC inference (csrc/gat_infer.hip, models/fused.py) against the
general autograd path of the same modules, both under bf16 autocast.

The fused kernels round to bf16 at the same points as autocast but reduce in
a different order (attention dot products, LayerNorm moments, pooling), so
the comparison is to bf16 precision: node embeddings within 3e-2 absolute
(LayerNorm-scaled values of magnitude ~1), logits within 2% of their range,
probabilities within 1e-2 absolute, and each graph's fused greedy action
within 1e-2 probability of the general path's best.  The batch is real
environment observations (Sioux Falls, 64 envs with random damage) so
feature scales are the trainer's.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _obs_batch(B=64, seed=0):
    from trafficrl.data import sioux_falls
    from trafficrl.env import VecRepairEnv
    from trafficrl.train import batched_topology
    env = VecRepairEnv(sioux_falls(), B, device="cuda", seeds=list(range(seed, seed + B)), reset=False)
    obs = env.reset()
    N, E = env.num_nodes, env.num_edges
    ei, bv = batched_topology(env.edge_index, N, B)
    return (obs.node_x.reshape(B * N, 4).clone(), ei, obs.edge_x.reshape(B * E, 6).clone(),
            obs.action_mask.reshape(-1).clone(), bv, B, E)


def _both(fn):
    from trafficrl.rl import sac
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        sac.FUSED_INFERENCE = False
        ref = fn()
        sac.FUSED_INFERENCE = True
        got = fn()
    torch.cuda.synchronize()
    return ref, got


@pytest.mark.parametrize("seed", [0, 1])
def test_actor_fused_matches_general(seed):
    from trafficrl.rl.sac import Actor
    torch.manual_seed(seed)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=seed)
    (lr, pr, _), (lf, pf, _) = _both(lambda: actor(node_x, ei, ea, mask, bv, num_graphs=B))
    valid = mask > 0
    span = (lr[valid].max() - lr[valid].min()).item()
    assert torch.isfinite(pf).all()
    assert (lf[valid] - lr[valid]).abs().max().item() <= 0.02 * span + 1e-3
    assert torch.equal(lf[~valid], lr[~valid])                      # masked to -1e9 on both
    assert (pf - pr).abs().max().item() < 1e-2
    torch.testing.assert_close(pf.view(B, E).sum(1), torch.ones(B, device="cuda"), atol=1e-5, rtol=0)
    # greedy actions agree up to near-ties: the fused argmax is (one of) the
    # general path's best links within the probability tolerance
    af = pf.view(B, E).argmax(1)
    prv = pr.view(B, E)
    gap = prv.max(1).values - prv.gather(1, af[:, None]).squeeze(1)
    assert gap.max().item() < 1e-2
    print(f"max|dlogit| {(lf[valid] - lr[valid]).abs().max().item():.3e} (span {span:.3f}), "
          f"max|dprob| {(pf - pr).abs().max().item():.3e}, argmax agree "
          f"{(af == prv.argmax(1)).float().mean().item():.3f}")


def test_critic_fused_matches_general():
    from trafficrl.rl.sac import Critic
    torch.manual_seed(3)
    critic = Critic(4, 6, 256, 256, 3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=5)
    qr, qf = _both(lambda: critic(node_x, ei, ea, bv, B))
    span = (qr.max() - qr.min()).item()
    assert (qf - qr).abs().max().item() <= 0.02 * span + 1e-3


def test_encoder_fused_matches_general():
    from trafficrl.models import fused
    from trafficrl.models.gat_encoder import GATEncoder
    torch.manual_seed(7)
    enc = GATEncoder(4, 256, 256, edge_dim=6, heads=4, num_layers=3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=9)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        emb_r, ctx_r, _ = enc(node_x, ei, ea, bv, num_graphs=B)
        topo = fused.topology(ei, bv, B)
        assert topo is not None and topo.n == 24 and topo.e == 76 and topo.max_graph_edges == 100
        emb_f, ctx_f = fused.encoder_infer(enc, node_x, ea, topo)
    de = (emb_f.float() - emb_r.float()).abs().max().item()
    dc = (ctx_f - ctx_r.float()).abs().max().item()
    print(f"max|d emb| {de:.3e}, max|d ctx| {dc:.3e}")
    assert de < 3e-2 and dc < 3e-2


def test_irregular_batch_takes_general_path():
    """Graphs of different sizes: no fused topology, same call still works."""
    from trafficrl.models import fused
    from trafficrl.rl.sac import Actor
    torch.manual_seed(2)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    sizes = [5, 9, 7]
    x, eis, bvs, off = [], [], [], 0
    for b, n in enumerate(sizes):
        src = torch.arange(n)
        dst = (src + 1) % n
        eis.append(torch.stack([torch.cat([src, dst]), torch.cat([dst, src])]) + off)
        bvs.append(torch.full((n,), b))
        off += n
    ei = torch.cat(eis, 1).cuda()
    bv = torch.cat(bvs).cuda()
    node_x = torch.randn(off, 4, device="cuda")
    ea = torch.randn(ei.shape[1], 6, device="cuda")
    mask = torch.ones(ei.shape[1], device="cuda")
    assert fused.topology(ei, bv, len(sizes)) is None
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        _, probs, _ = actor(node_x, ei, ea, mask, bv, num_graphs=len(sizes))
    assert torch.isfinite(probs).all()
    sums = torch.zeros(len(sizes), device="cuda").index_add_(0, bv[ei[0]], probs)
    torch.testing.assert_close(sums, torch.ones(len(sizes), device="cuda"), atol=1e-5, rtol=0)


def test_prologue_matches_torch_ops():
    """trx_gat_prologue_infer (input LayerNorms, self-loop means, every
    layer's a_edge in CSR order) against the same quantities from torch ops:
    LayerNorm outputs to fp32 rounding, a_edge to one bf16 ulp (the 6-term
    dot products are summed in another order before the bf16 rounding)."""
    from trafficrl.models import fused
    from trafficrl.models.gat_encoder import _LoopMean
    from trafficrl.rl.sac import Actor
    torch.manual_seed(5)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=3)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        topo = fused.topology(ei, bv, B)
        x0, ean, a_all = fused.prologue(actor, node_x, ea, topo)
        lnf = torch.nn.functional.layer_norm
        x_ref = lnf(node_x.float(), (4,), actor.node_norm.weight, actor.node_norm.bias, actor.node_norm.eps)
        e_ref = lnf(ea.float(), (6,), actor.edge_norm.weight, actor.edge_norm.bias, actor.edge_norm.eps)
        g = topo.g
        full = torch.cat([e_ref, _LoopMean.apply(e_ref, g)], 0)
        Ms = [(l.lin_edge.weight.view(l.heads, l.out_channels, -1) * l.att_edge.view(l.heads, l.out_channels, 1))
              .sum(1) for l in actor.encoder.layers]
        a_ref = (full @ torch.cat(Ms, 0).t())[g.perm].float()
    torch.testing.assert_close(x0, x_ref.float(), atol=2e-6, rtol=2e-6)
    torch.testing.assert_close(ean, e_ref.float(), atol=2e-6, rtol=2e-6)
    assert a_all.shape == a_ref.shape
    torch.testing.assert_close(a_all, a_ref, atol=1e-3, rtol=1.6e-2)


def test_fused_draw_is_inverse_cdf_of_probs():
    """select_actions' in-kernel categorical draw: for each graph and uniform
    u the action is the first link whose cumulative probability exceeds u
    (checked in float64, skipping u within 1e-5 of a boundary), masked links
    are never drawn, and the action frequencies over many draws follow the
    probabilities."""
    from trafficrl.models import fused
    from trafficrl.rl.sac import Actor
    torch.manual_seed(6)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=5)
    gen = torch.Generator(device="cuda").manual_seed(2)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        counts = torch.zeros(B, E, device="cuda", dtype=torch.float64)
        for _ in range(200):
            u = torch.rand(B, device="cuda", generator=gen)
            logits, probs, act = actor._fused(node_x, ei, ea, bv, B, mask=mask, u=u)
            cdf = probs.view(B, E).double().cumsum(1)
            want = (cdf <= u.double()[:, None]).sum(1).clamp(max=E - 1)
            near = ((cdf - u.double()[:, None]).abs() < 1e-5).any(1)
            assert torch.equal(act[~near], want[~near])
            assert bool((mask.view(B, E).gather(1, act[:, None]) > 0).all())
            counts[torch.arange(B, device="cuda"), act] += 1
    freq = counts / 200
    p = probs.view(B, E).double()
    # binomial standard error at n=200 is <= 0.036; 5 sigma
    assert (freq - p).abs().max().item() < 0.18


def test_edge_scores_training_kernels_match_torch_ops():
    """Training-path edge scorer (trx_edge_head_infer forward + trx_edge_head_
    backward) against the autograd torch ops of _EdgeHead.edge_scores under
    bf16 autocast: logits and the gradients of node embeddings, context,
    link features and the edge-MLP weights to bf16 precision."""
    from trafficrl.rl import sac
    from trafficrl.rl.sac import Critic, regular_layout
    torch.manual_seed(7)
    critic = Critic(4, 6, 256, 256, 3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(B=32, seed=9)
    N = node_x.shape[0]
    g = torch.Generator(device="cuda").manual_seed(3)
    emb = torch.randn(N, 256, device="cuda", generator=g).requires_grad_()
    ctx = torch.randn(B, 512, device="cuda", generator=g).requires_grad_()
    eat = torch.randn(B * E, 6, device="cuda", generator=g).requires_grad_()
    gl = torch.randn(B * E, device="cuda", generator=g)
    src, dst = ei
    reg = regular_layout(ei, bv, B)

    def run(flag):
        sac.FUSED_EDGE_TRAIN = flag
        for t in [emb, ctx, eat] + list(critic.edge_mlp.parameters()):
            t.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg = critic.edge_scores(emb, ctx, eat, src, dst, bv[src], reg).float()
        lg.backward(gl)
        grads = [t.grad.float().clone() for t in [emb, ctx, eat] + list(critic.edge_mlp.parameters())]
        return lg.detach(), grads

    try:
        ref_l, ref_g = run(False)
        got_l, got_g = run(True)
    finally:
        sac.FUSED_EDGE_TRAIN = True
    span = (ref_l.max() - ref_l.min()).item()
    assert (got_l - ref_l).abs().max().item() <= 0.01 * span + 1e-3
    names = ["emb", "ctx", "edge_attr", "W1", "b1", "W2", "b2"]
    for name, a, b in zip(names, got_g, ref_g):
        scale = b.abs().max().item() + 1e-6
        err = (a - b).abs().max().item()
        assert err <= 0.03 * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def test_prepared_weights_follow_updates():
    """The fused no-grad path reuses prepared bf16 weight copies between
    updates.  A parameter change the version counter does not see (what a
    HIP-graph replay of the SAC update does; emulated with .data) must reach
    the kernels once fused.weights_changed() is called -- Trainer.update and
    DiscreteSAC.apply_gradients call it after every update."""
    from trafficrl.models import fused
    from trafficrl.rl.sac import Actor
    torch.manual_seed(8)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(B=16, seed=2)

    def logits():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return actor._fused(node_x, ei, ea, bv, B, mask=mask)[0].clone()

    before = logits()
    torch.testing.assert_close(logits(), before, atol=0, rtol=0)      # cached copies reproduce the result
    actor.edge_mlp[0].weight.data.mul_(-1.0)                           # invisible to the version counter
    actor.encoder.layers[1].lin.weight.data.mul_(0.5)
    fused.weights_changed()
    after = logits()
    (ref, _, _), _ = _both(lambda: actor(node_x, ei, ea, mask, bv, num_graphs=B))
    valid = mask > 0
    assert not torch.allclose(after[valid], before[valid])
    # to bf16 precision of the logits' magnitude (the span can be tiny here)
    assert (after[valid] - ref[valid]).abs().max().item() <= 1e-2 * ref[valid].abs().max().item() + 1e-3


def test_layer0_linear_form_matches_fp32_restatement():
    """trx_gat_layer0_infer (csrc/gat_layer0.hip: attention logits as 4-dots,
    aggregate of the raw features, LayerNorm moments as float64 forms)
    against layer 0 restated in plain fp32 torch ops from the same inputs
    (the prologue's normalised features and edge logits in CSR order):
    GATConv lin, per-head <xh, att> logits, leaky ReLU 0.2, softmax over each
    node's in-edges (+1e-16), aggregate + bias, LayerNorm, + input_proj,
    ReLU (src/models/gat_encoder.py:36-47).  Both outputs (fp32 residual,
    bf16 GEMM input) within 2e-5 relative to the row scale / one bf16 ulp."""
    from trafficrl.models import fused
    from trafficrl.rl.sac import Actor
    torch.manual_seed(11)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    with torch.no_grad():   # non-trivial LayerNorm / bias parameters
        for p in (actor.encoder.layers[0].bias, actor.encoder.norms[0].weight, actor.encoder.norms[0].bias):
            p.add_(0.1 * torch.randn_like(p))
    enc = actor.encoder
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=13)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        topo = fused.topology(ei, bv, B)
        x0, eaf, a_all = fused.prologue(actor, node_x, ea, topo)
        N = x0.shape[0]
        out32 = torch.empty(N, 1024, device="cuda")
        out16 = torch.empty(N, 1024, device="cuda", dtype=torch.bfloat16)
        fused.layer0_infer(enc, x0, topo, a_all, 0, out32, out16)
    torch.cuda.synchronize()
    l0, ln, ip = enc.layers[0], enc.norms[0], enc.input_proj
    H, C = l0.heads, l0.out_channels
    with torch.no_grad():
        x = x0.double()
        xh = x @ l0.lin.weight.double().t()
        a_s = (xh.view(N, H, C) * l0.att_src.double().view(1, H, C)).sum(-1)
        a_d = (xh.view(N, H, C) * l0.att_dst.double().view(1, H, C)).sum(-1)
        rp, col = topo.g.rowptr.long(), topo.g.col.long()
        dst = torch.repeat_interleave(torch.arange(N, device="cuda"), rp.diff())
        logit = torch.nn.functional.leaky_relu(a_s[col] + a_d[dst] + a_all[:, :H].double(), 0.2)
        mx = torch.full((N, H), -1e300, device="cuda", dtype=torch.float64).scatter_reduce(
            0, dst[:, None].expand(-1, H), logit, "amax")
        ex = torch.exp(logit - mx[dst])
        den = torch.zeros(N, H, device="cuda", dtype=torch.float64).index_add_(0, dst, ex) + 1e-16
        alpha = ex / den[dst]
        agg = torch.zeros(N, H, C, device="cuda", dtype=torch.float64).index_add_(
            0, dst, alpha[:, :, None] * xh.view(N, H, C)[col]).reshape(N, H * C)
        v = agg + l0.bias.double()
        y = torch.nn.functional.layer_norm(v, (H * C,), ln.weight.double(), ln.bias.double(), ln.eps)
        ref = torch.relu(y + x @ ip.weight.double().t() + ip.bias.double())
    scale = ref.abs().amax(1, keepdim=True).clamp(min=1e-3)
    err = ((out32.double() - ref).abs() / scale).max().item()
    print(f"layer0 linear form: max error / row scale {err:.2e}")
    assert err < 2e-5
    torch.testing.assert_close(out16, out32.to(torch.bfloat16), rtol=0, atol=0)   # one rounding of the same row


def test_actor_layer0_kernels_agree():
    """The acting pass with the linear-form layer 0 and with the round-3
    layer kernel (bf16 projection) agree to bf16 precision."""
    from trafficrl.models import fused
    from trafficrl.rl.sac import Actor
    torch.manual_seed(4)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=21)
    outs = []
    for lin in (False, True):
        fused.LAYER0_LINEAR = lin
        try:
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                outs.append(actor(node_x, ei, ea, mask, bv, num_graphs=B))
        finally:
            fused.LAYER0_LINEAR = True
    (l0, p0, _), (l1, p1, _) = outs
    valid = mask > 0
    span = (l0[valid].max() - l0[valid].min()).item()
    assert (l1[valid] - l0[valid]).abs().max().item() <= 0.02 * span + 1e-3
    assert (p1 - p0).abs().max().item() < 1e-2


def test_mid_layer_regenerated_residual_matches_stored_residual():
    """trx_gat_mid_infer (layer 1 with layer 0's output regenerated from the
    per-node descriptor) against trx_gat_layer_infer fed with layer 0's
    float32 rows from HBM: the same function, the LayerNorm sums taken in
    another order -- within 1e-5 of the row scale (bf16 outputs within one
    bf16 ulp)."""
    import torch.nn.functional as F
    from trafficrl import _lib
    from trafficrl.models import fused
    from trafficrl.rl.sac import Actor
    torch.manual_seed(17)
    actor = Actor(4, 6, 256, 256, 3).cuda()
    enc = actor.encoder
    assert fused.mid_supported(enc)
    node_x, ei, ea, mask, bv, B, E = _obs_batch(seed=23)
    L = _lib.load()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        topo = fused.topology(ei, bv, B)
        x0, eaf, a_all = fused.prologue(actor, node_x, ea, topo)
        N = x0.shape[0]
        y0 = torch.empty(N, 1024, device="cuda")
        y0b = torch.empty(N, 1024, device="cuda", dtype=torch.bfloat16)
        desc = torch.empty(N, 24, device="cuda")
        fused.layer0_infer(enc, x0, topo, a_all, 0, y0, y0b, desc)
        w1 = fused.prepared_encoder(enc, list(enc.layers))[1]
        xh = F.linear(y0b, w1)
        got32 = torch.empty(N, 1024, device="cuda")
        got16 = torch.empty(N, 1024, device="cuda", dtype=torch.bfloat16)
        fused.mid_infer(enc, xh, desc, topo, a_all, 4, got32, got16)
        # the round-3 layer kernel with the stored float32 residual
        l1, n1 = enc.layers[1], enc.norms[1]
        args = _lib.TrxGatLayerArgs()
        args.num_graphs, args.nodes_per_graph, args.heads, args.channels = B, topo.n, l1.heads, l1.out_channels
        args.concat, args.max_graph_edges, args.in_dim, args.xh = 1, topo.max_graph_edges, 0, xh.data_ptr()
        args.rowptr, args.col = topo.g.rowptr.data_ptr(), topo.g.col.data_ptr()
        args.a_edge, args.a_edge_stride, args.a_edge_offset = a_all.data_ptr(), a_all.shape[1], 4
        keep = [l1.att_src.detach().reshape(-1).contiguous(), l1.att_dst.detach().reshape(-1).contiguous()]
        args.att_src, args.att_dst, args.bias = keep[0].data_ptr(), keep[1].data_ptr(), l1.bias.detach().data_ptr()
        args.negative_slope = float(l1.negative_slope)
        args.ln_weight, args.ln_bias, args.ln_eps = n1.weight.detach().data_ptr(), n1.bias.detach().data_ptr(), n1.eps
        args.residual, args.res, args.activation = 1, y0.data_ptr(), 0
        ref32 = torch.empty(N, 1024, device="cuda")
        args.out_f32 = ref32.data_ptr()
        _lib.check(L.trx_gat_layer_infer(args, _lib.stream_ptr(y0.device)), "trx_gat_layer_infer")
    torch.cuda.synchronize()
    scale = ref32.abs().amax(1, keepdim=True).clamp(min=1e-3)
    err = ((got32 - ref32).abs() / scale).max().item()
    print(f"mid layer: max error / row scale {err:.2e}")
    assert err < 1e-5
    torch.testing.assert_close(got16, got32.to(torch.bfloat16), rtol=0, atol=0)

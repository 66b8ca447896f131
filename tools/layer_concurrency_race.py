"""Is one network's fused training forward deterministic when copies of it
run concurrently on side streams of a captured HIP graph?

The same critic forward (rl/fused_update.py net_forward, save=True: prologue,
three GAT layer kernels with saves, GEMMs, edge scorer) on the same batch is
captured on S side streams at once and replayed; every saved tensor of every
branch is compared with branch 0 of the same replay and with the first
replay.  Identical inputs, so any difference is a race.

usage: python tools/layer_concurrency_race.py [streams] [replays] [what]
what: train (save=True, the default) | next (save=False)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from test_gat import batched_graph
    from trafficrl.models import fused
    from trafficrl.rl import fused_update as FU
    from trafficrl.rl.sac import DiscreteSAC
    from trafficrl import train as T

    S = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    save = (sys.argv[3] if len(sys.argv) > 3 else "train") == "train"
    dev = "cuda"
    torch.manual_seed(0)
    B = 256
    ei, bv, N, E = batched_graph(B, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    nx = torch.rand(B * N, 4, device=dev, generator=g)
    ex = torch.rand(B * E, 6, device=dev, generator=g)
    ag = DiscreteSAC(4, 6, 256, 256, num_layers=3, share_critic_encoder=False, device=dev,
                     amp_dtype=torch.bfloat16, capturable=True)
    topo = fused.topology(ei, bv, B)
    net = ag.critic1
    side = [torch.cuda.Stream() for _ in range(S)]

    def flat(lg, cx):
        ts = {"logits": lg}
        if cx is not None:
            for key in ("x0", "ea", "a_all", "emb", "ctx", "p", "c"):
                ts[key] = getattr(cx, key)
            for i, r in enumerate(cx.layers):
                for key, t in r.items():
                    if isinstance(t, torch.Tensor):
                        ts[f"L{i}.{key}"] = t
        return ts

    chain = os.environ.get("TRX_RACE_CHAIN") == "1"   # branch k waits for branch k-1: streams without concurrency

    def body():
        main_s = torch.cuda.current_stream()
        outs = []
        for k, st in enumerate(side):
            st.wait_stream(side[k - 1] if chain and k > 0 else main_s)
            with torch.cuda.stream(st), torch.no_grad():
                outs.append(flat(*FU.net_forward(net, nx, ex, topo, save=save)))
        for st in side:
            main_s.wait_stream(st)
        return outs

    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        body()
    torch.cuda.current_stream().wait_stream(s0)
    torch.cuda.synchronize()
    held = []
    if os.environ.get("TRX_RACE_HOLD") == "1":   # no block freed during the capture: no memory reuse at all
        _empty, _empty_like = torch.empty, torch.empty_like

        def empty(*a, **k):
            t = _empty(*a, **k)
            held.append(t)
            return t

        def empty_like(*a, **k):
            t = _empty_like(*a, **k)
            held.append(t)
            return t
        torch.empty, torch.empty_like = empty, empty_like
    gr, outs = T.capture_graph(body)
    first = None
    diffs = {}
    for r in range(R):
        gr.replay()
        torch.cuda.synchronize()
        snap = [{k: v.clone() for k, v in o.items()} for o in outs]
        if first is None:
            first = snap[0]
        for b, o in enumerate(snap):
            for k, v in o.items():
                if not torch.equal(v, first[k]):
                    diffs[k] = diffs.get(k, 0) + 1
    print(f"{S} concurrent {'training' if save else 'no-grad'} forwards, {R} replays: tensors differing "
          f"(name: branch-replays out of {S * R}): {sorted(diffs.items())}", flush=True)


if __name__ == "__main__":
    main()

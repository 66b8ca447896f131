"""How much do independent network passes overlap when replayed from HIP
graphs?  Three copies of one critic's training forward (batch 256, hidden =
embed = 256, rl/fused_update.py net_forward) are captured

  serial    -- one graph, one stream, the three passes back to back;
  branches  -- one graph, the passes on three side streams forked from and
               joined into the capture stream (the shipped update's pattern);
  separate  -- three graphs, each captured on its own side stream, replayed on
               those streams with events (fork / join outside the graphs);

and each is replayed 30 times (HIP events, median of 5 rounds).
usage: python tools/branch_probe.py [copies]"""
import os
import statistics
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
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = "cuda"
    B = 256
    torch.manual_seed(0)
    ei, bv, N, E = batched_graph(B, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    nx = torch.rand(B * N, 4, device=dev, generator=g)
    ex = torch.rand(B * E, 6, device=dev, generator=g)
    ag = DiscreteSAC(4, 6, 256, 256, num_layers=3, share_critic_encoder=False, device=dev,
                     amp_dtype=torch.bfloat16, capturable=True)
    topo = fused.topology(ei, bv, B)
    nets = [ag.critic1, ag.critic2, ag.target1][:S] if S <= 3 else [ag.critic1] * S
    side = [torch.cuda.Stream() for _ in range(S)]
    keep = []

    def fwd(net):
        with torch.no_grad():
            keep.append(FU.net_forward(net, nx, ex, topo, save=True))

    for net in nets:   # warm-up (caches, allocator)
        fwd(net)
    torch.cuda.synchronize()

    def serial():
        for net in nets:
            fwd(net)

    def branches():
        m = torch.cuda.current_stream()
        for st, net in zip(side, nets):
            st.wait_stream(m)
            with torch.cuda.stream(st):
                fwd(net)
        for st in side:
            m.wait_stream(st)

    g_serial, _ = T.capture_graph(serial)
    g_branch, _ = T.capture_graph(branches)
    g_sep = []
    for st, net in zip(side, nets):
        gg = torch.cuda.CUDAGraph(keep_graph=True)
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(gg, stream=st, capture_error_mode="thread_local"):
            fwd(net)
        from trafficrl import _lib
        _lib.patch_graph_memsets(gg)
        gg.instantiate()
        g_sep.append(gg)
    torch.cuda.synchronize()

    def rep_sep():
        m = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(m)
        for st, gg in zip(side, g_sep):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                gg.replay()
        for st in side:
            m.wait_stream(st)

    def timeit(fn, K=30, R=5):
        ms = []
        for _ in range(R):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(K):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1) / K)
        return statistics.median(ms)

    for name, fn in (("serial", g_serial.replay), ("branches", g_branch.replay), ("separate", rep_sep),
                     ("serial", g_serial.replay), ("branches", g_branch.replay), ("separate", rep_sep)):
        print(f"{S} forwards, {name:9s}: {timeit(fn) * 1e3:8.1f} us per replay", flush=True)


if __name__ == "__main__":
    main()

"""Minimal HIP-graph replay checks on the plain torch.cuda.graph path:
captured memset nodes, full / column reductions, vector norms, memcpy nodes.
On ROCm 7.2 (packet capture on, the default) memset nodes < ~1 MiB do not
replay -- the column sum and memset lines show False / garbage after the
first replay; DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 fixes them at a large launch
cost.  --patched runs the same checks through trafficrl.train.capture_graph
(memset nodes rewritten into fill kernels), which must be all-correct.
Usage: python tools/graph_memset_check.py [--patched]
"""
import os
import sys
import torch


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def _capture(fn):
    if "--patched" in sys.argv:
        from trafficrl.train import capture_graph
        return capture_graph(fn)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def replay_check(name, setup, body, ref, replays=4):
    state = setup()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            body(state)
    torch.cuda.current_stream().wait_stream(side)
    g, out = _capture(lambda: body(state))
    res = []
    for r in range(replays):
        for t in state.values():
            if t.is_floating_point():
                t.normal_()
        g.replay()
        torch.cuda.synchronize()
        res.append(bool(torch.allclose(out.float(), ref(state).float(), rtol=1e-4, atol=1e-3)))
    print(f"{name:>40}: {res}", flush=True)


def main():
    replay_check("memset+add (int32[16])", lambda: {"z": torch.zeros(16, dtype=torch.int32, device="cuda")},
                 lambda s: s["z"].zero_().add_(1), lambda s: torch.ones(16, device="cuda"))
    replay_check("memset+add (float[1M])", lambda: {"z": torch.zeros(1 << 20, device="cuda")},
                 lambda s: s["z"].zero_().add_(1), lambda s: torch.ones(1 << 20, device="cuda"))
    for n in (1 << 12, 1 << 16, 1 << 20):
        replay_check(f"full sum fp32 [{n}]", lambda n=n: {"x": torch.randn(n, device="cuda")},
                     lambda s: s["x"].sum(), lambda s: s["x"].double().sum())
    replay_check("vector_norm fp32 [1M]", lambda: {"x": torch.randn(1 << 20, device="cuda")},
                 lambda s: torch.linalg.vector_norm(s["x"]), lambda s: s["x"].double().norm())
    replay_check("col sum fp32 [6144,1024]", lambda: {"x": torch.randn(6144, 1024, device="cuda")},
                 lambda s: s["x"].sum(0), lambda s: s["x"].double().sum(0))
    replay_check("col sum fp32 [98304,4]", lambda: {"x": torch.randn(98304, 4, device="cuda")},
                 lambda s: s["x"].sum(0), lambda s: s["x"].double().sum(0))


if __name__ == "__main__":
    main()


def memset_node_check(nbytes_list=(4, 64, 4096, 1 << 20), replays=4):
    """hipMemsetAsync captured into a graph (the call torch's multi-block
    reductions use to clear their semaphores) followed by an add."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    for nbytes in nbytes_list:
        z = torch.zeros(max(1, nbytes // 4), dtype=torch.int32, device="cuda")
        rcs = []

        def body():
            st = torch.cuda.current_stream().cuda_stream
            rcs.append(hip.hipMemsetAsync(ctypes.c_void_p(z.data_ptr()), 0, nbytes, ctypes.c_void_p(st)))
            z.add_(1)

        g, _ = _capture(body)
        rc = rcs[0]
        res = []
        for _ in range(replays):
            g.replay()
            torch.cuda.synchronize()
            res.append(int(z.max()))
        print(f"memset node {nbytes:>8} B (rc {rc}): z.max after replays {res}  (1 = memset replayed)", flush=True)


if __name__ == "__main__":
    memset_node_check()


def memcpy_node_check(sizes=(1, 16, 1024, 1 << 20), replays=4):
    """Device-to-device copies (torch copy_ -> hipMemcpyAsync) captured into a
    graph: does each replay copy the current source?"""
    for n in sizes:
        a = torch.zeros(n, device="cuda")
        b = torch.zeros(n, device="cuda")
        g, _ = _capture(lambda: b.copy_(a))
        res = []
        for r in range(replays):
            a.fill_(float(r + 1))
            g.replay()
            torch.cuda.synchronize()
            res.append(float(b.max()) == float(r + 1) and float(b.min()) == float(r + 1))
        print(f"memcpy node {4 * n:>8} B: replays correct {res}", flush=True)


if __name__ == "__main__":
    memcpy_node_check()

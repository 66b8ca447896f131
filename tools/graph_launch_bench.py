"""Cost per node of HIP-graph replay vs eager launches for a chain of tiny
kernels (the shape of the SAC update: ~1500 small kernels).
Usage: python tools/graph_launch_bench.py [n_kernels]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def main():
    from trafficrl.train import capture_graph
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    x = torch.zeros(4096, device="cuda")

    def body():
        for _ in range(n):
            x.add_(1.0)

    body()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        body()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / 5
    g, _ = capture_graph(body)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / 5
    print(f"{n} tiny kernels: eager {eager * 1e3:.2f} ms ({eager / n * 1e6:.1f} us/kernel), "
          f"graph replay {graph * 1e3:.2f} ms ({graph / n * 1e6:.1f} us/node) "
          f"[env {os.environ.get('DEBUG_HIP_GRAPH_BATCH_SIZE', '-')}/{os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '-')}"
          f"/{os.environ.get('DEBUG_HIP_FORCE_GRAPH_QUEUES', '-')}]", flush=True)


if __name__ == "__main__":
    main()

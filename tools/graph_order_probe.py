"""Does the capture order of a graph's parallel branches decide how they overlap on
replay?  Three branches of K dependent small kernels each (an elementwise op on a
batch-256-sized tensor, the update's kernel scale), forked from and joined into the
capture stream, captured two ways:

  blocked     -- branch 0's K launches, then branch 1's, then branch 2's (how the
                 SAC update's branches are issued today);
  interleaved -- launch k of branch 0, 1, 2, then launch k + 1 of each, ...

plus the single-stream serial graph for scale.  Each graph is replayed R times
back to back (HIP events).  Usage: python tools/graph_order_probe.py [K] [R]"""
import statistics
import sys

import torch


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda:0")
    xs = [torch.randn(6144, 256, device=dev) for _ in range(3)]
    streams = [torch.cuda.Stream(dev) for _ in range(3)]

    def op(x):
        x.mul_(1.0001).add_(1e-4)    # two dependent launches per step

    def build(mode):
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            cur = torch.cuda.current_stream()
            if mode == "serial":
                for i in range(3):
                    for _ in range(K):
                        op(xs[i])
                return g
            for s in streams:
                s.wait_stream(cur)
            if mode == "blocked":
                for i, s in enumerate(streams):
                    with torch.cuda.stream(s):
                        for _ in range(K):
                            op(xs[i])
            else:
                for _ in range(K):
                    for i, s in enumerate(streams):
                        with torch.cuda.stream(s):
                            op(xs[i])
            for s in streams:
                cur.wait_stream(s)
        return g

    graphs = {m: build(m) for m in ("serial", "blocked", "interleaved")}
    for rnd in range(3):
        for m, g in graphs.items():
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(R):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            print(f"round {rnd} {m:>12}: {e0.elapsed_time(e1) / R * 1e3:8.1f} us per replay "
                  f"({3 * 2 * K} kernels)", flush=True)


if __name__ == "__main__":
    main()

"""Do multi-branch HIP graphs keep their fork / join dependencies on replay?

Each captured body: a producer on the capture stream, NB side-stream branches
forked from it (chains of elementwise kernels of different lengths reading the
producer's output), a join, and a consumer that sums the branches.  Before
every replay the static input is set to a new value, so a branch that starts
before its producer or a consumer that starts before a branch ends reads a
stale value and the replay's result differs from the eager computation.

usage: python tools/graph_branch_race.py"""
import torch

dev = "cuda"


def body(inp, side, NB, L):
    main = torch.cuda.current_stream()
    b = inp * 2.0 + 1.0
    outs = []
    for k in range(NB):
        st = side[k]
        st.wait_stream(main)
        with torch.cuda.stream(st):
            y = b
            for j in range(L + 3 * k):
                y = y * 1.0 + float(k + 1)
            outs.append(y)
    for st in side[:NB]:
        main.wait_stream(st)
    for o in outs:
        o.record_stream(main)
    return torch.stack(outs).sum(0)


def main():
    side = [torch.cuda.Stream() for _ in range(8)]
    for NB in (2, 3, 4, 5, 6, 8):
        for n in (1 << 12, 1 << 20):
            inp = torch.zeros(n, device=dev)
            L = 8
            s0 = torch.cuda.Stream()
            s0.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s0):
                body(inp, side, NB, L)
            torch.cuda.current_stream().wait_stream(s0)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = body(inp, side, NB, L)
            bad = 0
            for r in range(50):
                inp.fill_(float(r))
                g.replay()
                torch.cuda.synchronize()
                ref = body(inp, side, NB, L)
                torch.cuda.synchronize()
                bad += int(not torch.equal(out, ref))
            print(f"branches {NB} elems {n:8d}: {bad}/50 replays differ from eager", flush=True)


if __name__ == "__main__":
    main()

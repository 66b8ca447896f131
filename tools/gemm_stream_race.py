"""Are torch GEMMs on concurrent streams inside a captured HIP graph
bit-reproducible?  Each op kind runs on six side streams forked from the
capture stream (as compute_gradients_fused's forward does) and its results
are compared bitwise with the same op run alone, over 20 replays.

usage: python tools/gemm_stream_race.py"""
import torch
import torch.nn.functional as F

dev = "cuda"
torch.manual_seed(0)
N, K, M = 6144, 256, 256
xs = [torch.randn(N, K, device=dev).bfloat16() for _ in range(6)]
ws = [torch.randn(M, K, device=dev).bfloat16() for _ in range(6)]
cs = [torch.randn(256, 512, device=dev).bfloat16() for _ in range(6)]
wc = [torch.randn(512, 256, device=dev).bfloat16() for _ in range(6)]
bias = torch.randn(256, device=dev)

OPS = {
    "linear_bf16": lambda k: F.linear(xs[k], ws[k]),
    "mm_out_f32": lambda k: torch.mm(cs[k], wc[k], out_dtype=torch.float32),
    "addmm_out_f32": lambda k: torch.addmm(bias, cs[k], wc[k], out_dtype=torch.float32),
    "bmm_splitk": lambda k: torch.bmm(xs[k].view(4, N // 4, K).transpose(1, 2), xs[(k + 1) % 6].view(4, N // 4, K)),
    "linear_then_mm": lambda k: torch.mm(F.linear(xs[k], ws[k]), ws[(k + 2) % 6].t(), out_dtype=torch.float32),
}


def run(op, side):
    main = torch.cuda.current_stream()
    outs = []
    for k in range(6):
        st = side[k]
        st.wait_stream(main)
        with torch.cuda.stream(st):
            outs.append(op(k))
    for st in side:
        main.wait_stream(st)
    return outs


def main():
    side = [torch.cuda.Stream() for _ in range(6)]
    for name, op in OPS.items():
        ref = [op(k).clone() for k in range(6)]
        # warm on the side streams (workspaces, algorithm selection) outside the capture
        s0 = torch.cuda.Stream()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            for _ in range(2):
                run(op, side)
        torch.cuda.current_stream().wait_stream(s0)
        torch.cuda.synchronize()
        eager_bad = 0
        for _ in range(20):
            o = run(op, side)
            torch.cuda.synchronize()
            eager_bad += sum(int(not torch.equal(a, b)) for a, b in zip(o, ref))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            outs = run(op, side)
        bad = 0
        for _ in range(20):
            g.replay()
            torch.cuda.synchronize()
            bad += sum(int(not torch.equal(a, b)) for a, b in zip(outs, ref))
        print(f"{name:16s} eager mismatches {eager_bad}/120, graph mismatches {bad}/120", flush=True)


if __name__ == "__main__":
    main()

"""Is a GEMM's consumer ordered after it inside a multi-branch HIP graph?

Six side-stream branches, each: GEMM (F.linear bf16 / torch.mm out_dtype=
float32) -> an elementwise consumer of its output, as the fused update's
forwards do (GEMM -> GAT layer kernel).  The static input changes before
every replay; each replay's consumer outputs are compared with an eager run
of the same body.  A consumer that starts before its GEMM has finished reads
the previous replay's product.

usage: python tools/gemm_consumer_race.py"""
import torch
import torch.nn.functional as F

dev = "cuda"
N, K, M = 6144, 1024, 1024


def body(xs, ws, side, kind):
    main = torch.cuda.current_stream()
    outs = []
    for k, st in enumerate(side):
        st.wait_stream(main)
        with torch.cuda.stream(st):
            if kind == "linear_bf16":
                y = F.linear(xs[k], ws[k])
            elif kind == "mm_out_f32":
                y = torch.mm(xs[k], ws[k].t(), out_dtype=torch.float32)
            else:   # bmm split-K (the update's weight gradients)
                y = torch.bmm(xs[k].view(4, N // 4, K).transpose(1, 2), xs[k].view(4, N // 4, K)).sum(0)
            outs.append(y.float() * 0.5 + 1.0)
    for st in side:
        main.wait_stream(st)
    for o in outs:
        o.record_stream(main)
    return outs


def main():
    torch.manual_seed(0)
    side = [torch.cuda.Stream() for _ in range(6)]
    xs = [torch.randn(N, K, device=dev).bfloat16() for _ in range(6)]
    ws = [torch.randn(M, K, device=dev).bfloat16() * 0.03 for _ in range(6)]
    for kind in ("linear_bf16", "mm_out_f32", "bmm"):
        s0 = torch.cuda.Stream()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            for _ in range(2):
                body(xs, ws, side, kind)
        torch.cuda.current_stream().wait_stream(s0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            outs = body(xs, ws, side, kind)
        bad = 0
        for r in range(30):
            for x in xs:
                x.add_(0.25)   # a new input every replay
            g.replay()
            torch.cuda.synchronize()
            ref = body(xs, ws, side, kind)
            torch.cuda.synchronize()
            bad += sum(int(not torch.equal(a, b)) for a, b in zip(outs, ref))
        print(f"{kind:12s}: {bad}/180 branch outputs differ from eager", flush=True)


if __name__ == "__main__":
    main()

"""Probe: device time of the small context projection GEMM of the edge
scorer (ctx [256, 512] @ W_ctx^T, W_ctx a column slice of W1 [256, 1030])
in several layouts / dtypes.  Usage: python tools/mm_probe.py"""
import torch


def t(fn, reps=200):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


ctx = torch.randn(256, 512, device="cuda")
W1 = torch.randn(256, 1030, device="cuda")
Wc = W1[:, 518:]
xb, Wcb = ctx.bfloat16(), Wc.bfloat16().contiguous()
with torch.autocast("cuda", dtype=torch.bfloat16):
    print(f"autocast ctx @ W1[:, 518:].t()   {t(lambda: ctx @ Wc.t()):7.2f} us")
    print(f"autocast F.linear(ctx, Wc)      {t(lambda: torch.nn.functional.linear(ctx, Wc)):7.2f} us")
print(f"bf16 mm(x, Wc^T) contiguous W   {t(lambda: xb @ Wcb.t()):7.2f} us")
WcbT = Wcb.t().contiguous()
print(f"bf16 mm(x, WT) NN               {t(lambda: xb @ WcbT):7.2f} us")
print(f"fp32 mm                         {t(lambda: ctx @ Wc.t()):7.2f} us")
print(f"bf16 cast of Wc (strided)       {t(lambda: Wc.bfloat16()):7.2f} us")
for shp in ((6144, 1024, 1024), (6144, 1024, 256), (6144, 256, 512), (256, 6144, 1024)):
    a = torch.randn(shp[0], shp[2], device="cuda").bfloat16()
    b = torch.randn(shp[1], shp[2], device="cuda").bfloat16()
    print(f"bf16 linear {shp}  {t(lambda: torch.nn.functional.linear(a, b)):7.2f} us")



def tg(fn, reps=50):
    """device time per call from a captured graph of `reps` calls (no host gaps)"""
    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s_)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(5):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / (5 * reps) * 1e3


for lib in ("cublaslt", "cublas"):
    torch.backends.cuda.preferred_blas_library(lib)
    res = []
    for shp in ((256, 256, 512), (6144, 1024, 1024), (6144, 1024, 256), (1024, 1024, 6144), (6144, 256, 4),
                (6144, 512, 256)):
        a = torch.randn(shp[0], shp[2], device="cuda").bfloat16()
        b = torch.randn(shp[1], shp[2], device="cuda").bfloat16()
        res.append(f"{shp}: {tg(lambda: torch.nn.functional.linear(a, b)):6.2f}")
    print("graphed", lib, " | ".join(res))

torch.backends.cuda.preferred_blas_library("cublaslt")
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_max_tuning_duration(30)
res = []
for shp in ((256, 256, 512), (6144, 1024, 1024), (6144, 1024, 256), (1024, 1024, 6144), (6144, 256, 4),
            (6144, 512, 256), (98304, 1024, 1024)):
    a = torch.randn(shp[0], shp[2], device="cuda").bfloat16()
    b = torch.randn(shp[1], shp[2], device="cuda").bfloat16()
    torch.nn.functional.linear(a, b)  # tune outside the capture
    torch.cuda.synchronize()
    res.append(f"{shp}: {tg(lambda: torch.nn.functional.linear(a, b), reps=20):6.2f}")
print("graphed tunableop", " | ".join(res))

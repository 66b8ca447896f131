"""Kernel timeline of one graphed SAC update (the bench's update: batch 256,
Sioux Falls, hidden = embed = 256, float32 actor).

Run mode (under rocprofv3 --kernel-trace): prime the update (eager warm-ups +
capture), then replay it N times with a host sleep between replays, so each
update is an isolated burst of kernels in the trace.
    rocprofv3 --kernel-trace -d gpurun_out/updtl -o run --output-format csv -- python3 tools/upd_timeline.py run
Report mode (on the CSV): split the trace into bursts, take the median burst,
print its wall span, its kernels in start order (start offset, duration,
queue) and the time covered by at least one kernel (busy) vs idle gaps.
    python tools/upd_timeline.py report gpurun_out/updtl/<...>_kernel_trace.csv"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))


def run(n=12):
    import torch
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    cfg.update(num_envs=1024, batch_start=256, update_unit="iterations", eval_every=0, output_dir="/tmp/trx_upd",
               buffer_size=65536)
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    for it in range(4):
        obs, _ = tr.iteration(obs, it)
    tr.prime_update()
    for _ in range(n):
        torch.cuda.synchronize()
        time.sleep(0.02)
        tr.update()
    torch.cuda.synchronize()
    print("done", flush=True)


def short(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        mt = [p for p in name.split("_") if p.startswith("MT")]
        return "GEMM " + (mt[0] if mt else "")
    return name.replace("void ", "").replace("trx::", "").replace("(anonymous namespace)::", "")[:60]


def report(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    bursts, cur = [], []
    for r in rows:
        if cur and r[0] - max(x[1] for x in cur) > 5_000_000:   # > 5 ms gap: a new update
            bursts.append(cur)
            cur = []
        cur.append(r)
    bursts.append(cur)
    bursts = [b for b in bursts if len(b) > 50]
    spans = sorted((max(x[1] for x in b) - b[0][0], i) for i, b in enumerate(bursts))
    span, i = spans[len(spans) // 2]
    b = bursts[i]
    t0 = b[0][0]
    print(f"{len(bursts)} updates, spans (us): {[round(s / 1e3) for s, _ in spans]}")
    print(f"median update: {span / 1e3:.1f} us, {len(b)} kernels")
    busy, end = 0, t0
    for s, e, _, _ in b:
        if e > end:
            busy += e - max(s, end)
            end = e
    print(f"covered by >= 1 kernel: {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")
    tot = {}
    for s, e, n, q in b:
        k = short(n)
        tot[k] = tot.get(k, 0) + (e - s)
    print("kernel time by name (us):")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:30]:
        print(f"  {v / 1e3:8.1f}  {k}")
    print("timeline (start us, dur us, queue, kernel):")
    for s, e, n, q in b:
        print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q}  {short(n)}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2])

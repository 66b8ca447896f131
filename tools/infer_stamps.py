"""Diagnostic: per-phase cycle shares of the fused GAT layer kernel
(trafficrl/libtrafficrl_stamps.so from `make stamps`, loaded INSTEAD of the
shipped library) over acting passes at B graphs.  Usage: python tools/infer_stamps.py [B]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))
import torch  # noqa: E402
from trafficrl import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "sac-gat-her_transportationrl_amd", "trafficrl", "libtrafficrl_stamps.so")
L = _lib.load()
L.trx_debug_infer_cycles.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
from trafficrl.train import Trainer, sf_config  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cfg = sf_config()
cfg.update(num_envs=B, batch_start=10 ** 9, eval_every=0, output_dir="/tmp/trx_stamps", buffer_size=4096)
tr = Trainer(cfg, device="cuda:0", log=False)
tr._reset_envs(None)
obs = tr.env.observe()
tr.act(obs)
buf = (ctypes.c_ulonglong * 32)()
L.trx_debug_infer_cycles(buf, 1)
reps = 10
for _ in range(reps):
    tr.act(obs)
L.trx_debug_infer_cycles(buf, 0)
names = ["stage", "layer0 xh", "att dots", "edge logits", "softmax", "aggregate+LN", "pool sync", "pool"]
for row, title in enumerate(["layer 0 (HC 1024, IN 4)", "HC 1024", "HC 256 (last)", "edge scorer"]):
    vals = [buf[row * 8 + i] for i in range(8)]
    if row == 3:
        names = ["stage", "links", "softmax", "draw", "", "", "", ""]
    tot = sum(vals) or 1
    print(f"== {title}: {tot / reps / B:.0f} cycles per workgroup")
    for n, v in zip(names, vals):
        if v:
            print(f"{n:>14}: {v / tot * 100:6.2f} %  ({v / reps / B:.0f} cycles/WG)")

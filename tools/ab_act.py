"""A/B timing of the graphed acting pass (B envs, SF) for one build of
libtrafficrl.so per process: TRX_LIB=<lib.so> python tools/ab_act.py [B] [reps].
Prints the mean wall time per acting pass over `reps` replays (after warm-up)
(kernel times: rocprofv3 --kernel-trace --stats over the same command)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

import torch  # noqa: E402

from trafficrl.train import GEMM_TUNING_GFX950, Trainer, sf_config  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cfg = sf_config()
cfg.update(num_envs=B, batch_start=10 ** 9, eval_every=0, output_dir=f"/tmp/trx_abact_{os.getpid()}",
           buffer_size=4096, amp="bf16", gemm_tuning=GEMM_TUNING_GFX950)
tr = Trainer(cfg, device="cuda:0", log=False)
tr._reset_envs(None)
obs = tr.env.observe()
for _ in range(20):
    tr.act(obs)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    tr.act(obs)
torch.cuda.synchronize()
lib = os.path.basename(os.environ.get("TRX_LIB", "libtrafficrl.so"))
print(f"{lib}: act {(time.perf_counter() - t0) / reps * 1e3:.4f} ms/pass (B={B}, {reps} graph replays)", flush=True)

"""DiscreteSAC.apply_gradients over the fused update's flat gradient buffer.

The reference (src/rl/sac.py:224-263) clips and steps three Adam optimizers
(critics, actor, log_alpha), clamps log_alpha and Polyak-averages the target
critics.  After a fused update (rl/fused_update.py) every gradient is a view
of `agent.grad_flat`, so the whole step is trx_sac_adam: three launches
(csrc/sac_optim.hip) instead of ~40 torch launches.  The moments live in two
flat buffers here; when the agent takes the autograd path instead, the
moments and step counts are handed over to the torch optimizers (and back),
so both paths continue one Adam trajectory.
"""
from typing import List, Optional

import numpy as np
import torch

from .. import _lib

CHUNK = 8192   # floats per block of the norm / apply kernels


class FlatAdam:
    def __init__(self, agent):
        self.agent = agent
        crit = list(agent.critic1.parameters()) + list(agent.critic2.parameters())
        tgt = list(agent.target1.parameters()) + list(agent.target2.parameters())
        assert len(crit) == len(tgt) and all(p.shape == t.shape for p, t in zip(crit, tgt))
        self.groups = [crit, list(agent.actor.parameters()), [agent.log_alpha]]
        self.targets = tgt
        self.opts = [agent.critic_opt, agent.actor_opt, agent.alpha_opt]
        self.params: List[torch.Tensor] = [p for g in self.groups for p in g]
        self.moff, off = [], 0
        for p in self.params:
            self.moff.append(off)
            off += p.numel()
        dev = agent.log_alpha.device
        self.m = torch.zeros(off, device=dev)
        self.v = torch.zeros(off, device=dev)
        self.step_t = torch.zeros(3, device=dev)
        self.scal = torch.zeros(12, device=dev)
        self._key = None
        self.owner = "torch"    # who holds the live moments: "torch" optimizers or this object

    # ------------------------------------------------------------ state handoff
    def _pairs(self):
        k = 0
        for gi, (g, opt) in enumerate(zip(self.groups, self.opts)):
            for p in g:
                yield gi, p, opt, self.moff[k]
                k += 1

    @torch.no_grad()
    def import_torch(self):
        """Take the moments / step counts from the torch optimizers."""
        steps = [0.0, 0.0, 0.0]
        for gi, p, opt, mo in self._pairs():
            st = opt.state.get(p)
            n = p.numel()
            if st and "exp_avg" in st:
                self.m[mo:mo + n].copy_(st["exp_avg"].reshape(-1))
                self.v[mo:mo + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps[gi] = float(st["step"])
            else:
                self.m[mo:mo + n].zero_()
                self.v[mo:mo + n].zero_()
        self.step_t.copy_(torch.tensor(steps))
        self.owner = "flat"

    @torch.no_grad()
    def export_torch(self):
        """Write the moments / step counts back into the torch optimizers."""
        steps = self.step_t.cpu().tolist()
        for gi, p, opt, mo in self._pairs():
            n = p.numel()
            if steps[gi] == 0:
                opt.state.pop(p, None)
                continue
            cap = opt.defaults.get("capturable", False) or opt.defaults.get("fused", False)
            st = opt.state.setdefault(p, {})
            st["step"] = (torch.tensor(steps[gi], dtype=torch.float32, device=p.device) if cap
                          else torch.tensor(steps[gi], dtype=torch.float32))
            st["exp_avg"] = self.m[mo:mo + n].view_as(p).clone()
            st["exp_avg_sq"] = self.v[mo:mo + n].view_as(p).clone()
        self.owner = "torch"

    # ------------------------------------------------------------------ step
    def usable(self) -> bool:
        flat = getattr(self.agent, "grad_flat", None)
        if flat is None or self.agent.share_critic_encoder or not flat.is_cuda:
            return False
        base, end = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
        for p in self.params:
            g = p.grad
            if g is None or g.dtype != torch.float32 or not g.is_contiguous() or not (
                    base <= g.data_ptr() and g.data_ptr() + 4 * g.numel() <= end):
                return False
        return True

    def _tables(self, flat):
        base = flat.data_ptr()
        key = tuple((p.data_ptr(), (p.grad.data_ptr() - base) // 4) for p in self.params)
        if key == self._key:
            return
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("FlatAdam: gradient layout changed inside a graph capture")
        segs, blocks = [], []
        tg = {id(p): t for p, t in zip(self.groups[0], self.targets)}
        k = 0
        for gi, g in enumerate(self.groups):
            for p in g:
                goff = (p.grad.data_ptr() - base) // 4
                t = tg.get(id(p))
                segs.append((p.data_ptr(), t.data_ptr() if t is not None else 0, goff, self.moff[k], p.numel(), gi))
                for b0 in range(0, p.numel(), CHUNK):
                    blocks.append((k, b0, min(p.numel(), b0 + CHUNK), 0))
                k += 1
        seg_np = np.zeros(len(segs), dtype=[("p", "<u8"), ("t", "<u8"), ("goff", "<i8"), ("moff", "<i8"),
                                            ("n", "<i8"), ("group", "<i4"), ("pad", "<i4")])
        for i, s in enumerate(segs):
            seg_np[i] = s + (0,)
        dev = flat.device
        self.seg_t = torch.from_numpy(seg_np.view(np.uint8).copy()).to(dev)
        self.blk_t = torch.from_numpy(np.asarray(blocks, dtype=np.int32)).to(dev)
        self.partial = torch.zeros(len(blocks), device=dev)
        self.nseg, self.nblocks = len(segs), len(blocks)
        self._key = key

    def step(self, lrs, grad_clip: Optional[float], tau: float, alpha_max: Optional[float]):
        flat = self.agent.grad_flat
        if self.owner != "flat":
            self.import_torch()
        self._tables(flat)
        a = _lib.TrxAdamArgs()
        a.segs, a.blocks, a.nseg, a.nblocks = self.seg_t.data_ptr(), self.blk_t.data_ptr(), self.nseg, self.nblocks
        a.g_base, a.m, a.v = flat.data_ptr(), self.m.data_ptr(), self.v.data_ptr()
        a.partial, a.step, a.scal = self.partial.data_ptr(), self.step_t.data_ptr(), self.scal.data_ptr()
        clip = float(grad_clip) if grad_clip is not None and grad_clip > 0 else 0.0
        for i in range(3):
            a.lr[i] = float(lrs[i])
            a.max_norm[i] = clip
        b1, b2 = self.opts[0].defaults["betas"]
        a.beta1, a.beta2, a.eps, a.tau = float(b1), float(b2), float(self.opts[0].defaults["eps"]), float(tau)
        a.log_alpha_min = float(np.log(0.01))
        a.log_alpha_max = float(np.log(alpha_max)) if alpha_max is not None else float("inf")
        _lib.check(_lib.load().trx_sac_adam(a, _lib.stream_ptr(flat.device)), "trx_sac_adam")

"""Worker for tests/test_determinism.py: one single-rank Trainer run at the
bench's network sizes (hidden = embed = 256: the fused acting pass and the
fused, graphed SAC update on its default concurrent side streams) from fixed
seeds; writes per-iteration checksums
(actions, flows, the update's TD errors) and the final parameters.

Usage: python det_worker.py <out.pt> <iters> [fill_nan]
fill_nan = 1: the caching allocator's fresh blocks are poisoned with NaN
(PYTORCH_NO_... is not needed: every torch.empty of the run goes through
torch.empty, which this worker wraps), so a read of memory no kernel wrote
shows up as NaN instead of as run-to-run noise."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

import torch  # noqa: E402


def _digest(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    out, iters = sys.argv[1], int(sys.argv[2])
    fill = len(sys.argv) > 3 and sys.argv[3] == "1"
    if fill:
        _empty = torch.empty

        def poisoned(*a, **k):
            t = _empty(*a, **k)
            if t.is_cuda and t.is_floating_point():
                t.fill_(float("nan"))   # captured into a graph too: poisoned on every replay
            return t
        torch.empty = poisoned
    from trafficrl.train import Trainer, sf_config
    cfg = sf_config()
    cfg.update(num_envs=512, batch_start=512, batch_size=256, hidden_dim=256, embed_dim=256, eval_every=0,
               output_dir=os.path.join(os.path.dirname(out), "det_run"), update_every=1, update_unit="iterations",
               her_ratio=0.0, assignment_method="msa", assignment_iters=30, fixed_damage=True, fixed_damage_seed=42,
               sp_backend="scipy", early_stop_patience=10 ** 6, episodes=10 ** 6, max_steps=0, amp="bf16")
    tr = Trainer(cfg, device="cuda:0", log=False)
    tr._reset_envs(None)
    obs = tr.env.observe()
    trace = []
    acts = []
    orig_act = tr.act

    def act(o, *a, **k):
        r = orig_act(o, *a, **k)
        acts.append(_digest(r))
        return r
    tr.act = act
    for it in range(iters):
        obs, _ = tr.iteration(obs, it)
        torch.cuda.synchronize()
        rec = {"act": acts[-1], "flow": _digest(tr.env.flow), "tstt": _digest(tr.env.tstt)}
        if tr.last_losses:
            rec["td"] = _digest(tr.last_losses["td_errors"])
        bad = [f"{m}.{k}" for m in ("actor", "critic1", "critic2") for k, p in getattr(tr.agent, m).named_parameters()
               if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
        if bad:
            rec["nonfinite_grads"] = ",".join(bad)
            print(f"iteration {it}: non-finite gradients in {bad}", flush=True)
        print(f"iteration {it}: {rec.get('td', '-')}", flush=True)
        rec["actor"] = _digest(torch.cat([p.detach().reshape(-1) for p in tr.agent.actor.parameters()]))
        rec["critic1"] = _digest(torch.cat([p.detach().reshape(-1) for p in tr.agent.critic1.parameters()]))
        trace.append(rec)
    params = {f"{m}.{k}": v.detach().cpu() for m in ("actor", "critic1", "critic2", "target1", "target2")
              for k, v in getattr(tr.agent, m).state_dict().items()}
    torch.save({"trace": trace, "params": params, "graphed": tr._graphed is not None and tr._graphed.g_grads is not None,
                "update_path": tr.agent.last_update_path}, out)


if __name__ == "__main__":
    main()

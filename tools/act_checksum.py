"""A/B check: checksum of the acting pass's outputs (masked logits, probabilities,
draws) for a fixed random-init agent and fixed observations, with the library
TRX_LIB (or the shipped one).  Two builds that should compute the same function
print the same checksum.  Usage: TRX_LIB=<lib.so> python tools/act_checksum.py [B]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "sac-gat-her_transportationrl_amd")]
import torch  # noqa: E402

from test_sac_e2e import flat, make_agent, observations  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
env, obs, _ = observations(B)
agent = make_agent()
nx_, ei, ex_, mask, bv = flat(env, obs, B)
u = torch.rand(B, device="cuda", generator=torch.Generator("cuda").manual_seed(5))
with torch.no_grad(), agent._amp():
    lg, pr, act = agent.actor._fused(nx_, ei, ex_, bv, B, mask=mask, u=u)
    q = agent.critic1._fused(nx_, ei, ex_, bv, B)
h = hashlib.sha256()
for t in (lg, pr, act, q):
    h.update(t.detach().cpu().numpy().tobytes())
print(f"{os.path.basename(os.environ.get('TRX_LIB', 'libtrafficrl.so'))}: act checksum {h.hexdigest()[:16]}")

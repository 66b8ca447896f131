"""The reference's float32 PER sum tree (src/train.py:27-91) pinned bit for bit.

tests/golden/per_tree_ref.npz holds the reference ReplayBuffer's own outputs
(tools/gen_golden_r2.py): capacity 1000 (not a power of two, leaves at two
depths), 1500 adds (the ring wraps), three rounds of sample(256) with fixed
uniforms + update_priorities with float32 TD errors, then 300 more adds.

CPU: the restatement oracle/per_tree.py replays the protocol and must match
every tree, index, weight and max_priority exactly.  GPU: DeviceReplay with
tree_dtype="float32" (trx_per32_add_range / trx_per32_update /
trx_per32_sample) must match the same fixture -- trees, sampled indices and
max_priority bit-exact; IS weights within 4 float32 ulps (numpy's float32 pow
on the host vs the device powf) -- and the restatement at the reference's
buffer_size 1e6 with 4096-transition ring adds and repeated update indices.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from per_tree import RefTree

ADD_BATCHES = (700, 500, 300)     # 1500 adds in ring pieces (the second and third wrap)


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(golden("per_tree_ref.npz")))


def test_restatement_matches_reference_fixture(fx):
    rb = RefTree(int(fx["capacity"]), float(fx["alpha"]), float(fx["beta"]), float(fx["eps"]))
    for _ in range(1500):
        rb.add()
    np.testing.assert_array_equal(rb.tree, fx["tree_after_add"])
    for r in range(3):
        idx, _, w = rb.sample(fx[f"s{r}_u"])
        np.testing.assert_array_equal(idx, fx[f"s{r}_idx"])
        np.testing.assert_array_equal(w, fx[f"s{r}_w"])
        rb.update_priorities(idx, fx[f"s{r}_td"])
        np.testing.assert_array_equal(rb.tree, fx[f"s{r}_tree"])
        assert rb.max_p == float(fx[f"s{r}_max_p"])
    for _ in range(300):
        rb.add()
    np.testing.assert_array_equal(rb.tree, fx["tree_final"])
    assert (rb.ptr, rb.size, rb.max_p) == (int(fx["final_ptr"]), int(fx["final_size"]), float(fx["final_max_p"]))


def test_fixture_exercises_the_float32_semantics(fx):
    """The fixture is not also what a float64 tree would give: float32 delta
    propagation leaves the root different from the exact leaf sum."""
    t = fx["tree_final"]
    cap = int(fx["capacity"])
    assert float(t[1]) != float(np.sum(t[cap:].astype(np.float64)))


def _device_replay(cap, fx_or_none=None, device="cuda"):
    from trafficrl.rl.replay import DeviceReplay
    kw = {} if fx_or_none is None else dict(alpha=float(fx_or_none["alpha"]), beta=float(fx_or_none["beta"]),
                                            eps=float(fx_or_none["eps"]))
    return DeviceReplay(cap, 1, 1, node_dim=1, edge_dim=1, device=device, tree_dtype="float32", **kw)


def _adds(rb, B):
    d = rb.device
    z = lambda *s, **kw: torch.zeros(*s, device=d, **kw)
    rb.add_batch(z(B, 1, 1), z(B, 1, 1), z(B, 1), torch.zeros(B, dtype=torch.int64, device=d), z(B), z(B, 1, 1),
                 z(B, 1, 1), z(B, 1), z(B), z(B, 1), z(B, dtype=torch.float64), z(B, dtype=torch.float64),
                 z(B, dtype=torch.float64))


def _ulps32(a, b):
    a, b = np.asarray(a, np.float32).view(np.int32), np.asarray(b, np.float32).view(np.int32)
    return np.abs(a.astype(np.int64) - b.astype(np.int64))


def test_tree_dtype_validated():
    from trafficrl.rl.replay import DeviceReplay
    with pytest.raises(ValueError):
        DeviceReplay(8, 1, 1, device="cpu", tree_dtype="float16")


@pytest.mark.gpu
def test_device_tree_matches_reference_fixture(fx):
    cap = int(fx["capacity"])
    rb = _device_replay(cap, fx)
    for B in ADD_BATCHES:
        _adds(rb, B)
    np.testing.assert_array_equal(rb.tree.cpu().numpy(), fx["tree_after_add"])
    for r in range(3):
        u = torch.tensor(fx[f"s{r}_u"], dtype=torch.float64, device="cuda")
        s = rb.sample(256, u=u)
        np.testing.assert_array_equal(s.idx.cpu().numpy(), fx[f"s{r}_idx"])
        assert _ulps32(s.weights.cpu().numpy(), fx[f"s{r}_w"]).max() <= 4
        td = torch.tensor(fx[f"s{r}_td"], dtype=torch.float32, device="cuda")   # the trainer's float32 TD errors
        rb.update_priorities(s.idx, td)
        np.testing.assert_array_equal(rb.tree.cpu().numpy(), fx[f"s{r}_tree"])
        assert rb.max_priority.item() == float(fx[f"s{r}_max_p"])
    _adds(rb, 300)
    np.testing.assert_array_equal(rb.tree.cpu().numpy(), fx["tree_final"])
    assert (rb.ptr, rb.size, rb.max_priority.item()) == (int(fx["final_ptr"]), int(fx["final_size"]),
                                                         float(fx["final_max_p"]))


@pytest.mark.gpu
def test_device_tree_at_reference_buffer_size():
    """buffer_size 1e6 (configs/*.yaml) with 4096-env ring adds, a 256-draw
    sample and an update whose indices repeat (leaf chains), vs the restatement."""
    cap = 1_000_000
    ref = RefTree(cap)
    rb = _device_replay(cap)
    rng = np.random.default_rng(5)
    for B in (4096, 4096, 1000):
        _adds(rb, B)
        for _ in range(B):
            ref.add()
    np.testing.assert_array_equal(rb.tree.cpu().numpy(), ref.tree)
    for r in range(2):
        u = rng.random(256)
        s = rb.sample(256, u=torch.tensor(u, device="cuda"))
        idx, _, w = ref.sample(u)
        np.testing.assert_array_equal(s.idx.cpu().numpy(), idx)
        assert _ulps32(s.weights.cpu().numpy(), w).max() <= 4
        idx_u = np.concatenate([idx, idx[:40], idx[10:20]])          # repeats: later occurrences see earlier ones
        td = (rng.standard_normal(len(idx_u)) * 3).astype(np.float32)
        rb.update_priorities(torch.tensor(idx_u, device="cuda"), torch.tensor(td, device="cuda"))
        ref.update_priorities(idx_u, td.astype(np.float64))
        np.testing.assert_array_equal(rb.tree.cpu().numpy(), ref.tree)
        assert rb.max_priority.item() == ref.max_p


@pytest.mark.gpu
@pytest.mark.parametrize("beta", [0.4, 1.0, 0.5, 2.0])
@pytest.mark.parametrize("n", [256, 3000])
def test_weighted_sample_matches_descent_and_torch_weights(beta, n):
    """trx_per32_sample_weighted (the sample + weights launch DeviceReplay.sample
    uses) against trx_per32_sample and the weights as torch ops state them
    (probs = pri / total, (size * probs) ** -beta, / max): indices and
    priorities bit-exact, weights within 2 float32 ulps (torch's powf build vs
    ours); n = 3000 takes the multi-pass (n > 1024 lanes) path; beta 1.0 / 0.5 /
    2.0 hit torch's closed-form exponents (-1, -0.5, -2)."""
    from trafficrl import _lib
    cap = 1000
    rb = _device_replay(cap)
    _adds(rb, 700)
    L = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(n)
    u = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
    idx0 = torch.empty(n, dtype=torch.int64, device="cuda")
    pri0 = torch.empty(n, dtype=torch.float32, device="cuda")
    _lib.check(L.trx_per32_sample(_lib.ptr(rb.tree), cap, _lib.ptr(u), n, _lib.ptr(idx0), _lib.ptr(pri0), None),
               "trx_per32_sample")
    idx, pri, w = (torch.empty(n, dtype=t, device="cuda") for t in (torch.int64, torch.float32, torch.float32))
    _lib.check(L.trx_per32_sample_weighted(_lib.ptr(rb.tree), cap, _lib.ptr(u), n, _lib.ptr(rb.size_t), beta,
                                           _lib.ptr(idx), _lib.ptr(pri), _lib.ptr(w), None), "trx_per32_sample_weighted")
    assert torch.equal(idx, idx0) and torch.equal(pri, pri0)
    ref = (rb.size_t.float() * (pri0 / rb.total)) ** (-beta)
    ref = ref / torch.where(ref.max() > 0, ref.max(), torch.ones_like(ref.max()))
    assert _ulps32(w.cpu().numpy(), ref.cpu().numpy()).max() <= 2


@pytest.mark.gpu
def test_overlapped_adds_match_in_order_adds():
    """overlap_adds (the trainer's default: the float32 tree's ring adds on a
    side stream beside the next acting pass) gives the same tree, max priority
    and device fill level as in-order adds, after add-only iterations and after
    a sample + priority update; `total` joins the pending adds itself."""
    cap = 50_000
    rbs = [_device_replay(cap), _device_replay(cap)]
    rbs[1].overlap_adds = True
    rng = np.random.default_rng(11)
    for B in (4096, 4096, 4096):
        for rb in rbs:
            _adds(rb, B)
    totals = [float(rb.total) for rb in rbs]
    assert totals[0] == totals[1]
    rbs[1].sync_adds()
    for a, b in ((rbs[0].tree, rbs[1].tree), (rbs[0].max_priority, rbs[1].max_priority),
                 (rbs[0].size_t, rbs[1].size_t)):
        assert torch.equal(a, b)
    for _ in range(2):
        for rb in rbs:
            _adds(rb, 1000)
        u = torch.tensor(rng.random(256), device="cuda")
        td = torch.tensor((rng.standard_normal(256) * 3).astype(np.float32), device="cuda")
        s = [rb.sample(256, u=u) for rb in rbs]
        assert torch.equal(s[0].idx, s[1].idx) and torch.equal(s[0].weights, s[1].weights)
        for rb, sm in zip(rbs, s):
            rb.update_priorities(sm.idx, td)
    rbs[1].sync_adds()
    torch.cuda.synchronize()
    assert torch.equal(rbs[0].tree, rbs[1].tree) and torch.equal(rbs[0].max_priority, rbs[1].max_priority)
    assert torch.equal(rbs[0].size_t, rbs[1].size_t)

"""Known answers of SURVEY.md §4 (measured by running the reference in the
build container) and the reference's only known-answer style check,
scripts/check_tstt_drop.py:13-46, reproduced as unit tests.

CPU tests pin the C oracle (oracle/trx_oracle.c) to the survey's table; the
GPU test drives the product facade (trafficrl.env.RepairEnv, the HIP path)
through check_tstt_drop's steps.
"""
import numpy as np
import pytest

# fixed_damage_seed=42, damaged_ratio=0.3 (repair_env.py:167-196)
SEED42_DAMAGED = [2, 8, 10, 12, 18, 20, 22, 32, 35, 36, 43, 44, 45, 49, 53, 55, 67, 68, 69, 71, 72, 74]


def _damaged_caps(og):
    d = np.zeros(og.E, np.float32)
    d[SEED42_DAMAGED] = 1.0
    cap = np.where(d > 0, np.float32(1e-3), og.cap0).astype(np.float32)   # capacity_damage (repair_env.py:196)
    return d, cap


@pytest.mark.parametrize("method,iters,tstt,rtol", [
    ("msa", 30, 4085.9051802551303, 0.0),     # bit-exact
    ("fw", 30, 4023.7556073211313, 0.0),      # bit-exact
    ("cfw", 60, 4010.759667221298, 1e-6),     # reference np.dot = BLAS sdot, order library-defined (oracle: 4010.7593)
])
def test_reset_tstt_seed42(oracle_graph, method, iters, tstt, rtol):
    """reset() TSTT of the seed-42 damage set (repair_env.py:167-205 -> 299-345)."""
    d, cap = _damaged_caps(oracle_graph)
    _, _, ts, un = oracle_graph.assign(cap, d, np.zeros(oracle_graph.E, np.float32), method=method, iters=iters)
    assert un == 0.0
    if rtol == 0.0:
        assert ts == tstt
    else:
        np.testing.assert_allclose(ts, tstt, rtol=rtol)


@pytest.mark.parametrize("method,iters,sum_ft", [
    ("fw", 1000, 7477941.0),   # the classic Sioux Falls UE ~ 7.48e6: the sanity anchor
    ("msa", 30, 7928867.0),
    ("fw", 30, 7606285.5),
])
def test_undamaged_total_travel_time(oracle_graph, method, iters, sum_ft):
    """Undamaged network: sum(flow * t) against the survey's table (quoted to
    the unit / half unit, so |difference| < 1)."""
    z = np.zeros(oracle_graph.E, np.float32)
    f, t, _, _ = oracle_graph.assign(oracle_graph.cap0, z, z, method=method, iters=iters)
    total = float(np.dot(f.astype(np.float64), t.astype(np.float64)))
    assert abs(total - sum_ft) < 1.0


def test_check_tstt_drop_rule_picks_a_repaired_link(oracle_graph):
    """check_tstt_drop.py:35-38 picks argmax(edge_features[:, 2] * action_mask).
    get_state zeroes the V/C feature of damaged links (repair_env.py:768-773)
    while the action mask is is_damaged (:811), so the product is all zeros and
    the script picks link 0 -- an undamaged link, for which step() returns
    reward -1 with TSTT unchanged (:207-211) and the script raises.  Recorded
    here as the reference's behaviour (a stale script, not a port decision)."""
    d, cap = _damaged_caps(oracle_graph)
    f, _, ts, _ = oracle_graph.assign(cap, d, np.zeros(oracle_graph.E, np.float32), method="msa", iters=30)
    _, ex, mask = oracle_graph.observe(cap, d, d, f, ts)
    assert np.all(ex[0, SEED42_DAMAGED, 2] == 0.0) and np.all(mask[0] == d)
    assert int(np.argmax(ex[0, :, 2] * mask[0])) == 0 and d[0] == 0.0


def test_tstt_drops_after_repairing_max_vc_link(oracle_graph):
    """The check's intent: repair the damaged link with the largest raw V/C
    (flow / max(cap, 1e-6), repair_env.py:770) and TSTT must move by > 1e-6."""
    d, cap = _damaged_caps(oracle_graph)
    f, _, ts0, _ = oracle_graph.assign(cap, d, np.zeros(oracle_graph.E, np.float32), method="msa", iters=30)
    raw_vc = f / np.maximum(cap, np.float32(1e-6))
    a = int(np.argmax(np.where(d > 0, raw_vc, -1.0)))
    assert d[a] == 1.0
    cap2, d2 = cap.copy(), d.copy()
    cap2[a], d2[a] = oracle_graph.cap0[a], 0.0
    _, _, ts1, _ = oracle_graph.assign(cap2, d2, f, method="msa", iters=30)
    assert abs(ts0 - ts1) >= 1e-6 and ts1 < ts0


@pytest.mark.gpu
def test_check_tstt_drop_on_device():
    """scripts/check_tstt_drop.py through the HIP facade (configs/sioux_falls.yaml:
    damaged_ratio 0.3, assignment_iters 30, msa; fixed damage seed 42): the
    script's own rule is a no-op repair (reward -1, TSTT unchanged); the
    max-raw-V/C damaged link lowers TSTT, to the oracle's value bit for bit."""
    import oracle as O
    from conftest import golden
    from trafficrl.data import sioux_falls
    from trafficrl.env import RepairEnv

    env = RepairEnv(sioux_falls(), damaged_ratio=0.3, assignment_iters=30, assignment_method="msa",
                    fixed_damage=True, fixed_damage_seed=42, seed=42)
    state = env.reset(damaged_ratio=0.3)
    assert sorted(np.nonzero(np.asarray(env.is_damaged))[0].tolist()) == SEED42_DAMAGED
    assert env.tstt == 4085.9051802551303
    ef, mask = np.asarray(state.edge_features), np.asarray(state.action_mask)
    a = int(np.argmax(ef[:, 2] * mask))
    t0 = env.tstt
    _, r, done, info = env.step(a)
    assert a == 0 and r == -1.0 and not done and info["tstt"] == t0
    og = O.OracleGraph.from_npz(golden("sf_graph.npz"))
    d, cap = _damaged_caps(og)
    f, _, ts0, _ = og.assign(cap, d, np.zeros(og.E, np.float32), method="msa", iters=30)
    raw_vc = f / np.maximum(cap, np.float32(1e-6))
    b = int(np.argmax(np.where(d > 0, raw_vc, -1.0)))
    _, _, _, info = env.step(b)
    cap[b], d[b] = og.cap0[b], 0.0
    _, _, ts1, _ = og.assign(cap, d, f, method="msa", iters=30)
    assert info["tstt"] == ts1 and abs(info["tstt"] - t0) >= 1e-6

"""The CPU oracle (oracle/trx_oracle.c) pinned against the reference's own
outputs (tests/golden/*, written by tools/gen_golden.py from
/root/reference/src/env/repair_env.py run read-only).

'crpow' fixtures: reference with the host-independent BPR power -> must be
bit-exact.  'native' fixtures: reference as run on the AVX-512 host (numpy
SVML powf, 1-ulp jitter in t) -> flows bit-exact where the SPT is stable,
TSTT within 1e-6 relative.  CFW: reference np.dot is BLAS sdot (order
library-defined) -> tolerance only.
"""
import json

import numpy as np
import pytest

import oracle as O
from conftest import golden

KEYS = ["msa30", "fw30", "msa60", "fw50", "msa1", "fw2"]


def split_key(k):
    m = k.rstrip("0123456789")
    return m, int(k[len(m):])


def caps_for(gr, dmg):
    return np.where(dmg > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)


def test_graph_arrays(sf_graph_npz, oracle_graph):
    assert oracle_graph.N == 24 and oracle_graph.E == 76
    assert len(sf_graph_npz["od_v"]) == 528
    assert oracle_graph.total_demand == 360600.0


def test_scipy_predecessors_with_ties(oracle_graph):
    """Fibonacci-heap restatement reproduces scipy's predecessor choice,
    including the tied OD rows at t = t0 (SURVEY §7 hard part 1)."""
    z = np.load(golden("sf_scipy_pred.npz"))
    assert z["tie"].sum() > 100  # the fixture really exercises ties
    for i in range(len(z["seeds"])):
        d, p = oracle_graph.all_pairs(z["t"][i])
        np.testing.assert_array_equal(d, z["dist"][i])
        np.testing.assert_array_equal(p, z["pred"][i])


def test_pairwise_sum_matches_numpy():
    rng = np.random.default_rng(3)
    for n in (1, 7, 8, 76, 127, 128, 129, 914):
        a = (rng.random(n) * rng.choice([1.0, 1e3, 1e6], n)).astype(np.float32)
        assert O.pairwise_sum_f32(a) == float(np.sum(a))


@pytest.mark.parametrize("key", KEYS)
def test_reset_seed42_crpow_bitexact(sf_graph_npz, oracle_graph, key):
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    m, k = split_key(key)
    dmg = r[key + "_damaged"]
    f, t, ts, un = oracle_graph.assign(caps_for(sf_graph_npz, dmg), dmg, np.zeros(76, np.float32), method=m, iters=k)
    np.testing.assert_array_equal(f, r[key + "_flow"])
    np.testing.assert_array_equal(t, r[key + "_t"])
    assert ts == float(r[key + "_tstt"])
    assert un == float(r[key + "_unassigned"])


@pytest.mark.parametrize("key", KEYS)
def test_reset_seed42_native_tolerance(sf_graph_npz, oracle_graph, key):
    r = np.load(golden("sf_reset_seed42_native.npz"))
    m, k = split_key(key)
    dmg = r[key + "_damaged"]
    f, t, ts, un = oracle_graph.assign(caps_for(sf_graph_npz, dmg), dmg, np.zeros(76, np.float32), method=m, iters=k)
    np.testing.assert_array_equal(f, r[key + "_flow"])
    # t: 1-ulp SVML powf jitter in the reference
    np.testing.assert_array_max_ulp(t, r[key + "_t"], maxulp=2)
    assert abs(ts - float(r[key + "_tstt"])) <= 1e-6 * float(r[key + "_tstt"])


def test_reset_seed42_cfw_tolerance(sf_graph_npz, oracle_graph):
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    dmg = r["cfw60_damaged"]
    f, t, ts, un = oracle_graph.assign(caps_for(sf_graph_npz, dmg), dmg, np.zeros(76, np.float32), method="cfw", iters=60)
    assert abs(ts - float(r["cfw60_tstt"])) <= 1e-6 * float(r["cfw60_tstt"])
    np.testing.assert_allclose(f, r["cfw60_flow"], rtol=1e-5, atol=0.05)


def test_iteration_trace(sf_graph_npz, oracle_graph):
    z = np.load(golden("sf_trace_seed42_crpow.npz"))
    t = oracle_graph.bpr(np.zeros(76, np.float32), z["capacities"], z["damaged"])
    np.testing.assert_array_equal(t, z["t_init"])
    flow = np.zeros(76, np.float32)
    for it in range(3):
        aux, un = oracle_graph.aon(t)
        np.testing.assert_array_equal(aux, z[f"aux_{it}"])
        assert un == float(z[f"unassigned_{it}"])
        s = 1.0 / (it + 1.0)
        flow = np.float32(1 - s) * flow + np.float32(s) * aux
        np.testing.assert_array_equal(flow, z[f"flow_{it}"])
        t = oracle_graph.bpr(flow, z["capacities"], z["damaged"])
        np.testing.assert_array_equal(t, z[f"t_{it}"])


@pytest.mark.parametrize("variant", ["crpow", "native"])
def test_random_resets_and_steps(sf_graph_npz, oracle_graph, variant):
    """32 RNG damage patterns (many with tied shortest paths at reset),
    reset + 4 steps each (incl. an already-repaired action: reward -1, no
    assignment).  crpow: bit-exact; native: TSTT 1e-6."""
    z = np.load(golden(f"sf_random_resets_{variant}.npz"))
    cap0 = sf_graph_npz["cap0"]
    B = len(z["seeds"])
    dmg = z["damaged"].copy()
    cap = np.where(dmg > 0, np.float32(1e-3), cap0).astype(np.float32)
    flow, t, tstt, un = oracle_graph.assign(cap, dmg, np.zeros((B, 76), np.float32), iters=30, nthreads=4)
    exact = variant == "crpow"
    if exact:
        np.testing.assert_array_equal(flow, z["flow"])
        np.testing.assert_array_equal(tstt, z["tstt"])
    else:
        np.testing.assert_allclose(tstt, z["tstt"], rtol=1e-6)
    init = tstt.copy()
    for j in range(4):
        a = z["step_actions"][:, j]
        prev = tstt.copy()
        valid = dmg[np.arange(B), a] > 0
        dmg[np.arange(B)[valid], a[valid]] = 0.0
        cap[np.arange(B)[valid], a[valid]] = cap0[a[valid]]
        flow, t, tstt2, un = oracle_graph.assign(cap, dmg, flow, iters=30, env_mask=valid.astype(np.uint8), nthreads=4)
        tstt = np.where(valid, tstt2, prev)
        for b in range(B):
            if valid[b]:
                r = O.reward("rel_improve", prev[b], tstt[b], init[b], complete=False, alpha=1.0, beta=0.0,
                             gamma=0.0, clip=2.0)
            else:
                r = -1.0
            if exact:
                assert r == z["step_reward"][b, j]
            else:
                assert abs(r - z["step_reward"][b, j]) <= 1e-4
        if exact:
            np.testing.assert_array_equal(flow, z["step_flow"][:, j])
            np.testing.assert_array_equal(tstt, z["step_tstt"][:, j])
        else:
            np.testing.assert_allclose(tstt, z["step_tstt"][:, j], rtol=1e-6)


def test_summary_greedy_sequences_match_survey():
    s = json.load(open(golden("sf_summary.json")))
    assert s["crpow"]["greedy_msa30_actions"] == [55, 72, 68, 22, 45, 10, 36, 74, 18, 44, 12, 8, 43, 49, 53, 20, 69,
                                                  2, 71, 67, 32, 35]
    assert s["native"]["greedy_fw30_actions"] == s["crpow"]["greedy_fw30_actions"]


# ---------------------------------------------------- large graph (config #5)
def _ana_oracle():
    return O.OracleGraph.from_npz(golden("ana_graph.npz"))


@pytest.mark.parametrize("key,method", [("msa30", "msa"), ("fw30", "fw")])
def test_oracle_anaheim_synth_reset_bitexact(key, method):
    """Oracle == reference on the 416-node synthetic network (fixed damage 42)."""
    og = _ana_oracle()
    r = np.load(golden("ana_resets_crpow.npz"))
    d = r[key + "_damaged"]
    cap = np.where(d > 0, np.float32(1e-3), og.cap0).astype(np.float32)
    f, t, ts, un = og.assign(cap, d, np.zeros(og.E, np.float32), method=method, iters=30)
    np.testing.assert_array_equal(f, r[key + "_flow"])
    np.testing.assert_array_equal(t, r[key + "_t"])
    assert ts == float(r[key + "_tstt"]) and un == float(r[key + "_unassigned"])


def test_oracle_anaheim_synth_steps_bitexact():
    og = _ana_oracle()
    z = np.load(golden("ana_steps_crpow.npz"))
    for i in range(len(z["seeds"])):
        d = z["damaged"][i].copy()
        cap = np.where(d > 0, np.float32(1e-3), og.cap0).astype(np.float32)
        f, _, ts, _ = og.assign(cap, d, np.zeros(og.E, np.float32), iters=30)
        np.testing.assert_array_equal(f, z["flow"][i])
        assert ts == z["tstt"][i]
        for j in range(3):
            a = int(z["actions"][i, j])
            if d[a] == 0:  # already repaired: no assignment (repair_env.py:210-212)
                assert z["step_reward"][i, j] == -1.0
                continue
            d[a] = 0.0
            cap[a] = og.cap0[a]
            f, _, ts, _ = og.assign(cap, d, f, iters=30)
            np.testing.assert_array_equal(f, z["step_flow"][i, j])
            assert ts == z["step_tstt"][i, j]


def test_oracle_anaheim_synth_scipy_preds():
    """Oracle's scipy-heap Dijkstra == scipy's predecessors (38 origins, 6 patterns)."""
    og = _ana_oracle()
    z = np.load(golden("ana_scipy_pred.npz"))
    for k in range(len(z["seeds"])):
        _, p = og.all_pairs(z["t"][k])
        np.testing.assert_array_equal(p[z["origins"]], z["pred"][k])


# ------------------------------------------------ GP path assignment oracle
GP_CASES = {"s1k2i30": (1.0, 2, 30), "s1k3i10": (1.0, 3, 10), "s0k3i10": (0.0, 3, 10), "s05k2i8": (0.5, 2, 8)}


@pytest.mark.parametrize("tag", sorted(GP_CASES))
def test_oracle_gp_reset_and_steps_bitexact(tag, oracle_graph):
    """GP restatement (oracle.gp_assign) == reference on seed-42 resets and on
    4 random-seed reset + 3-step trajectories (path sets carried across steps)."""
    step, keep, iters = GP_CASES[tag]
    og = oracle_graph
    z = np.load(golden("sf_gp_crpow.npz"))
    d = z[f"reset_{tag}_damaged"]
    cap = np.where(d > 0, np.float32(1e-3), og.cap0).astype(np.float32)
    f, t, ts, un = O.gp_assign(og, cap, d, np.zeros(og.E, np.float32), O.GPPaths(), iters, step, keep, reset=True)
    np.testing.assert_array_equal(f, z[f"reset_{tag}_flow"])
    np.testing.assert_array_equal(t, z[f"reset_{tag}_t"])
    assert ts == float(z[f"reset_{tag}_tstt"])
    dm = z[f"steps_{tag}_damaged"]
    for i in range(len(dm)):
        d = dm[i].copy()
        cap = np.where(d > 0, np.float32(1e-3), og.cap0).astype(np.float32)
        st = O.GPPaths()
        f, _, ts, _ = O.gp_assign(og, cap, d, np.zeros(og.E, np.float32), st, iters, step, keep, reset=True)
        np.testing.assert_array_equal(f, z[f"steps_{tag}_flow"][i])
        for j in range(3):
            a = int(z[f"steps_{tag}_actions"][i, j])
            if d[a] == 0:
                assert z[f"steps_{tag}_step_reward"][i, j] == -1.0
                continue
            d[a] = 0.0
            cap[a] = og.cap0[a]
            f, _, ts, _ = O.gp_assign(og, cap, d, f, st, iters, step, keep)
            np.testing.assert_array_equal(f, z[f"steps_{tag}_step_flow"][i, j])
            assert ts == z[f"steps_{tag}_step_tstt"][i, j]

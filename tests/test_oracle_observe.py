"""The oracle's C get_state (oracle/trx_oracle.c orc_observe_batch, the CPU
baseline's observation leg) vs the reference's observations on the greedy
MSA-30 trajectory (tests/golden/sf_greedy_msa30_native.npz): betweenness
bit-exact (networkx Brandes order in float64), log features within the numpy
SVML tolerance used for the device kernel (tests/test_gpu_parity.py)."""
import numpy as np

from conftest import golden


def test_c_observe_vs_reference(oracle_graph, sf_graph_npz):
    z = np.load(golden("sf_greedy_msa30_native.npz"))
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    gr = sf_graph_npz
    dmg = r["msa30_damaged"].copy()
    goal = dmg.copy()
    states = [(dmg.copy(), z["reset_flow"], float(z["initial_tstt"]), z["reset_node_x"], z["reset_edge_x"])]
    for j, a in enumerate(z["actions"]):
        dmg[a] = 0.0
        states.append((dmg.copy(), z["flows"][j], float(z["tstt"][j]), z["node_x"][j], z["edge_x"][j]))
    D = np.array([s[0] for s in states])
    cap = np.where(D > 0, np.float32(1e-3), gr["cap0"]).astype(np.float32)
    G = np.repeat(goal[None], len(states), 0)
    F = np.array([s[1] for s in states], np.float32)
    T = np.array([s[2] for s in states])
    nx_, ex_, m = oracle_graph.observe(cap, D, G, F, T, nthreads=4)
    for k, s in enumerate(states):
        np.testing.assert_array_equal(nx_[k][:, 0], s[3][:, 0])
        np.testing.assert_allclose(nx_[k], s[3], rtol=4e-7, atol=0)
        np.testing.assert_allclose(ex_[k], s[4], rtol=5e-7, atol=1e-7)
        np.testing.assert_array_equal(m[k], s[0])

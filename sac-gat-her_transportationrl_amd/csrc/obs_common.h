// obs_common.h -- per-env and per-link feature math of RepairEnv.get_state
// (src/env/repair_env.py:764-819), shared by the small-graph and large-graph
// observation kernels.  Betweenness (node feature 0) is computed by the
// kernels themselves and handed in as float32 [N].
#pragma once
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

__device__ float pairwise_small(const float* a, int n, int stride) {
    // numpy pairwise_sum for n <= 128 (float32), strided reads
    if (n < 8) {
        float r = 0.0f;
        for (int i = 0; i < n; ++i) r = __fadd_rn(r, a[i * stride]);
        return r;
    }
    float r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j * stride];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], a[(i + j) * stride]);
    float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                          __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
    for (; i < n; ++i) res = __fadd_rn(res, a[i * stride]);
    return res;
}

__device__ float pairwise_any(const float* a, int n) {
    if (n <= 128) return pairwise_small(a, n, 1);
    int n2 = n / 2;
    n2 -= n2 % 8;
    // recursion depth <= log2(E/128)
    return __fadd_rn(pairwise_any(a, n2), pairwise_any(a + n2, n - n2));
}

// One thread per env: bw [N] = normalised-by-networkx betweenness (float32,
// before division by its max); prod = scratch of >= E floats.
// goal / dmg / flow: the env's [E] rows (global memory, or LDS copies staged by the caller).
__device__ void obs_env_features(const DevGraph& g, const trx_state& s, int gb, const float* goal, const float* dmg,
                                 const float* flow, const float* bw, float* prod, float* __restrict__ node_x) {
    const int N = g.N, E = g.E;
    float bmax = 0.0f;
    for (int v = 0; v < N; ++v) bmax = fmaxf(bmax, bw[v]);
    // remaining goal ratio, avg undamaged flow (np.mean), log10 tstt (772-785)
    for (int e = 0; e < E; ++e) prod[e] = __fmul_rn(goal[e], dmg[e]);
    float rem = pairwise_any(prod, E);
    for (int e = 0; e < E; ++e) prod[e] = goal[e];
    float gtot = pairwise_any(prod, E);
    double remaining_ratio = (double)rem / ((double)gtot > 1.0 ? (double)gtot : 1.0);
    int nund = 0;
    for (int e = 0; e < E; ++e)
        if (dmg[e] == 0.0f) prod[nund++] = flow[e];
    double avg_flow = 0.0;
    if (nund > 0) {
        float sm = pairwise_any(prod, nund);
        avg_flow = (double)(float)((double)sm / (double)nund);
    }
    double denom = g.total_demand / (double)(E > 1 ? E : 1);
    double avg_norm = avg_flow / (denom > 1.0 ? denom : 1.0);
    double ts = s.tstt[gb];
    double log_tstt = log10(ts > 1.0 ? ts : 1.0);
    for (int v = 0; v < N; ++v) {
        float b = bw[v];
        if (bmax > 0.0f) b = __fdiv_rn(b, bmax);
        float* nx = node_x + ((size_t)gb * N + v) * 4;
        nx[0] = b;
        nx[1] = (float)remaining_ratio;
        nx[2] = (float)avg_norm;
        nx[3] = (float)log_tstt;
    }
}

// Link e of env gb: t0_norm, cap_norm, clip(log1p(v/c)), damaged, goal, id/(E-1) (767-770, 796-808)
__device__ void obs_edge_features(const DevGraph& g, const trx_state& s, int gb, int e, float* __restrict__ edge_x,
                                  float* __restrict__ mask) {
    const int E = g.E;
    const double lt0 = log10((double)g.max_t0 + 1.0), lcap = log10((double)g.max_cap + 1.0);
    const float idn = (float)(E - 1 > 1 ? E - 1 : 1);
    size_t gi = (size_t)gb * E + e;
    float cap = s.capacity[gi], fl = s.flow[gi], dm = s.damaged[gi];
    float c6 = cap > 1e-6f ? cap : 1e-6f;
    float raw = __fdiv_rn(fl, c6);
    float vc = dm > 0.0f ? 0.0f : raw;
    vc = log1pf(vc);
    vc = vc < 0.0f ? 0.0f : (vc > 10.0f ? 10.0f : vc);
    float* ex = edge_x + gi * 6;
    ex[0] = (float)((double)log10f(__fadd_rn(g.t0[e], 1.0f)) / lt0);
    ex[1] = (float)((double)log10f(__fadd_rn(cap, 1.0f)) / lcap);
    ex[2] = vc;
    ex[3] = dm;
    ex[4] = s.goal[gi];
    ex[5] = __fdiv_rn((float)e, idn);
    if (mask) mask[gi] = dm;
}

}  // namespace
}  // namespace trx

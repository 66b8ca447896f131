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

// remaining goal ratio, avg undamaged flow (np.mean), log10 tstt (repair_env.py:772-785)
// from the three float32 link sums: rem = sum(goal * damaged), gtot = sum(goal),
// fsum = sum(flow of the nund undamaged links), each in numpy's pairwise order.
__device__ void obs_env_scalars(const DevGraph& g, const trx_state& s, int gb, float rem, float gtot, float fsum,
                                int nund, float* out3) {
    const int E = g.E;
    double remaining_ratio = (double)rem / ((double)gtot > 1.0 ? (double)gtot : 1.0);
    double avg_flow = nund > 0 ? (double)(float)((double)fsum / (double)nund) : 0.0;
    double denom = g.total_demand / (double)(E > 1 ? E : 1);
    double avg_norm = avg_flow / (denom > 1.0 ? denom : 1.0);
    double ts = s.tstt[gb];
    double log_tstt = log10(ts > 1.0 ? ts : 1.0);
    out3[0] = (float)remaining_ratio;
    out3[1] = (float)avg_norm;
    out3[2] = (float)log_tstt;
}

// node v of env gb: betweenness / max betweenness and the three per-env scalars
__device__ void obs_node_features(int N, int gb, int v, float bw, float bmax, const float* sc3,
                                  float* __restrict__ node_x) {
    float b = bw;
    if (bmax > 0.0f) b = __fdiv_rn(b, bmax);
    float* nx = node_x + ((size_t)gb * N + v) * 4;
    nx[0] = b;
    nx[1] = sc3[0];
    nx[2] = sc3[1];
    nx[3] = sc3[2];
}

// One thread per env: bw [N] = normalised-by-networkx betweenness (float32,
// before division by its max); prod = scratch of >= E floats.
// goal / dmg / flow: the env's [E] rows (global memory, or LDS copies staged by the caller).
__device__ void obs_env_features(const DevGraph& g, const trx_state& s, int gb, const float* goal, const float* dmg,
                                 const float* flow, const float* bw, float* prod, float* __restrict__ node_x) {
    const int N = g.N, E = g.E;
    float bmax = 0.0f;
    for (int v = 0; v < N; ++v) bmax = fmaxf(bmax, bw[v]);
    for (int e = 0; e < E; ++e) prod[e] = __fmul_rn(goal[e], dmg[e]);
    float rem = pairwise_any(prod, E);
    for (int e = 0; e < E; ++e) prod[e] = goal[e];
    float gtot = pairwise_any(prod, E);
    int nund = 0;
    for (int e = 0; e < E; ++e)
        if (dmg[e] == 0.0f) prod[nund++] = flow[e];
    float fsum = nund > 0 ? pairwise_any(prod, nund) : 0.0f;
    float sc3[3];
    obs_env_scalars(g, s, gb, rem, gtot, fsum, nund, sc3);
    for (int v = 0; v < N; ++v) obs_node_features(N, gb, v, bw[v], bmax, sc3, node_x);
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

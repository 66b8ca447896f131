// observe_kernel.hip -- RepairEnv.get_state (src/env/repair_env.py:751-819) for
// B envs on gfx950.
//
// Node feature 0 is networkx's betweenness_centrality(G.edge_subgraph(active),
// normalized=True) (networkx 3.4 betweenness.py: _single_source_shortest_path_basic,
// _accumulate_basic, _rescale), reproduced in its own order of float64
// operations: BFS queue order = networkx adjacency (edge file) order, the
// dependency sweep pops the queue in reverse, per-source contributions are
// summed over sources in networkx node order.  One lane per (env, source);
// per-lane BFS state lives node-major in LDS ([node][lane], conflict-free).
#include <hip/hip_runtime.h>

#include "obs_common.h"
#include "trx_internal.h"

namespace trx {

namespace {

constexpr int kObsThreads = 64;

}  // namespace

__global__ void __launch_bounds__(kObsThreads) observe_kernel(const DevGraph g, const trx_state s, int B, int EPW,
                                                              float* __restrict__ node_x, float* __restrict__ edge_x,
                                                              float* __restrict__ mask) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int N = g.N, E = g.E;
    const int L = kObsThreads;
    const int tid = threadIdx.x;
    const int env0 = blockIdx.x * EPW;
    // LDS: sigma[N][L] f64, delta[N][L] f64, dist[N][L] i16, queue[N][L] u8, dmg[EPW][E] f32, insub[EPW][N] u8
    double* sigma = reinterpret_cast<double*>(smem_raw);
    double* delta = sigma + (size_t)N * L;
    int16_t* dist = reinterpret_cast<int16_t*>(delta + (size_t)N * L);
    uint8_t* queue = reinterpret_cast<uint8_t*>(dist + (size_t)N * L);
    float* dmg = reinterpret_cast<float*>(queue + (((size_t)N * L + 15) & ~size_t(15)));
    uint8_t* insub = reinterpret_cast<uint8_t*>(dmg + (size_t)EPW * E);
    int* nsub = reinterpret_cast<int*>(insub + (((size_t)EPW * N + 15) & ~size_t(15)));
    float* goal_l = reinterpret_cast<float*>(nsub + 16);  // [EPW][E] staged for the per-env features
    float* flow_l = goal_l + (size_t)EPW * E;             // [EPW][E]
    // the graph's adjacency (read in every BFS step) staged as int16
    int16_t* gop = reinterpret_cast<int16_t*>(flow_l + (size_t)EPW * E);  // out_ptr [N+1]
    int16_t* gip = gop + (N + 1);                                          // in_ptr  [N+1]
    int16_t* goe = gip + (N + 1);                                          // out_eid [E]
    int16_t* god = goe + E;                                                // out_dst [E]
    int16_t* gie = god + E;                                                // in_eid  [E]
    int16_t* gis = gie + E;                                                // in_src  [E]
    int16_t* gnx = gis + E;                                                // nx_order [N]
    for (int i = tid; i <= N; i += L) {
        gop[i] = (int16_t)g.out_ptr[i];
        gip[i] = (int16_t)g.in_ptr[i];
    }
    for (int i = tid; i < E; i += L) {
        goe[i] = (int16_t)g.out_eid[i];
        god[i] = (int16_t)g.out_dst[i];
        gie[i] = (int16_t)g.in_eid[i];
        gis[i] = (int16_t)g.in_src[i];
    }
    for (int i = tid; i < N; i += L) gnx[i] = (int16_t)g.nx_order[i];

    for (int i = tid; i < EPW * E; i += L) {
        int el = i / E, gb = env0 + el;
        const size_t gi = (size_t)gb * E + (i - el * E);
        dmg[i] = gb < B ? s.damaged[gi] : 1.0f;
        goal_l[i] = gb < B ? s.goal[gi] : 0.0f;
        flow_l[i] = gb < B ? s.flow[gi] : 0.0f;
    }
    __syncthreads();
    for (int i = tid; i < EPW * N; i += L) {
        int el = i / N, v = i - el * N;
        int in = 0;
        for (int j = gop[v]; j < gop[v + 1] && !in; ++j) in = dmg[el * E + goe[j]] == 0.0f;
        for (int j = gip[v]; j < gip[v + 1] && !in; ++j) in = dmg[el * E + gie[j]] == 0.0f;
        insub[i] = (uint8_t)in;
    }
    __syncthreads();
    if (tid < EPW) {
        int c = 0;
        for (int v = 0; v < N; ++v) c += insub[tid * N + v];
        nsub[tid] = c;
    }

    // ---------------- Brandes from source = nx_order[j] for lane (env, j)
    const int lenv = tid / N, j = tid - lenv * N;
    const bool on = lenv < EPW && env0 + lenv < B;
    const int src = on ? gnx[j] : 0;
    const bool active_src = on && insub[lenv * N + src];
    if (on) {
        for (int v = 0; v < N; ++v) {
            sigma[v * L + tid] = 0.0;
            delta[v * L + tid] = 0.0;
            dist[v * L + tid] = -1;
        }
    }
    if (active_src) {
        const float* dm = dmg + lenv * E;
        sigma[src * L + tid] = 1.0;
        dist[src * L + tid] = 0;
        int qh = 0, qt = 0;
        queue[qt++ * L + tid] = (uint8_t)src;
        while (qh < qt) {
            int v = queue[qh++ * L + tid];
            int dv = dist[v * L + tid];
            double sv = sigma[v * L + tid];
            for (int k = gop[v]; k < gop[v + 1]; ++k) {
                if (dm[goe[k]] != 0.0f) continue;  // only active edges are in the subgraph
                int w = god[k];
                int dw = dist[w * L + tid];
                if (dw < 0) {
                    queue[qt++ * L + tid] = (uint8_t)w;
                    dist[w * L + tid] = (int16_t)(dv + 1);
                    dw = dv + 1;
                }
                if (dw == dv + 1) sigma[w * L + tid] += sv;
            }
        }
        // _accumulate_basic: pop in reverse BFS order
        for (int q = qt - 1; q >= 0; --q) {
            int w = queue[q * L + tid];
            double coeff = (1.0 + delta[w * L + tid]) / sigma[w * L + tid];
            int dw = dist[w * L + tid];
            for (int k = gip[w]; k < gip[w + 1]; ++k) {
                if (dm[gie[k]] != 0.0f) continue;
                int v = gis[k];
                if (dist[v * L + tid] >= 0 && dist[v * L + tid] == dw - 1)
                    delta[v * L + tid] += sigma[v * L + tid] * coeff;
            }
        }
    }
    __syncthreads();

    // ---------------- per (env, node): betweenness, then per-env features
    // betweenness[w] = sum over sources s (nx order, s != w, w reached) of delta_s[w]
    float* bwv = reinterpret_cast<float*>(sigma);  // reuse after the barrier below
    float bw_local[2] = {0.f, 0.f};
    int nloc = 0;
    for (int i = tid; i < EPW * N; i += L) {
        int el = i / N, w = i - el * N;
        double bc = 0.0;
        if (env0 + el < B && insub[i]) {
            for (int jj = 0; jj < N; ++jj) {
                int s_ = gnx[jj];
                int lane = el * N + jj;
                if (s_ == w || !insub[el * N + s_]) continue;
                if (dist[w * L + lane] < 0) continue;
                bc += delta[w * L + lane];
            }
            int n = nsub[el];
            if (n > 2) {
                double scale = 1.0 / ((double)(n - 1) * (double)(n - 2));
                bc *= scale;
            }
        }
        if (nloc < 2) bw_local[nloc++] = (float)bc;
    }
    __syncthreads();
    nloc = 0;
    for (int i = tid; i < EPW * N; i += L) {
        if (nloc < 2) bwv[i] = bw_local[nloc++];
    }
    __syncthreads();

    if (tid < EPW && env0 + tid < B) {
        // feature scratch reuses delta (>= E + 8 floats per env, checked at launch)
        obs_env_features(g, s, env0 + tid, goal_l + tid * E, dmg + tid * E, flow_l + tid * E, bwv + tid * N,
                         reinterpret_cast<float*>(delta) + tid * (E + 8), node_x);
    }
    for (int i = tid; i < EPW * E; i += L) {
        int el = i / E, e = i - el * E, gb = env0 + el;
        if (gb < B) obs_edge_features(g, s, gb, e, edge_x, mask);
    }
}

static size_t observe_smem(const DevGraph& g, int epw) {
    size_t n = (size_t)g.N * kObsThreads;
    size_t b = n * 8 * 2 + n * 2 + ((n + 15) & ~size_t(15));
    b += (size_t)epw * g.E * 4;
    b += (((size_t)epw * g.N + 15) & ~size_t(15)) + 16 * 4;
    b += (size_t)epw * g.E * 4 * 2;  // goal / flow staged for the per-env features
    b += ((size_t)2 * (g.N + 1) + 4 * (size_t)g.E + g.N) * 2 + 16;  // int16 adjacency
    // the feature scratch reuses delta: needs epw*(E+8) floats <= N*L doubles
    return b;
}

hipError_t launch_observe_kernel(const DevGraph& g, int B, const trx_state& s, float* node_x, float* edge_x,
                                 float* mask, hipStream_t stream) {
    int epw = kObsThreads / g.N;
    if (epw < 1) return hipErrorInvalidValue;
    if ((size_t)epw * (g.E + 8) > (size_t)g.N * kObsThreads * 2) return hipErrorInvalidValue;
    if (epw * g.N > 2 * kObsThreads) return hipErrorInvalidValue;  // bw_local holds 2 entries per thread
    int blocks = (B + epw - 1) / epw;
    hipLaunchKernelGGL(observe_kernel, dim3(blocks), dim3(kObsThreads), observe_smem(g, epw), stream, g, s, B, epw,
                       node_x, edge_x, mask);
    return hipGetLastError();
}

}  // namespace trx

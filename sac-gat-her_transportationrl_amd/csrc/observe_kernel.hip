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

#include "trx_internal.h"

namespace trx {

namespace {

constexpr int kObsThreads = 64;

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
    // depth is tiny for small graphs; recursion depth <= log2(E/128)
    return __fadd_rn(pairwise_any(a, n2), pairwise_any(a + n2, n - n2));
}

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

    for (int i = tid; i < EPW * E; i += L) {
        int el = i / E, gb = env0 + el;
        dmg[i] = gb < B ? s.damaged[(size_t)gb * E + (i - el * E)] : 1.0f;
    }
    __syncthreads();
    for (int i = tid; i < EPW * N; i += L) {
        int el = i / N, v = i - el * N;
        int in = 0;
        for (int j = g.out_ptr[v]; j < g.out_ptr[v + 1] && !in; ++j) in = dmg[el * E + g.out_eid[j]] == 0.0f;
        for (int j = g.in_ptr[v]; j < g.in_ptr[v + 1] && !in; ++j) in = dmg[el * E + g.in_eid[j]] == 0.0f;
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
    const int src = on ? g.nx_order[j] : 0;
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
            for (int k = g.out_ptr[v]; k < g.out_ptr[v + 1]; ++k) {
                if (dm[g.out_eid[k]] != 0.0f) continue;  // only active edges are in the subgraph
                int w = g.out_dst[k];
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
            for (int k = g.in_ptr[w]; k < g.in_ptr[w + 1]; ++k) {
                if (dm[g.in_eid[k]] != 0.0f) continue;
                int v = g.in_src[k];
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
                int s_ = g.nx_order[jj];
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
        const int el = tid, gb = env0 + tid;
        const size_t eb = (size_t)gb * E;
        float bmax = 0.0f;
        for (int v = 0; v < N; ++v) bmax = fmaxf(bmax, bwv[el * N + v]);
        // remaining goal ratio, avg undamaged flow (np.mean), log10 tstt
        float* prod = reinterpret_cast<float*>(delta) + el * (E + 8);  // scratch
        for (int e = 0; e < E; ++e) prod[e] = __fmul_rn(s.goal[eb + e], s.damaged[eb + e]);
        float rem = pairwise_any(prod, E);
        for (int e = 0; e < E; ++e) prod[e] = s.goal[eb + e];
        float gtot = pairwise_any(prod, E);
        double remaining_ratio = (double)rem / ((double)gtot > 1.0 ? (double)gtot : 1.0);
        int nund = 0;
        for (int e = 0; e < E; ++e)
            if (s.damaged[eb + e] == 0.0f) prod[nund++] = s.flow[eb + e];
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
            float b = bwv[el * N + v];
            if (bmax > 0.0f) b = __fdiv_rn(b, bmax);
            float* nx = node_x + ((size_t)gb * N + v) * 4;
            nx[0] = b;
            nx[1] = (float)remaining_ratio;
            nx[2] = (float)avg_norm;
            nx[3] = (float)log_tstt;
        }
    }
    // ---------------- edge features
    const double lt0 = log10((double)g.max_t0 + 1.0), lcap = log10((double)g.max_cap + 1.0);
    const float idn = (float)(E - 1 > 1 ? E - 1 : 1);
    for (int i = tid; i < EPW * E; i += L) {
        int el = i / E, e = i - el * E, gb = env0 + el;
        if (gb >= B) continue;
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
}

static size_t observe_smem(const DevGraph& g, int epw) {
    size_t n = (size_t)g.N * kObsThreads;
    size_t b = n * 8 * 2 + n * 2 + ((n + 15) & ~size_t(15));
    b += (size_t)epw * g.E * 4;
    b += (((size_t)epw * g.N + 15) & ~size_t(15)) + 16 * 4;
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

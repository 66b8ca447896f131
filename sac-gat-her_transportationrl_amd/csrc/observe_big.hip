// observe_big.hip -- RepairEnv.get_state (src/env/repair_env.py:751-819) for
// networks larger than the lane-per-source observation kernel takes (N > 32).
//
// Node feature 0 is networkx's betweenness_centrality(G.edge_subgraph(active),
// normalized=True) (networkx 3.4: _single_source_shortest_path_basic,
// _accumulate_basic, _rescale) in its own order of float64 operations.  One
// workgroup per env; each wave runs one source's Brandes pass at a time as a
// level-synchronous BFS that rebuilds networkx's exact queue order:
//   * a node of level L+1 is appended by the first of its level-L parents in
//     queue order, at that parent's adjacency (file-order) position -- the
//     wave claims each new node with an LDS atomicMin on (parent queue index,
//     adjacency slot) and appends winners with a wave prefix scan;
//   * sigma (exact integer path counts in float64) is pulled from the parents;
//   * the dependency sweep walks levels bottom-up; delta[v] adds its children's
//     sigma[v] * (1 + delta[w]) / sigma[w] in reverse queue order of w, which
//     is the order networkx's stack pops them.
// Sources are taken W at a time (one per wave) in networkx node order and
// their dependencies are added into betweenness in that same order after a
// workgroup barrier, so the float64 sums match networkx bit for bit.
#include <hip/hip_runtime.h>

#include <climits>

#include "obs_common.h"
#include "trx_internal.h"

namespace trx {

namespace {

struct SmemO {
    uint32_t optr, iptr;                // [N+1] i16
    uint32_t odst, isrc;                // [E] i16: head of CSR out-slot / tail of in-slot, -1 when damaged
    uint32_t insub;                     // [N] u8
    uint32_t srcs;                      // [N] i16 active sources in networkx order
    uint32_t misc;                      // [4] i32
    uint32_t bc;                        // [N] f64
    uint32_t bw;                        // [N] f32
    uint32_t sigma, delta;              // [W][N] f64
    uint32_t dist, queue, lvl;          // [W][N] i16 (lvl: [W][N+1])
    uint32_t claim;                     // [W][N] i32 (after the BFS: queue position)
    uint32_t total;
};

__host__ __device__ inline uint32_t a16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline SmemO smemo_layout(int N, int E, int W) {
    SmemO o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t b) {
        uint32_t r = off;
        off = a16(off + b);
        return r;
    };
    o.optr = take((N + 1) * 2);
    o.iptr = take((N + 1) * 2);
    o.odst = take(E * 2);
    o.isrc = take(E * 2);
    o.insub = take(N);
    o.srcs = take(N * 2);
    o.misc = take(16);
    o.bc = take(N * 8);
    o.bw = take(N * 4);
    o.sigma = take(W * N * 8);
    o.delta = take(W * N * 8);
    o.dist = take(W * N * 2);
    o.queue = take(W * N * 2);
    o.lvl = take(W * (N + 1) * 2);
    o.claim = take(W * N * 4);
    o.total = off;
    return o;
}

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_excl_scan(int c, int lane, int& total) {
    int x = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - c;
}

}  // namespace

__global__ void __launch_bounds__(512) observe_big_kernel(const DevGraph g, const trx_state s, int B,
                                                          float* __restrict__ node_x, float* __restrict__ edge_x,
                                                          float* __restrict__ mask) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int N = g.N, E = g.E;
    const int tid = threadIdx.x, L = blockDim.x, W = L / 64, wave = tid >> 6, lane = tid & 63;
    const int gb = blockIdx.x;
    const SmemO O = smemo_layout(N, E, W);
    int16_t* optr = (int16_t*)(smem_raw + O.optr);
    int16_t* iptr = (int16_t*)(smem_raw + O.iptr);
    int16_t* odst = (int16_t*)(smem_raw + O.odst);
    int16_t* isrc = (int16_t*)(smem_raw + O.isrc);
    uint8_t* insub = smem_raw + O.insub;
    int16_t* srcs = (int16_t*)(smem_raw + O.srcs);
    int* misc = (int*)(smem_raw + O.misc);
    double* bc = (double*)(smem_raw + O.bc);
    float* bw = (float*)(smem_raw + O.bw);
    double* sigma_all = (double*)(smem_raw + O.sigma);
    double* delta_all = (double*)(smem_raw + O.delta);
    int16_t* dist_all = (int16_t*)(smem_raw + O.dist);
    double* sigma = sigma_all + (size_t)wave * N;
    double* delta = delta_all + (size_t)wave * N;
    int16_t* dist = dist_all + (size_t)wave * N;
    int16_t* queue = (int16_t*)(smem_raw + O.queue) + (size_t)wave * N;
    int16_t* lvl = (int16_t*)(smem_raw + O.lvl) + (size_t)wave * (N + 1);
    int* claim = (int*)(smem_raw + O.claim) + (size_t)wave * N;

    // damaged links folded into the CSR slot tables: every adjacency step below
    // is one LDS read instead of two dependent ones
    const float* dm = s.damaged + (size_t)gb * E;
    for (int k = tid; k < E; k += L) {
        odst[k] = dm[g.out_eid[k]] == 0.0f ? (int16_t)g.out_dst[k] : (int16_t)-1;
        isrc[k] = dm[g.in_eid[k]] == 0.0f ? (int16_t)g.in_src[k] : (int16_t)-1;
    }
    for (int v = tid; v <= N; v += L) {
        optr[v] = (int16_t)g.out_ptr[v];
        iptr[v] = (int16_t)g.in_ptr[v];
    }
    for (int v = tid; v < N; v += L) bc[v] = 0.0;
    __syncthreads();
    // edge_subgraph(active): nodes incident to an active link
    for (int v = tid; v < N; v += L) {
        int in = 0;
        for (int k = optr[v]; k < optr[v + 1] && !in; ++k) in = odst[k] >= 0;
        for (int k = iptr[v]; k < iptr[v + 1] && !in; ++k) in = isrc[k] >= 0;
        insub[v] = (uint8_t)in;
    }
    __syncthreads();
    if (tid == 0) {
        int n = 0;
        for (int j = 0; j < N; ++j) {
            int v = g.nx_order[j];
            if (insub[v]) srcs[n++] = (int16_t)v;
        }
        misc[0] = n;
    }
    __syncthreads();
    const int nsrc = misc[0];

    for (int c0 = 0; c0 < nsrc; c0 += W) {
        if (c0 + wave < nsrc) {  // wave-uniform
            const int src = srcs[c0 + wave];
            for (int v = lane; v < N; v += 64) {
                dist[v] = -1;
                sigma[v] = 0.0;
                delta[v] = 0.0;
                claim[v] = INT_MAX;
            }
            wsync();
            if (lane == 0) {
                dist[src] = 0;
                sigma[src] = 1.0;
                queue[0] = (int16_t)src;
            }
            wsync();
            // ------------- BFS in networkx queue order (_single_source_shortest_path_basic)
            int ls = 0, le = 1, lev = 0;
            while (ls < le) {
                if (lane == 0) lvl[lev] = (int16_t)ls;
                for (int base = ls; base < le; base += 64) {
                    const int i = base + lane;
                    if (i < le) {
                        const int v = queue[i], k0 = optr[v];
                        for (int k = k0, k1 = optr[v + 1]; k < k1; ++k) {
                            const int w = odst[k];
                            if (w >= 0 && dist[w] < 0) atomicMin(&claim[w], i * 64 + (k - k0));
                        }
                    }
                }
                wsync();
                int added = 0;
                for (int base = ls; base < le; base += 64) {
                    const int i = base + lane;
                    int c = 0, v = 0, k0 = 0, k1 = 0;
                    if (i < le) {
                        v = queue[i];
                        k0 = optr[v];
                        k1 = optr[v + 1];
                        for (int k = k0; k < k1; ++k) {
                            const int w = odst[k];
                            if (w >= 0 && claim[w] == i * 64 + (k - k0)) ++c;
                        }
                    }
                    int tot;
                    int pos = le + added + wave_excl_scan(c, lane, tot);
                    if (i < le)
                        for (int k = k0; k < k1; ++k) {
                            const int w = odst[k];
                            if (w >= 0 && claim[w] == i * 64 + (k - k0)) queue[pos++] = (int16_t)w;
                        }
                    added += tot;
                }
                wsync();
                for (int q = le + lane; q < le + added; q += 64) {
                    const int w = queue[q];
                    claim[w] = INT_MAX;
                    dist[w] = (int16_t)(lev + 1);
                }
                wsync();
                for (int q = le + lane; q < le + added; q += 64) {  // sigma[w] = sum of parents' sigma (exact)
                    const int w = queue[q];
                    double sg = 0.0;
                    for (int k = iptr[w], k1 = iptr[w + 1]; k < k1; ++k) {
                        const int v = isrc[k];
                        if (v >= 0 && dist[v] == lev) sg += sigma[v];
                    }
                    sigma[w] = sg;
                }
                wsync();
                ls = le;
                le += added;
                ++lev;
            }
            if (lane == 0) lvl[lev] = (int16_t)le;
            for (int q = lane; q < le; q += 64) claim[queue[q]] = q;  // queue position
            wsync();
            // ------------- dependencies (_accumulate_basic), deepest level first
            for (int lv = lev - 2; lv >= 0; --lv) {
                for (int q = lvl[lv] + lane; q < lvl[lv + 1]; q += 64) {
                    const int v = queue[q];
                    const double sv = sigma[v];
                    double dv = 0.0;
                    int prev = INT_MAX;
                    for (;;) {  // children in reverse queue order (networkx's stack pops)
                        int bp = -1, bwn = -1;
                        for (int k = optr[v], k1 = optr[v + 1]; k < k1; ++k) {
                            const int w = odst[k];
                            if (w < 0 || dist[w] != lv + 1) continue;
                            const int p = claim[w];
                            if (p < prev && p > bp) {
                                bp = p;
                                bwn = w;
                            }
                        }
                        if (bp < 0) break;
                        const double coeff = __ddiv_rn(__dadd_rn(1.0, delta[bwn]), sigma[bwn]);
                        dv = __dadd_rn(dv, __dmul_rn(sv, coeff));
                        prev = bp;
                    }
                    delta[v] = dv;
                }
                wsync();
            }
        }
        __syncthreads();
        // betweenness[w] += delta_s[w] for the W sources of this chunk, in order
        for (int v = tid; v < N; v += L) {
            double b = bc[v];
            for (int j = 0; j < W && c0 + j < nsrc; ++j) {
                if (v == srcs[c0 + j] || dist_all[(size_t)j * N + v] < 0) continue;
                b = __dadd_rn(b, delta_all[(size_t)j * N + v]);
            }
            bc[v] = b;
        }
        __syncthreads();
    }
    // _rescale (normalized, directed): scale = 1 / ((n - 1) (n - 2))
    const int n = nsrc;
    for (int v = tid; v < N; v += L) {
        double b = bc[v];
        if (n > 2) b = __dmul_rn(b, 1.0 / ((double)(n - 1) * (double)(n - 2)));
        bw[v] = (float)b;
    }
    __syncthreads();
    if (tid == 0)
        obs_env_features(g, s, gb, s.goal + (size_t)gb * g.E, s.damaged + (size_t)gb * g.E, s.flow + (size_t)gb * g.E, bw,
                         reinterpret_cast<float*>(sigma_all), node_x);
    for (int e = tid; e < E; e += L) obs_edge_features(g, s, gb, e, edge_x, mask);
}

// waves per workgroup (one source per wave): the most resident waves per CU
// under the 160 KB LDS, ties to the wider workgroup (fewer source rounds per env)
static int observe_big_waves(const DevGraph& g) {
    int best = 0, best_res = 0;
    for (int w = 1; w <= 8; ++w) {
        const uint32_t t = smemo_layout(g.N, g.E, w).total;
        if (t > 160u * 1024u) break;
        const int res = w * (int)((160u * 1024u) / t);
        if (res >= best_res) best = w, best_res = res;
    }
    return best;
}

hipError_t launch_observe_big(const DevGraph& g, int B, const trx_state& s, float* node_x, float* edge_x, float* mask,
                              hipStream_t stream) {
    const int w = observe_big_waves(g);
    if (w == 0) return hipErrorInvalidConfiguration;
    // the per-env feature scratch reuses the sigma rows: needs E floats
    if ((size_t)w * g.N * 8 < (size_t)g.E * 4) return hipErrorInvalidConfiguration;
    if (B == 0) return hipSuccess;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(observe_big_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(observe_big_kernel, dim3(B), dim3(w * 64), smemo_layout(g.N, g.E, w).total, stream, g, s, B,
                       node_x, edge_x, mask);
    return hipGetLastError();
}

}  // namespace trx

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
// Damaged links are folded into per-env CSR slot tables (head / tail, -1 when
// damaged) so a BFS edge step is one LDS read, not two dependent ones.
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
    // LDS (sized so that 8 blocks of a 24-node graph share one CU):
    //   delta[N][L] f64, bfs[N][L] u32 packing a lane's dist (byte 0, 0xff = unreached),
    //   queue entry (byte 1) and sigma (bytes 2-3) -- one dword per (row, lane), so the
    //   byte / half-word accesses of a wave never share a bank (separate u8 / u16
    //   arrays put four / two lanes' entries in one dword: 1.1 conflicts per access),
    //   odst[EPW][E] i8 (head of CSR out-slot k, -1 when that link is damaged),
    //   isrc[EPW][E] i8 (tail of CSR in-slot k, -1 when damaged), insub[EPW][N] u8, nsub[16] i32,
    //   out_ptr / in_ptr [N+1] and nx_order [N] as int16.
    // (Keeping the BFS levels as node bit masks in registers instead of dist[]
    // measured 11% slower: 87 vs 78 us at B=4096.)
    // sigma counts shortest paths: every one of them takes one node from each BFS
    // level strictly between source and target, so sigma <= prod(level sizes) with
    // sum(level sizes) <= N-2, i.e. <= 3^10 = 59049 for N <= 32 -- exact in u16 and,
    // converted, the same float64 value networkx's float sigma holds.
    double* delta = reinterpret_cast<double*>(smem_raw);
    uint32_t* bfs = reinterpret_cast<uint32_t*>(delta + (size_t)N * L);
    uint8_t* const bfs8 = reinterpret_cast<uint8_t*>(bfs);
    uint16_t* const bfs16 = reinterpret_cast<uint16_t*>(bfs);
    auto dist = [&](int v, int ln) -> uint8_t& { return bfs8[4 * (v * L + ln)]; };
    auto queue = [&](int q) -> uint8_t& { return bfs8[4 * (q * L + tid) + 1]; };
    auto sigma = [&](int v) -> uint16_t& { return bfs16[2 * (v * L + tid) + 1]; };
    int8_t* odst = reinterpret_cast<int8_t*>(bfs + (size_t)N * L);
    int8_t* isrc = odst + (size_t)EPW * E;
    uint8_t* insub = reinterpret_cast<uint8_t*>(isrc + (size_t)EPW * E);
    int* nsub = reinterpret_cast<int*>(smem_raw + (((size_t)N * L * 12 + 2 * (size_t)EPW * E + EPW * N + 15) & ~size_t(15)));
    int16_t* gop = reinterpret_cast<int16_t*>(nsub + 16);  // out_ptr [N+1]
    int16_t* gip = gop + (N + 1);                          // in_ptr  [N+1]
    int16_t* gnx = gip + (N + 1);                          // nx_order [N]
    for (int i = tid; i <= N; i += L) {
        gop[i] = (int16_t)g.out_ptr[i];
        gip[i] = (int16_t)g.in_ptr[i];
    }
    for (int i = tid; i < N; i += L) gnx[i] = (int16_t)g.nx_order[i];
    // the envs' damaged flags staged first (coalesced, in link order), then the CSR slot
    // tables from LDS: no slot -> link -> flag chain of dependent global loads.  delta is
    // free until the Brandes initialisation below.
    uint8_t* dmg = reinterpret_cast<uint8_t*>(delta);  // [EPW][E], 1 = damaged or no env
    for (int i = tid; i < EPW * E; i += L) {
        const int el = i / E, k = i - el * E, gb = env0 + el;
        dmg[i] = gb < B ? (uint8_t)(s.damaged[(size_t)gb * E + k] != 0.0f) : (uint8_t)1;
    }
    __syncthreads();
    for (int i = tid; i < EPW * E; i += L) {
        const int el = i / E, k = i - el * E;
        odst[i] = dmg[el * E + g.out_eid[k]] ? (int8_t)-1 : (int8_t)g.out_dst[k];
        isrc[i] = dmg[el * E + g.in_eid[k]] ? (int8_t)-1 : (int8_t)g.in_src[k];
    }
    __syncthreads();
    for (int i = tid; i < EPW * N; i += L) {
        int el = i / N, v = i - el * N;
        int in = 0;
        for (int k = gop[v]; k < gop[v + 1] && !in; ++k) in = odst[el * E + k] >= 0;
        for (int k = gip[v]; k < gip[v + 1] && !in; ++k) in = isrc[el * E + k] >= 0;
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
            bfs[v * L + tid] = 0xffu;   // dist unreached, sigma 0
            delta[v * L + tid] = 0.0;
        }
    }
    if (active_src) {
        const int8_t* od = odst + lenv * E;
        const int8_t* is = isrc + lenv * E;
        sigma(src) = 1;
        dist(src, tid) = 0;
        int qh = 0, qt = 0;
        queue(qt++) = (uint8_t)src;
        while (qh < qt) {
            int v = queue(qh++);
            int dv1 = dist(v, tid) + 1;
            uint16_t sv = sigma(v);
            for (int k = gop[v], ke = gop[v + 1]; k < ke; ++k) {
                int w = od[k];
                if (w < 0) continue;  // only active links are in the subgraph
                int dw = dist(w, tid);
                if (dw == 0xff) {
                    queue(qt++) = (uint8_t)w;
                    dist(w, tid) = (uint8_t)dv1;
                    dw = dv1;
                }
                if (dw == dv1) sigma(w) += sv;
            }
        }
        // _accumulate_basic: pop in reverse BFS order
        for (int q = qt - 1; q >= 0; --q) {
            int w = queue(q);
            double coeff = (1.0 + delta[w * L + tid]) / (double)sigma(w);
            int dw1 = dist(w, tid) - 1;
            for (int k = gip[w], ke = gip[w + 1]; k < ke; ++k) {
                int v = is[k];
                if (v < 0) continue;
                if (dist(v, tid) == dw1) delta[v * L + tid] += (double)sigma(v) * coeff;
            }
        }
    }
    __syncthreads();

    // ---------------- per (env, node): betweenness, then per-env features
    // betweenness[w] = sum over sources s (nx order, s != w, w reached) of delta_s[w]
    float* bwv = reinterpret_cast<float*>(bfs);  // reuse after the barrier below
    float bw0 = 0.f, bw1 = 0.f;  // this thread's (at most 2) nodes, kept out of scratch
    int nloc = 0;
    for (int i = tid; i < EPW * N; i += L) {
        int el = i / N, w = i - el * N;
        double bc = 0.0;
        if (env0 + el < B && insub[i]) {
            for (int jj = 0; jj < N; ++jj) {
                int s_ = gnx[jj];
                int lane = el * N + jj;
                if (s_ == w || !insub[el * N + s_]) continue;
                if (dist(w, lane) == 0xff) continue;
                bc += delta[w * L + lane];
            }
            int n = nsub[el];
            if (n > 2) {
                double scale = 1.0 / ((double)(n - 1) * (double)(n - 2));
                bc *= scale;
            }
        }
        if (nloc == 0) bw0 = (float)bc;
        else bw1 = (float)bc;
        ++nloc;
    }
    __syncthreads();
    nloc = 0;
    for (int i = tid; i < EPW * N; i += L) {
        bwv[i] = nloc == 0 ? bw0 : bw1;
        ++nloc;
    }
    __syncthreads();

    if (E > 128) {  // numpy's recursive pairwise split: one thread per env
        if (tid < EPW && env0 + tid < B) {
            const size_t off = (size_t)(env0 + tid) * E;
            obs_env_features(g, s, env0 + tid, s.goal + off, s.damaged + off, s.flow + off, bwv + tid * N,
                             reinterpret_cast<float*>(delta) + tid * (E + 8), node_x);
        }
    } else {
        // The three per-env link sums in numpy's pairwise_sum order for n <= 128
        // (8 running partials r[j] over a[j], a[j+8], ..., a tree over r, then the
        // tail in order), the partials on 8 lanes each.  delta is free here:
        //   cflow[EPW][E] undamaged flows compacted in link order, part[EPW][3][8],
        //   sums[EPW][4] (rem, gtot, fsum, bmax), sc[EPW][3] scalars, nund[EPW].
        float* cflow = reinterpret_cast<float*>(delta);
        float* part = cflow + (size_t)EPW * E;
        float* sums = part + (size_t)EPW * 24;
        float* sc = sums + (size_t)EPW * 4;
        int* nund = reinterpret_cast<int*>(sc + (size_t)EPW * 3);
        for (int el = 0; el < EPW; ++el) {  // one wave: ballot compaction
            const int gb = env0 + el;
            if (gb >= B) break;
            const float* dm = s.damaged + (size_t)gb * E;
            const float* fl = s.flow + (size_t)gb * E;
            int cnt = 0;
            for (int b0 = 0; b0 < E; b0 += L) {
                const int e = b0 + tid;
                const bool und = e < E && dm[e] == 0.0f;
                const unsigned long long m = __ballot(und);
                if (und) cflow[el * E + cnt + __popcll(m & ((1ull << tid) - 1ull))] = fl[e];
                cnt += __popcll(m);
            }
            if (tid == 0) nund[el] = cnt;
        }
        __syncthreads();
        for (int t = tid; t < EPW * 24; t += L) {
            const int el = t / 24, q = (t / 8) % 3, jj = t % 8, gb = env0 + el;
            if (gb >= B) continue;
            const int n = q == 2 ? nund[el] : E;
            if (n < 8) continue;
            const float* go = s.goal + (size_t)gb * E;
            const float* dm = s.damaged + (size_t)gb * E;
            const float* cf = cflow + el * E;
            auto a = [&](int i) { return q == 0 ? __fmul_rn(go[i], dm[i]) : (q == 1 ? go[i] : cf[i]); };
            float r = a(jj);
            for (int i = 8; i < n - (n % 8); i += 8) r = __fadd_rn(r, a(i + jj));
            part[t] = r;
        }
        __syncthreads();
        for (int t = tid; t < EPW * 4; t += L) {
            const int el = t / 4, q = t % 4, gb = env0 + el;
            if (gb >= B) continue;
            float res = 0.0f;
            if (q == 3) {
                for (int v = 0; v < N; ++v) res = fmaxf(res, bwv[el * N + v]);
            } else {
                const int n = q == 2 ? nund[el] : E;
                const float* go = s.goal + (size_t)gb * E;
                const float* dm = s.damaged + (size_t)gb * E;
                const float* cf = cflow + el * E;
                auto a = [&](int i) { return q == 0 ? __fmul_rn(go[i], dm[i]) : (q == 1 ? go[i] : cf[i]); };
                int i = 0;
                if (n >= 8) {
                    const float* r = part + el * 24 + q * 8;
                    res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                                    __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
                    i = n - (n % 8);
                }
                for (; i < n; ++i) res = __fadd_rn(res, a(i));
            }
            sums[t] = res;
        }
        __syncthreads();
        if (tid < EPW && env0 + tid < B) {
            const float* sm = sums + tid * 4;
            obs_env_scalars(g, s, env0 + tid, sm[0], sm[1], sm[2], nund[tid], sc + tid * 3);
        }
        __syncthreads();
        for (int i = tid; i < EPW * N; i += L) {
            const int el = i / N, v = i - el * N, gb = env0 + el;
            if (gb < B) obs_node_features(N, gb, v, bwv[i], sums[el * 4 + 3], sc + el * 3, node_x);
        }
    }
    for (int i = tid; i < EPW * E; i += L) {
        int el = i / E, e = i - el * E, gb = env0 + el;
        if (gb < B) obs_edge_features(g, s, gb, e, edge_x, mask);
    }
}

static size_t observe_smem(const DevGraph& g, int epw) {
    size_t b = (((size_t)g.N * kObsThreads * 12 + 2 * (size_t)epw * g.E + (size_t)epw * g.N + 15) & ~size_t(15));
    b += 16 * 4 + ((size_t)3 * g.N + 2) * 2;
    // bwv reuses the packed BFS words (epw*N floats <= N*L u32) and the feature scratch reuses
    // delta (epw*(E+8) floats <= N*L doubles), both checked at launch
    return b;
}

hipError_t launch_observe_kernel(const DevGraph& g, int B, const trx_state& s, float* node_x, float* edge_x,
                                 float* mask, hipStream_t stream) {
    int epw = kObsThreads / g.N;
    if (epw < 1) return hipErrorInvalidValue;
    // feature scratch in delta: epw*(E+8) floats (E > 128) or epw*(E+32)+epw floats (E <= 128)
    if ((size_t)epw * (g.E + 33) > (size_t)g.N * kObsThreads * 2) return hipErrorInvalidValue;
    // bw0 / bw1 hold 2 entries per thread; i8 CSR heads / tails; the u16 sigma bound needs N <= 32
    if (epw * g.N > 2 * kObsThreads || g.N > kSmallMaxNodes || g.N > 127) return hipErrorInvalidValue;
    int blocks = (B + epw - 1) / epw;
    hipLaunchKernelGGL(observe_kernel, dim3(blocks), dim3(kObsThreads), observe_smem(g, epw), stream, g, s, B, epw,
                       node_x, edge_x, mask);
    return hipGetLastError();
}

}  // namespace trx

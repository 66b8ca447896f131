// assign_quad.hip -- fused batched static traffic assignment, gfx950, v2.
//
// The general small-graph (N <= 32) env kernel for both shortest-path rules:
// the dispatcher (capi.hip select_env_kernel) runs it for graphs outside the
// sparse kernel's exact-label / out-degree preconditions (scipy rule) and the
// torch-rule kernel's LDS budget (torch rule), and on TRX_KERNEL=quad.
// Contract: src/env/repair_env.py:299-345, 207-237, 167-205.  Mapping: each (env, origin) shortest-path tree is owned
// by a QUAD of lanes instead of one lane.  Lane j of the quad owns nodes
// v = 4i + j (i < NP/4), keeping their float64 labels and predecessor info in
// VGPRs.  One Dijkstra extraction is:
//     local argmin over the lane's <= 8 unscanned labels
//  -> 2 DPP quad_perm butterfly steps (xor 1, xor 2) on (label, node id)
//  -> relax the lane's own nodes from the extracted node u, reading one
//     contiguous LDS row slice  Wq[env][u][j][0..NP/4)
// so the critical path per extraction is ~60 VALU ops instead of ~360 and the
// kernel runs at ~40 VGPRs (8 waves/SIMD) instead of 256+AGPR spill.
// Tie handling is unchanged: extraction ties break by node id; any
// equal-label, equal-cost predecessor tie marks the tree ambiguous and it is
// replayed with the exact scipy Fibonacci heap (per-wave LDS block).
// AON loading walks each destination's predecessor path (4 lanes in parallel
// per tree) and adds the integer demand with LDS float atomics: exact and
// order-independent (integral demands, total < 2^24, checked on the host).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device_common.h"
#include "trx_internal.h"

#ifdef TRX_PHASE_STAMPS
// Diagnostic build only: per-phase cycle totals (thread 0 of each workgroup,
// summed over workgroups).  Never compiled into the shipped library.
__device__ unsigned long long trx_phase_cycles[8];
#define TRX_STAMP(slot)                                                     \
    do {                                                                    \
        if (threadIdx.x == 0) {                                             \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
            atomicAdd(&trx_phase_cycles[slot], now_ - stamp_prev_);          \
            stamp_prev_ = now_;                                             \
        }                                                                   \
    } while (0)
extern "C" int trx_debug_phase_cycles(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_phase_cycles), sizeof(unsigned long long) * 8) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(trx_phase_cycles), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define TRX_STAMP(slot) \
    do {                \
    } while (0)
#endif

namespace trx {

namespace {

constexpr int kQuad = 4;

// Byte offsets of the LDS regions (plain integers: the kernel derives typed
// LDS pointers from them, so no pointer table is ever materialised).
struct SmemQ {
    uint32_t flow, cap, dmg, goal, t, aux, dprev;  // [EPW*E] f32
    uint32_t w;      // [EPW][NP(u)][4(j)][NP/4(i)] f32: cost of u -> 4i+j
    uint32_t pred;   // [EPW*Z][NP] u8 per tree
    uint32_t ord;    // [EPW*Z][NP] u8 scan order per tree
    uint32_t dist;   // [EPW*Z][NP] f64 labels per tree (tie post-pass)
    uint32_t nscan;  // [EPW*Z] i32
    uint32_t inptr;  // [N+1] i16 in-edge CSR
    uint32_t insrc;  // [E] u8
    uint32_t eid;    // [NP*NP] i16
    uint32_t dem;    // [Z*N] f32
    uint32_t t0;     // [E] f32 free-flow times (read by every BPR pass)
    uint32_t unas;   // [L] f32
    uint32_t act;    // [EPW] i32
    uint32_t red;    // [EPW*2] f64
    uint32_t heap;   // [L/64] FibLane
    uint32_t total;
};

__host__ __device__ inline uint32_t align16q(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline SmemQ smemq_layout(int E, int N, int Z, int NP, int EPW, int L, bool fw = false) {
    SmemQ o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t bytes) {
        uint32_t r = off;
        off = align16q(off + bytes);
        return r;
    };
    const uint32_t el = (uint32_t)(EPW * E * 4);
    o.flow = take(el);
    o.cap = take(el);
    o.dmg = take(el);
    o.goal = take(el);
    o.t = take(el);
    o.aux = take(el);
    o.dprev = take(el);
    o.w = take((uint32_t)(EPW * NP * NP * 4));
    o.pred = take((uint32_t)(EPW * Z * NP));
    o.ord = take((uint32_t)(EPW * Z * NP));
    // (torch rule: the [EPW][NP][NP] u8 next-hop tables live here instead)
    o.dist = take((uint32_t)(fw && EPW * NP * NP > EPW * Z * NP * 8 ? EPW * NP * NP : EPW * Z * NP * 8));
    o.nscan = take((uint32_t)(EPW * Z * 4));
    o.inptr = take((uint32_t)((N + 1) * 2));
    o.insrc = take((uint32_t)E);
    o.eid = take((uint32_t)(NP * NP * 2));
    o.dem = take((uint32_t)(Z * N * 4));
    o.t0 = take((uint32_t)(E * 4));
    o.unas = take((uint32_t)(L * 4));
    o.act = take((uint32_t)(EPW * 4));
    o.red = take((uint32_t)(EPW * 2 * 8));
    o.heap = take((uint32_t)(((L + 63) / 64) * sizeof(FibLane)));
    o.total = off;
    return o;
}

// DPP quad_perm controls: xor 1 = [1,0,3,2], xor 2 = [2,3,0,1]
template <int CTRL>
__device__ __forceinline__ int qperm(int x) {
    return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double qperm_d(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(qperm<CTRL>(hi), qperm<CTRL>(lo));
}
template <int CTRL>
__device__ __forceinline__ void quad_min_step(double& best, int& bu) {
    double ob = qperm_d<CTRL>(best);
    int ou = qperm<CTRL>(bu);
    bool take = ob < best || (ob == best && ou < bu);
    best = take ? ob : best;
    bu = take ? ou : bu;
}

}  // namespace

// Shortest-path rule of the all-or-nothing step:
//  kSpScipy  _all_or_nothing, scipy branch (repair_env.py:481-503, 707-722):
//            Dijkstra, float64 labels, scipy heap order on ties;
//  kSpTorch  _all_or_nothing_torch (repair_env.py:520-573): float32 all-pairs
//            Floyd-Warshall (k ascending, strict <) and a next_hop walk per OD
//            pair (at most N hops; a pair that misses its destination is
//            unassigned; intrazonal pairs are skipped).
constexpr int kSpScipy = 0;
constexpr int kSpTorch = 1;

template <int NP, int SP = kSpScipy>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(5, 8))) env_kernel_q(const DevGraph g, const trx_params p, const trx_state s, int B,
                                                    int EPW, int mode, const int32_t* __restrict__ action,
                                                    double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                    uint8_t* __restrict__ valid_out,
                                                    const uint8_t* __restrict__ env_mask) {
    constexpr int NPL = NP / kQuad;  // nodes per lane
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N, Z = g.Z;
    const int L = blockDim.x;
    const int tid = threadIdx.x;
    const int EL = EPW * E;
    const int env0 = blockIdx.x * EPW;
    const SmemQ O = smemq_layout(E, N, Z, NP, EPW, L, SP == kSpTorch);
    struct {
        float *flow, *cap, *dmg, *goal, *t, *aux, *dprev, *w, *dem, *unas;
        uint8_t *pred, *ord, *insrc;
        double *dist, *red;
        int *nscan, *act;
        int16_t *inptr, *eid;
        FibLane* heap;
        float* t0;
    } S = {(float*)(smem_raw + O.flow), (float*)(smem_raw + O.cap),   (float*)(smem_raw + O.dmg),
           (float*)(smem_raw + O.goal), (float*)(smem_raw + O.t),     (float*)(smem_raw + O.aux),
           (float*)(smem_raw + O.dprev), (float*)(smem_raw + O.w),    (float*)(smem_raw + O.dem),
           (float*)(smem_raw + O.unas), smem_raw + O.pred,            smem_raw + O.ord,
           smem_raw + O.insrc,          (double*)(smem_raw + O.dist), (double*)(smem_raw + O.red),
           (int*)(smem_raw + O.nscan),  (int*)(smem_raw + O.act),     (int16_t*)(smem_raw + O.inptr),
           (int16_t*)(smem_raw + O.eid), (FibLane*)(smem_raw + O.heap), (float*)(smem_raw + O.t0)};
#ifdef TRX_PHASE_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif

    // ------------------------------------------------ per-env activation
    if (tid < EPW) {
        int gb = env0 + tid;
        int active = 0;
        if (gb < B) {
            if (mode == kModeStep) {
                int a = action[gb];
                // out-of-range ids (the host check is optional: check=False) are
                // memory-safe no-ops, reported like an already-repaired link
                active = (unsigned)a < (unsigned)E && s.damaged[(size_t)gb * E + a] != 0.0f;  // repair_env.py:210
                if (!active) {
                    reward_out[gb] = -1.0;
                    done_out[gb] = 0;
                    valid_out[gb] = 0;
                }
            } else {
                active = env_mask ? (env_mask[gb] != 0) : 1;
            }
        }
        S.act[tid] = active;
    }
    for (int i = tid; i < NP * NP; i += L) S.eid[i] = g.eid_of[i];
    // the cost-table region doubles as the [E] i16 scratch of link positions below
    int16_t* wpos_tmp = reinterpret_cast<int16_t*>(S.w);
    for (int i = tid; i < E; i += L) wpos_tmp[i] = -1;
    for (int i = tid; i < Z * N; i += L) S.dem[i] = g.dem[i];
    for (int i = tid; i <= N; i += L) S.inptr[i] = (int16_t)g.in_ptr[i];
    for (int i = tid; i < E; i += L) S.insrc[i] = (uint8_t)g.in_src[i];
    for (int i = tid; i < E; i += L) S.t0[i] = g.t0[i];
    __syncthreads();
    // cost tables in quad layout: entries without a link stay +inf for the whole
    // launch; only the link entries are rewritten per MSA iteration.  Thread i
    // (< EPW*E <= L) keeps the table position of env-link i in a register.
    for (int i = tid; i < NP * NP; i += L) {
        const int e = S.eid[i];
        if (e >= 0) {
            const int u = i / NP, v = i - u * NP;
            wpos_tmp[e] = (int16_t)(u * NP + (v & (kQuad - 1)) * NPL + (v >> 2));
        }
    }
    __syncthreads();
    const bool wpos_reg = EL <= L;
    int my_wpos = -1;
    if (wpos_reg && tid < EL) {
        const int el = tid / E, e = tid - el * E;
        const int pos = wpos_tmp[e];
        my_wpos = pos >= 0 ? el * NP * NP + pos : -1;
    }
    __syncthreads();
    for (int x = tid; x < EPW * NP * NP; x += L) S.w[x] = kInfF;

    // ------------------------------------------------------- load state
    for (int i = tid; i < EL; i += L) {
        int el = i / E, e = i % E;
        int gb = env0 + el;
        float fl = 0.f, cp = 0.f, dm = 0.f, gl = 0.f;
        if (S.act[el]) {
            size_t gi = (size_t)gb * E + e;
            if (mode == kModeReset) {
                dm = s.damaged[gi];  // repair_env.py:193-198
                cp = dm != 0.0f ? p.capacity_damage : g.cap0[e];
                gl = dm;
            } else {
                fl = s.flow[gi];
                cp = s.capacity[gi];
                dm = s.damaged[gi];
                gl = s.goal[gi];
                if (mode == kModeStep && e == action[gb]) {  // repair_env.py:215-216
                    dm = 0.0f;
                    cp = g.cap0[e];
                }
            }
        }
        S.flow[i] = fl;
        S.cap[i] = cp;
        S.dmg[i] = dm;
        S.goal[i] = gl;
        S.aux[i] = 0.0f;
        S.dprev[i] = 0.0f;
        S.t[i] = S.act[el] ? bpr_cost(fl, cp, S.t0[e], dm, p.bpr_alpha, p.bpr_beta) : 0.0f;
    }
    __syncthreads();
    TRX_STAMP(0);

    // thread -> (tree = (env, origin zone), lane j of its quad)
    const int tree = tid / kQuad;
    const int j = tid & (kQuad - 1);
    const int lenv = tree / Z;
    const int zi = tree - lenv * Z;
    const bool tree_on = (lenv < EPW) && S.act[lenv];
    const int origin = tree_on ? g.origins[zi] : 0;
    float unassigned_lane = 0.0f;

    for (int it = 0; it < p.iters; ++it) {
      if constexpr (SP == kSpTorch) {
        // ---------------- _all_or_nothing_torch (repair_env.py:524-543): per env a
        //                  row-major float32 dist table D[u][v] (the cost-table
        //                  region) and u8 next-hop table H[u][v] (0xFF = -1)
        float* D = S.w;
        uint8_t* H = reinterpret_cast<uint8_t*>(S.dist);
        for (int x = tid; x < EPW * NP * NP; x += L) {
            const int el = x / (NP * NP), r = x - el * NP * NP;
            const int u = r / NP, v = r - u * NP;
            const int e = S.eid[r];
            // dist = 1e12, diag 0, then dist[row, col] = t per link (524-535)
            D[x] = e >= 0 ? S.t[el * E + e] : (u == v ? 0.0f : 1e12f);
            H[x] = e >= 0 ? (uint8_t)v : (uint8_t)0xFF;
        }
        __syncthreads();
        // k ascending, strict <; row k and column k do not change during step k
        // (D[k][k] + w is never < w for w >= 0), so the in-place update is the
        // reference's whole-matrix torch.where (537-542)
        for (int k = 0; k < N; ++k) {
            for (int x = tid; x < EPW * N * N; x += L) {
                const int el = x / (N * N), r = x - el * N * N;
                const int i = r / N, j2 = r - i * N;
                const int base = el * NP * NP;
                const float alt = __fadd_rn(D[base + i * NP + k], D[base + k * NP + j2]);
                if (alt < D[base + i * NP + j2]) {
                    D[base + i * NP + j2] = alt;
                    H[base + i * NP + j2] = H[base + i * NP + k];
                }
            }
            __syncthreads();
        }
        TRX_STAMP(2);
        // next_hop walk per OD pair (548-568), lane j of the origin's quad walks
        // destinations v = 4i + j; integer demands make the LDS float atomics exact
        if (tree_on) {
            const uint8_t* Hl = H + lenv * NP * NP;
            const float* dm = S.dem + zi * N;
            float* aux = S.aux + lenv * E;
            float un = 0.0f;
            for (int i = 0; i < NPL; ++i) {
                const int v = kQuad * i + j;
                if (v >= N || v == origin) continue;  // origin == dest: skipped (551-552)
                const float dv = dm[v];
                if (!(dv > 0.0f)) continue;
                int cur = origin, hops = 0;
                while (cur != v && hops < N) {
                    const int nx = Hl[cur * NP + v];
                    if (nx == 0xFF) break;
                    cur = nx;
                    ++hops;
                }
                if (cur != v) {
                    un += dv;  // unassigned; the partial path is dropped (564-566)
                    continue;
                }
                cur = origin;
                while (cur != v) {
                    const int nx = Hl[cur * NP + v];
                    atomicAdd(&aux[S.eid[cur * NP + nx]], dv);
                    cur = nx;
                }
            }
            unassigned_lane = un;
        }
        __syncthreads();
        TRX_STAMP(4);
      } else {
        // ---------------- per-env cost rows in quad layout (LDS): the link entries
        //                  (u -> v = 4*ii + jj at column c = jj * NPL + ii of row u)
        if (wpos_reg) {
            if (my_wpos >= 0) S.w[my_wpos] = S.t[tid];
        } else {
            for (int x = tid; x < EPW * NP * NP; x += L) {
                int el = x / (NP * NP), r = x - el * NP * NP;
                int u = r / NP, c = r - u * NP;  // c = jj * NPL + ii  ->  v = 4*ii + jj
                int v = kQuad * (c % NPL) + c / NPL;
                int e = S.eid[u * NP + v];
                S.w[x] = e >= 0 ? S.t[el * E + e] : kInfF;
            }
        }
        __syncthreads();
        TRX_STAMP(1);

        // ---------------- shortest-path tree per quad (Dijkstra, float64 labels)
        bool amb_tree = false;
        if (tree_on) {
            const float* Wl = S.w + lenv * NP * NP;
            uint8_t* ord = S.ord + tree * NP;
            double d[NPL];
            uint32_t pr[NPL];  // predecessor node id, kNoPred = none
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                d[i] = (kQuad * i + j == origin) ? 0.0 : kInfD;
                pr[i] = kNoPred;
            }
            uint32_t scanned = 0u;
            int k = 0;
            for (; k < N; ++k) {
                double best = kInfD;
                int bu = 0x7fffffff;
#pragma unroll
                for (int i = 0; i < NPL; ++i) {
                    bool c = !((scanned >> i) & 1u) && d[i] < best;
                    best = c ? d[i] : best;
                    bu = c ? kQuad * i + j : bu;
                }
                quad_min_step<0xB1>(best, bu);
                quad_min_step<0x4E>(best, bu);
                if (!(best < kInfD)) break;  // quad-uniform
                const int u = bu;
                if ((u & (kQuad - 1)) == j) scanned |= 1u << (u >> 2);
                if (j == 0) ord[k] = (uint8_t)u;
                const float* row = Wl + u * NP + j * NPL;
                float wv[NPL];
                if constexpr (NPL % 4 == 0) {
#pragma unroll
                    for (int q = 0; q < NPL / 4; ++q) {
                        float4 w4 = reinterpret_cast<const float4*>(row)[q];
                        wv[4 * q] = w4.x; wv[4 * q + 1] = w4.y; wv[4 * q + 2] = w4.z; wv[4 * q + 3] = w4.w;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < NPL / 2; ++q) {
                        float2 w2 = reinterpret_cast<const float2*>(row)[q];
                        wv[2 * q] = w2.x; wv[2 * q + 1] = w2.y;
                    }
                }
                // strict improvement (scipy `current_node.val > next_val`); scanned
                // labels never improve since costs are > 0
#pragma unroll
                for (int i = 0; i < NPL; ++i) {
                    double nd = __dadd_rn(best, (double)wv[i]);
                    bool better = nd < d[i];
                    d[i] = better ? nd : d[i];
                    pr[i] = better ? (uint32_t)u : pr[i];
                }
            }
            if (j == 0) S.nscan[tree] = k;
            double* dl = S.dist + tree * NP;
            uint8_t* pl = S.pred + tree * NP;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                dl[kQuad * i + j] = d[i];
                pl[kQuad * i + j] = (uint8_t)pr[i];
            }
            // tie post-pass: ambiguous iff some node has >= 2 equal-cost tails at
            // the smallest tail label (scipy's heap order then picks the pred).
            // Labels of other lanes are read back from LDS (same wave: in order).
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int amb = 0;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int v = kQuad * i + j;
                if (v < N && v != origin && d[i] < kInfD) {
                    double m = kInfD;
                    int cnt = 0;
                    for (int q = S.inptr[v]; q < S.inptr[v + 1]; ++q) {
                        int u = S.insrc[q];
                        double du = dl[u];
                        double nd = __dadd_rn(du, (double)Wl[u * NP + j * NPL + i]);
                        if (nd == d[i]) {
                            cnt = du < m ? 1 : (du == m ? cnt + 1 : cnt);
                            m = du < m ? du : m;
                        }
                    }
                    amb |= cnt > 1;
                }
            }
            amb |= qperm<0xB1>(amb);
            amb |= qperm<0x4E>(amb);
            amb_tree = amb != 0;
        }
        TRX_STAMP(2);
        {
            uint64_t pending = __ballot(tree_on && amb_tree && j == 0);
            FibLane* h = S.heap + (tid >> 6);
            while (pending) {
                int leader = __ffsll((unsigned long long)pending) - 1;
                if ((tid & 63) == leader) {
                    const float* Wl = S.w + lenv * NP * NP;
                    S.nscan[tree] = exact_sssp(
                        N, g.indptr, g.indices,
                        [Wl](int a_, int b_) { return Wl[a_ * NP + (b_ & 3) * NPL + (b_ >> 2)]; }, origin, h,
                        S.ord + tree * NP, S.pred + tree * NP, 1, 0);
                }
                pending &= pending - 1;
            }
        }
        __syncthreads();
        TRX_STAMP(3);

        // ---------------- all-or-nothing: subtree accumulation in reverse scan
        // order (repair_env.py:490-502 summed per tree; integer demands make
        // the float sums exact in any order).  Reachable <=> has a predecessor.
        if (tree_on) {
            uint32_t pr[NPL];
#pragma unroll
            for (int i = 0; i < NPL; ++i) pr[i] = S.pred[tree * NP + kQuad * i + j];
            const int nscan = S.nscan[tree];
            const float* dm = S.dem + zi * N;
            float acc[NPL];
            float un = 0.0f;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int v = kQuad * i + j;
                float dv = v < N ? dm[v] : 0.0f;
                bool reach = pr[i] != kNoPred;
                acc[i] = reach ? dv : 0.0f;
                un += reach ? 0.0f : dv;  // unreachable or intrazonal (repair_env.py:708)
            }
            unassigned_lane = un;
            uint32_t ow[NP / 4];
            const uint32_t* ordw = reinterpret_cast<const uint32_t*>(S.ord + tree * NP);
#pragma unroll
            for (int q = 0; q < NP / 4; ++q) ow[q] = ordw[q];
            float* aux = S.aux + lenv * E;
#pragma unroll
            for (int k = NP - 1; k >= 1; --k) {
                if (k < nscan) {  // quad-uniform
                    const int v = (ow[k >> 2] >> (8 * (k & 3))) & 0xFF;
                    const int slot = v >> 2;
                    float av = 0.0f;
                    int pv = 0;
#pragma unroll
                    for (int i = 0; i < NPL; ++i) {
                        av = (i == slot) ? acc[i] : av;
                        pv = (i == slot) ? (int)pr[i] : pv;
                    }
                    const bool mine = (v & (kQuad - 1)) == j;
                    av = mine ? av : 0.0f;
                    pv = mine ? pv : 0;
                    // exactly one lane holds the values: quad sums broadcast them
                    av += __int_as_float(qperm<0xB1>(__float_as_int(av)));
                    av += __int_as_float(qperm<0x4E>(__float_as_int(av)));
                    pv |= qperm<0xB1>(pv);
                    pv |= qperm<0x4E>(pv);
                    if (av != 0.0f) {
                        const bool pmine = (pv & (kQuad - 1)) == j;
                        const int ps = pv >> 2;
#pragma unroll
                        for (int i = 0; i < NPL; ++i) acc[i] = (pmine && i == ps) ? acc[i] + av : acc[i];
                        if (pmine) atomicAdd(&aux[S.eid[pv * NP + v]], av);
                    }
                }
            }
        }
        __syncthreads();
        TRX_STAMP(4);
      }  // SP

        // ---------------- flow update + BPR (repair_env.py:317-342)
        if (p.method == TRX_METHOD_CFW) {
            if (tid < EPW && S.act[tid]) {
                double num = 0.0, den = 0.0;
                const float* fl = S.flow + tid * E;
                const float* ax = S.aux + tid * E;
                const float* dp = S.dprev + tid * E;
                for (int e = 0; e < E; ++e) {
                    float dfw = __fsub_rn(ax[e], fl[e]);
                    num += (double)__fmul_rn(dfw, __fsub_rn(dfw, dp[e]));
                    den += (double)__fmul_rn(dp[e], dp[e]);
                }
                S.red[2 * tid] = num;
                S.red[2 * tid + 1] = den;
            }
            __syncthreads();
        }
        const double stepd = (p.method == TRX_METHOD_MSA) ? 1.0 / (it + 1.0) : 2.0 / (it + 2.0);
        const float s32 = (float)stepd, om32 = (float)(1.0 - stepd);
        for (int i = tid; i < EL; i += L) {
            int el = i / E, e = i - el * E;
            if (!S.act[el]) continue;
            float fl = S.flow[i];
            float ax = S.aux[i];
            float nf;
            if (p.method == TRX_METHOD_CFW) {
                float dfw = __fsub_rn(ax, fl);
                float dir;
                if (it == 0) {
                    dir = dfw;
                } else {
                    float num = (float)S.red[2 * el];
                    double den = (double)(float)S.red[2 * el + 1] + 1e-12;
                    double b = (double)num / den;
                    b = b < 0.0 ? 0.0 : b;
                    dir = __fadd_rn(dfw, __fmul_rn((float)b, S.dprev[i]));
                }
                nf = __fadd_rn(fl, __fmul_rn(s32, dir));
                nf = nf > 0.0f ? nf : 0.0f;
                S.dprev[i] = dir;
            } else {
                nf = __fadd_rn(__fmul_rn(om32, fl), __fmul_rn(s32, ax));
            }
            if (nf != nf) nf = 0.0f;  // nan_to_num guard (repair_env.py:338-340)
            S.flow[i] = nf;
            S.aux[i] = 0.0f;
            S.t[i] = bpr_cost(nf, S.cap[i], S.t0[e], S.dmg[i], p.bpr_alpha, p.bpr_beta);
        }
        __syncthreads();
        TRX_STAMP(5);
    }

    // ---------------- per-env unassigned (tree order, exact integers)
    S.unas[tid] = unassigned_lane;
    __syncthreads();
    for (int i = tid; i < EL; i += L) S.aux[i] = __fmul_rn(S.flow[i], S.t[i]);
    __syncthreads();

    if (tid < EPW && S.act[tid]) {
        int gb = env0 + tid;
        double un = 0.0;
        for (int x = 0; x < Z * kQuad; ++x) un += (double)S.unas[tid * Z * kQuad + x];
        double base = (double)pairwise_sum(S.aux + tid * E, E);
        double td = g.total_demand > 1.0 ? g.total_demand : 1.0;
        double tstt = base / td + (un > 0 ? p.unassigned_penalty * (un / td) : 0.0);  // repair_env.py:724-735
        double prev = s.tstt[gb];
        s.tstt[gb] = tstt;
        s.unassigned[gb] = un;
        if (mode == kModeReset) s.initial_tstt[gb] = tstt;
        if (mode == kModeStep) {
            float rem = 0.0f;
            for (int e = 0; e < E; ++e) rem += __fmul_rn(S.goal[tid * E + e], S.dmg[tid * E + e]);
            bool complete = rem == 0.0f;  // is_goal_complete (293-294)
            reward_out[gb] = reward_fn(p, prev, tstt, s.initial_tstt[gb], complete);
            done_out[gb] = complete ? 1 : 0;
            valid_out[gb] = 1;
        }
    }
    for (int i = tid; i < EL; i += L) {
        int el = i / E;
        if (!S.act[el]) continue;
        size_t gi = (size_t)(env0 + el) * E + (i - el * E);
        s.flow[gi] = S.flow[i];
        if (s.t) s.t[gi] = S.t[i];
        if (mode != kModeAssign) {
            s.capacity[gi] = S.cap[i];
            s.damaged[gi] = S.dmg[i];
            s.goal[gi] = S.goal[i];
        }
    }
    __syncthreads();
    TRX_STAMP(6);
}

LaunchCfg quad_launch_cfg(const DevGraph& g, int num_envs, int sp_rule) {
    LaunchCfg c{};
    c.np = g.NP;
    // envs per workgroup: fill up to 512 threads with whole envs (Z quads each)
    int per_env = g.Z * kQuad;
    static const int epw_env = [] {
        const char* e = getenv("TRX_EPW");  // tuning knob (A/B runs)
        return e ? atoi(e) : 0;
    }();
    int epw = epw_env > 0 ? epw_env : 2;  // SF: 2 envs = 192 threads, 6 workgroups/CU at 96 VGPRs
    while (epw > 1 && epw * per_env > 512) --epw;
    c.epw = epw;
    c.threads = ((epw * per_env + 63) / 64) * 64;
    c.smem = smemq_layout(g.E, g.N, g.Z, c.np, c.epw, c.threads, sp_rule == TRX_SP_TORCH).total;
    c.blocks = (num_envs + c.epw - 1) / c.epw;
    return c;
}

bool quad_ok(const DevGraph& g, int sp_rule) {
    if (g.N > kSmallMaxNodes) return false;
    const LaunchCfg c = quad_launch_cfg(g, 1, sp_rule);
    return c.threads <= 512 && c.smem <= 64 * 1024;
}

hipError_t launch_env_kernel_quad(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                  const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                  const uint8_t* env_mask, hipStream_t stream) {
    LaunchCfg c = quad_launch_cfg(g, num_envs, p.sp_rule);
    if (c.blocks == 0) return hipSuccess;
    if (c.threads > 512 || c.smem > 64 * 1024) return hipErrorInvalidConfiguration;
    dim3 grid(c.blocks), block(c.threads);
    if (p.sp_rule == TRX_SP_TORCH) {
        switch (c.np) {
            case 8:
                hipLaunchKernelGGL((env_kernel_q<8, kSpTorch>), grid, block, c.smem, stream, g, p, s, num_envs, c.epw,
                                   mode, action, reward, done, valid, env_mask);
                break;
            case 16:
                hipLaunchKernelGGL((env_kernel_q<16, kSpTorch>), grid, block, c.smem, stream, g, p, s, num_envs,
                                   c.epw, mode, action, reward, done, valid, env_mask);
                break;
            case 24:
                hipLaunchKernelGGL((env_kernel_q<24, kSpTorch>), grid, block, c.smem, stream, g, p, s, num_envs,
                                   c.epw, mode, action, reward, done, valid, env_mask);
                break;
            default:
                hipLaunchKernelGGL((env_kernel_q<32, kSpTorch>), grid, block, c.smem, stream, g, p, s, num_envs,
                                   c.epw, mode, action, reward, done, valid, env_mask);
                break;
        }
        return hipGetLastError();
    }
    switch (c.np) {
        case 8:
            hipLaunchKernelGGL(env_kernel_q<8>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
        case 16:
            hipLaunchKernelGGL(env_kernel_q<16>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
        case 24:
            hipLaunchKernelGGL(env_kernel_q<24>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
        default:
            hipLaunchKernelGGL(env_kernel_q<32>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
    }
    return hipGetLastError();
}

}  // namespace trx

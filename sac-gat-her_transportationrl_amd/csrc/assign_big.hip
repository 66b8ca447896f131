// assign_big.hip -- fused batched static traffic assignment for networks larger
// than the register-resident kernel takes (N > 32: Anaheim-sized, SURVEY.md
// §8(d) config #5), gfx950.
//
// Same contract as assign_quad.hip (src/env/repair_env.py:299-345 assignment,
// 207-237 step, 167-205 reset, 724-735 TSTT, 244-294 reward): one workgroup
// per env, the env's link flows / costs / aux flows resident in LDS for the
// whole call, HBM touched at the start and the end.  Shortest-path trees
// (env, origin zone) are handed to waves by an LDS counter; a tree is owned by
// G lanes (G = 64: one tree per wave; G = 32: two trees per wave, each half
// running its own tree through the same instruction stream):
//
//   labels   pull-based Bellman-Ford in float64.  Rounded addition is
//            monotone and costs are > 0, so the least fixed point of
//                d[v] = min_u fl(d[u] + w(u,v)),  d[origin] = 0
//            is exactly the label set scipy's Dijkstra computes, whatever the
//            relaxation order.  Nodes are numbered by DFS position and dealt
//            to the G lanes in contiguous chunks (capi.hip); each lane relaxes
//            its nodes' in-links Gauss-Seidel against the LDS labels (a label
//            found early in the chunk is used by the rest of the chunk in the
//            same sweep), alternating the sweep direction.
//   preds    scipy records for v the first scanned tail achieving d[v], i.e.
//            the achieving tail with the smallest label.  A post pass picks it;
//            if two achieving tails share that label the heap order decides,
//            and the tree is replayed with the exact scipy Fibonacci heap
//            (device_common.h, per-tree scratch in the caller's workspace).
//   AON      the tree's lanes walk its OD destinations back to the origin
//            along packed (link | tail << 16) predecessors and add the demand
//            with LDS float atomics: exact in any order (integral demands,
//            total < 2^24).
//
// Algorithmic bytes per assignment: SURVEY.md §8(d) (bench.py roofline).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device_common.h"
#include "trx_internal.h"

#ifdef TRX_BIG_STATS
// Diagnostic build only: [0] trees, [1] label sweeps, [2] exact replays,
// [3] label cycles, [4] pred cycles, [5] walk cycles (s_memtime, per wave).
__device__ unsigned long long trx_big_stats[8];
extern "C" int trx_debug_big_stats(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_big_stats), sizeof(unsigned long long) * 8) != hipSuccess) return -2;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(trx_big_stats), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#define TRX_BIG_COUNT(i, n)                                                    \
    do {                                                                       \
        if (lane == 0) atomicAdd(&trx_big_stats[i], (unsigned long long)(n)); \
    } while (0)
#define TRX_BIG_CLOCK() __builtin_amdgcn_s_memtime()
#else
#define TRX_BIG_COUNT(i, n) \
    do {                    \
    } while (0)
#define TRX_BIG_CLOCK() 0ull
#endif

namespace trx {

namespace {

constexpr int kBigMaxWaves = 8;

struct SmemB {
    uint32_t flow, cap, t, aux;  // [E] f32
    uint32_t dmg;                // [E] u8
    uint32_t lsrc;               // [E] i16 tail (DFS position) of each link
    uint32_t ent;                // [KMAX][G] uint2 {packed entry, cost bits}
    uint32_t lnk;                // [KMAX][G] i16 link id of each entry
    uint32_t dist;               // [trees][N+1] f64 labels (+ dummy node N = inf)
    uint32_t pe;                 // [trees][N] i32 predecessor (link | tail << 16), -1 = none
    uint32_t unas;               // [W*64] f32
    uint32_t red;                // [2] f64
    uint32_t misc;               // [4] i32: active, tree counter
    uint32_t total;
};

__host__ __device__ inline uint32_t align16b(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline SmemB smemb_layout(int E, int N, int KMAX, int G, int W) {
    const int trees = W * (64 / G);
    SmemB o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t bytes) {
        uint32_t r = off;
        off = align16b(off + bytes);
        return r;
    };
    o.flow = take(E * 4);
    o.cap = take(E * 4);
    o.t = take(E * 4);
    o.aux = take(E * 4);
    o.dmg = take(E);
    o.lsrc = take(E * 2);
    o.ent = take((uint32_t)(KMAX * G * 8));
    o.lnk = take((uint32_t)(KMAX * G * 2));
    o.dist = take((uint32_t)(trees * (N + 1) * 8));
    o.pe = take((uint32_t)(trees * N * 4));
    o.unas = take((uint32_t)(W * 64 * 4));
    o.red = take(16);
    o.misc = take(16);
    o.total = off;
    return o;
}

// per-tree FibBig scratch: val f64 | parent,left,right,child i16 | rank,state u8 | roots i16[32]
__host__ __device__ inline size_t fib_slot_bytes(int N) {
    size_t n = (size_t)((N + 7) & ~7);
    return ((n * 8 + n * 2 * 4 + n * 2 + 64) + 255) & ~(size_t)255;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// exact scipy-heap replay of one tree (rare: equal-label ties), one lane
__device__ __forceinline__ void exact_replay(const DevGraph& g, const float* tt, int origin, unsigned char* slot_base,
                                          int32_t* pe) {
    const size_t n = (size_t)((g.N + 7) & ~7);
    FibBig fb;
    fb.val = (double*)slot_base;
    fb.parent = (int16_t*)(slot_base + n * 8);
    fb.left = fb.parent + n;
    fb.right = fb.left + n;
    fb.child = fb.right + n;
    fb.rank = (uint8_t*)(fb.child + n);
    fb.state = fb.rank + n;
    fb.roots = (int16_t*)(fb.state + n);
    const int32_t* ce = g.b_csr_eid;
    exact_sssp_links(g.N, g.b_indptr, g.b_indices, ce, [tt, ce](int j) { return tt[ce[j]]; }, origin, &fb, pe);
}

}  // namespace

// entry word: u | v << 16 | first << 30 | last << 31 (u, v: DFS positions)
template <int G>
__global__ void __launch_bounds__(512) env_kernel_big(const DevGraph g, const trx_params p, const trx_state s, int B,
                                                      int mode, const int32_t* __restrict__ action,
                                                      double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                      uint8_t* __restrict__ valid_out,
                                                      const uint8_t* __restrict__ env_mask,
                                                      unsigned char* __restrict__ ws) {
    constexpr int TPW = 64 / G;  // trees per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N, Z = g.Z, KMAX = g.KMAX;
    const int tid = threadIdx.x, L = blockDim.x;
    const int W = L / 64, wave = tid >> 6, lane = tid & 63;
    const int lt = lane & (G - 1), half = lane / G;
    const int gb = blockIdx.x;
    const SmemB O = smemb_layout(E, N, KMAX, G, W);
    float* flow = (float*)(smem_raw + O.flow);
    float* cap = (float*)(smem_raw + O.cap);
    float* tt = (float*)(smem_raw + O.t);
    float* aux = (float*)(smem_raw + O.aux);
    uint32_t* const auxi = (uint32_t*)(smem_raw + O.aux);  // the AON loads, as integers (u32 LDS atomics are
                                                           // native and fast; float ones are not)
    uint8_t* dmg = smem_raw + O.dmg;
    int16_t* lsrc = (int16_t*)(smem_raw + O.lsrc);
    uint2* ent = (uint2*)(smem_raw + O.ent);
    int16_t* lnk = (int16_t*)(smem_raw + O.lnk);
    const int slot = wave * TPW + half;
    double* dist = (double*)(smem_raw + O.dist) + (size_t)slot * (N + 1);
    int32_t* pe = (int32_t*)(smem_raw + O.pe) + (size_t)slot * N;
    float* unas = (float*)(smem_raw + O.unas);
    double* red = (double*)(smem_raw + O.red);
    int* misc = (int*)(smem_raw + O.misc);
    const size_t fib_bytes = (size_t)B * W * TPW * fib_slot_bytes(N);
    unsigned char* fib_slot = ws + ((size_t)blockIdx.x * W * TPW + slot) * fib_slot_bytes(N);
    float* dprev = reinterpret_cast<float*>(ws + fib_bytes) + (size_t)gb * E;  // CFW direction (workspace)

    if (tid == 0) {
        int active = 0;
        if (gb < B) {
            if (mode == kModeStep) {
                int a = action[gb];
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
        misc[0] = active;
    }
    __syncthreads();
    if (!misc[0]) return;  // workgroup-uniform

    // static in-link lists + link tails; state (repair_env.py:193-198, 215-216)
    for (int i = tid; i < KMAX * G; i += L) {
        ent[i].x = g.blist[i];
        lnk[i] = g.blink[i];
    }
    const int a_step = mode == kModeStep ? action[gb] : -1;
    for (int e = tid; e < E; e += L) {
        lsrc[e] = g.b_lsrc[e];
        size_t gi = (size_t)gb * E + e;
        float fl = 0.f, cp, dm;
        if (mode == kModeReset) {
            dm = s.damaged[gi];
            cp = dm != 0.0f ? p.capacity_damage : g.cap0[e];
        } else {
            fl = s.flow[gi];
            cp = s.capacity[gi];
            dm = s.damaged[gi];
            if (e == a_step) {
                dm = 0.0f;
                cp = g.cap0[e];
            }
        }
        flow[e] = fl;
        cap[e] = cp;
        dmg[e] = dm != 0.0f;
        aux[e] = 0.0f;
        if (p.method == TRX_METHOD_CFW) dprev[e] = 0.0f;
        tt[e] = bpr_cost(fl, cp, g.t0[e], dm, p.bpr_alpha, p.bpr_beta);
    }
    __syncthreads();

    float unassigned_lane = 0.0f;
    for (int it = 0; it < p.iters; ++it) {
        // ---------------- per-entry link costs for this iteration
        for (int i = tid; i < KMAX * G; i += L) {
            int e = lnk[i];
            ent[i].y = __float_as_uint(e >= 0 ? tt[e] : kInfF);
        }
        if (tid == 0) misc[1] = 0;
        __syncthreads();

        float un = 0.0f;
        for (;;) {
            int z0 = 0;
            if (lane == 0) z0 = atomicAdd(&misc[1], TPW);
            z0 = __shfl(z0, 0, 64);
            if (z0 >= Z) break;  // wave-uniform
            const int zi = z0 + half;
            const bool on = zi < Z;  // a half without a tree keeps every label at +inf
            const int origin = on ? g.b_origin[zi] : -1;
            TRX_BIG_COUNT(0, (Z - z0) < TPW ? (Z - z0) : TPW);
            [[maybe_unused]] unsigned long long clk0 = TRX_BIG_CLOCK();
            for (int v = lt; v <= N; v += G) dist[v] = v == origin ? 0.0 : kInfD;
            for (int v = lt; v < N; v += G) pe[v] = -1;
            wave_sync();
            // ---------------- labels: alternating Gauss-Seidel sweeps.  Branch-free
            // entry step (the own label is re-stored at every entry, changed
            // only at a group end) and the next entry word prefetched, so the
            // per-entry chain is one label load pair and one store.
            auto relax = [&](const uint2 e, const bool end, double& m, bool& changed) {
                const int v = (e.x >> 16) & 0x3FFF;
                const double xu = dist[e.x & 0xFFFF], dv = dist[v];
                m = __builtin_fmin(m, __dadd_rn(xu, (double)__uint_as_float(e.y)));
                const bool better = end && m < dv;  // strict improvement
                dist[v] = better ? m : dv;
                changed |= better;
                m = end ? kInfD : m;
            };
            int dir = 0;
            for (int sweep = 0; sweep <= N; ++sweep) {
                bool changed = false;
                double m = kInfD;
                if (dir == 0) {
                    uint2 e = ent[lt];
#pragma unroll 2
                    for (int k = 0; k < KMAX; ++k) {
                        const uint2 en = ent[(k + 1 < KMAX ? k + 1 : k) * G + lt];
                        relax(e, (e.x >> 31) != 0, m, changed);
                        e = en;
                    }
                } else {
                    uint2 e = ent[(KMAX - 1) * G + lt];
#pragma unroll 2
                    for (int k = KMAX - 1; k >= 0; --k) {
                        const uint2 en = ent[(k > 0 ? k - 1 : k) * G + lt];
                        relax(e, ((e.x >> 30) & 1u) != 0, m, changed);
                        e = en;
                    }
                }
                wave_sync();
                if (__ballot(changed) == 0) {
                    TRX_BIG_COUNT(1, (sweep + 1) * ((Z - z0) < TPW ? (Z - z0) : TPW));
                    break;
                }
                dir ^= 1;
            }
            [[maybe_unused]] unsigned long long clk1 = TRX_BIG_CLOCK();
            TRX_BIG_COUNT(3, clk1 - clk0);
            // ---------------- predecessors: smallest-label achieving tail
            bool amb = false;
            {
                double mdu = kInfD;
                int cnt = 0, best = -1;
                for (int k = 0; k < KMAX; ++k) {
                    const uint2 e = ent[k * G + lt];
                    if ((e.x >> 30) & 1u) {
                        mdu = kInfD;
                        cnt = 0;
                        best = -1;
                    }
                    const int u = e.x & 0xFFFF, v = (e.x >> 16) & 0x3FFF;
                    const double du = dist[u], dv = dist[v];
                    const double nd = __dadd_rn(du, (double)__uint_as_float(e.y));
                    if (nd == dv && dv < kInfD) {
                        if (du < mdu) {
                            mdu = du;
                            cnt = 1;
                            best = (int)(uint16_t)lnk[k * G + lt] | (u << 16);
                        } else if (du == mdu) {
                            ++cnt;
                        }
                    }
                    if (e.x >> 31) {
                        const bool real = v != origin && v < N && dv < kInfD;
                        if (v < N) pe[v] = real ? best : -1;
                        amb |= real && cnt > 1;
                    }
                }
            }
            wave_sync();
            const uint64_t ambm = __ballot(amb);
            [[maybe_unused]] unsigned long long clk2 = TRX_BIG_CLOCK();
            TRX_BIG_COUNT(4, clk2 - clk1);
            if (ambm != 0) {  // equal-label tie: scipy's heap order decides
                const uint64_t mine = G == 64 ? ambm : (ambm >> (half * G)) & ((1ull << G) - 1);
                TRX_BIG_COUNT(2, 1);
                if (mine != 0 && lt == 0) exact_replay(g, tt, origin, fib_slot, pe);
                wave_sync();
            }
            // ---------------- all-or-nothing by path walks (repair_env.py:490-502, 707-722)
            if (on) {
                for (int q = g.od_ptr[zi] + lt; q < g.od_ptr[zi + 1]; q += G) {
                    const int d = g.b_od_dst[q];
                    const float dm = g.od_dem[q];
                    if (d == origin || pe[d] < 0) {
                        un += dm;  // intrazonal or unreachable (708-709)
                        continue;
                    }
                    int v = d;
                    for (int h = 0; h < N && v != origin; ++h) {
                        const int pk = pe[v];
                        if (pk < 0) break;
                        atomicAdd(&auxi[pk & 0xFFFF], (uint32_t)dm);  // integral demands: u32 atomics
                        v = pk >> 16;
                    }
                }
            }
            wave_sync();
            TRX_BIG_COUNT(5, TRX_BIG_CLOCK() - clk2);
        }
        unassigned_lane = un;
        __syncthreads();
        for (int e = tid; e < E; e += L) aux[e] = (float)auxi[e];  // exact: < 2^24
        __syncthreads();

        // ---------------- flow update + BPR (repair_env.py:317-342)
        if (p.method == TRX_METHOD_CFW) {
            if (tid == 0) {
                double num = 0.0, den = 0.0;
                for (int e = 0; e < E; ++e) {
                    float dfw = __fsub_rn(aux[e], flow[e]);
                    num += (double)__fmul_rn(dfw, __fsub_rn(dfw, dprev[e]));
                    den += (double)__fmul_rn(dprev[e], dprev[e]);
                }
                red[0] = num;
                red[1] = den;
            }
            __syncthreads();
        }
        const double stepd = (p.method == TRX_METHOD_MSA) ? 1.0 / (it + 1.0) : 2.0 / (it + 2.0);
        const float s32 = (float)stepd, om32 = (float)(1.0 - stepd);
        for (int e = tid; e < E; e += L) {
            float fl = flow[e];
            float ax = aux[e];
            float nf;
            if (p.method == TRX_METHOD_CFW) {
                float dfw = __fsub_rn(ax, fl);
                float dir;
                if (it == 0) {
                    dir = dfw;
                } else {
                    float num = (float)red[0];
                    double den = (double)(float)red[1] + 1e-12;
                    double b = (double)num / den;
                    b = b < 0.0 ? 0.0 : b;
                    dir = __fadd_rn(dfw, __fmul_rn((float)b, dprev[e]));
                }
                nf = __fadd_rn(fl, __fmul_rn(s32, dir));
                nf = nf > 0.0f ? nf : 0.0f;
                dprev[e] = dir;
            } else {
                nf = __fadd_rn(__fmul_rn(om32, fl), __fmul_rn(s32, ax));
            }
            if (nf != nf) nf = 0.0f;  // nan_to_num guard (repair_env.py:338-340)
            flow[e] = nf;
            aux[e] = 0.0f;
            tt[e] = bpr_cost(nf, cap[e], g.t0[e], dmg[e] ? 1.0f : 0.0f, p.bpr_alpha, p.bpr_beta);
        }
        __syncthreads();
    }

    // ---------------- TSTT, reward, done (repair_env.py:724-735, 220-236)
    unas[tid] = unassigned_lane;
    for (int e = tid; e < E; e += L) aux[e] = __fmul_rn(flow[e], tt[e]);
    __syncthreads();
    if (tid == 0) {
        double un = 0.0;
        for (int x = 0; x < L; ++x) un += (double)unas[x];
        double base = (double)pairwise_sum_any(aux, E);
        double td = g.total_demand > 1.0 ? g.total_demand : 1.0;
        double tstt = base / td + (un > 0 ? p.unassigned_penalty * (un / td) : 0.0);
        double prev = s.tstt[gb];
        s.tstt[gb] = tstt;
        s.unassigned[gb] = un;
        if (mode == kModeReset) s.initial_tstt[gb] = tstt;
        if (mode == kModeStep) {
            const float* goal = s.goal + (size_t)gb * E;
            float rem = 0.0f;
            for (int e = 0; e < E; ++e) rem += __fmul_rn(goal[e], dmg[e] ? 1.0f : 0.0f);
            bool complete = rem == 0.0f;  // is_goal_complete (293-294)
            reward_out[gb] = reward_fn(p, prev, tstt, s.initial_tstt[gb], complete);
            done_out[gb] = complete ? 1 : 0;
            valid_out[gb] = 1;
        }
    }
    for (int e = tid; e < E; e += L) {
        size_t gi = (size_t)gb * E + e;
        s.flow[gi] = flow[e];
        if (s.t) s.t[gi] = tt[e];
        if (mode != kModeAssign) {
            s.capacity[gi] = cap[e];
            s.damaged[gi] = dmg[e] ? 1.0f : 0.0f;
            if (mode == kModeReset) s.goal[gi] = dmg[e] ? 1.0f : 0.0f;  // goal_mask = is_damaged (200)
        }
    }
}

size_t big_smem_bytes(const DevGraph& g, int waves) { return smemb_layout(g.E, g.N, g.KMAX, g.big_g, waves).total; }

int big_waves(const DevGraph& g) {
    static const int env_w = [] {
        const char* e = getenv("TRX_BIG_WAVES");  // tuning knob (A/B runs)
        return e ? atoi(e) : 0;
    }();
    const int wmax = env_w > 0 && env_w <= kBigMaxWaves ? env_w : kBigMaxWaves;
    // two workgroups per CU when they fit, else as many waves as fit one
    int w = wmax;
    while (w > 1 && big_smem_bytes(g, w) > 80 * 1024) --w;
    if (big_smem_bytes(g, w) <= 80 * 1024) return w;
    w = wmax;
    while (w > 0 && big_smem_bytes(g, w) > 160 * 1024) --w;
    return w;
}

size_t big_workspace_bytes(const DevGraph& g, int num_envs) {
    int w = big_waves(g);
    size_t b = (size_t)(num_envs > 0 ? num_envs : 0);
    return b * (size_t)(w > 0 ? w : 1) * (64 / g.big_g) * fib_slot_bytes(g.N) + b * (size_t)g.E * 4;
}

template <int G>
static void launch_g(const DevGraph& g, int w, const trx_params& p, const trx_state& s, int num_envs, int mode,
                     const int32_t* action, double* reward, uint8_t* done, uint8_t* valid, const uint8_t* env_mask,
                     void* workspace, hipStream_t stream) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(env_kernel_big<G>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(env_kernel_big<G>, dim3(num_envs), dim3(w * 64), big_smem_bytes(g, w), stream, g, p, s,
                       num_envs, mode, action, reward, done, valid, env_mask, static_cast<unsigned char*>(workspace));
}

hipError_t launch_env_kernel_big(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                 const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                 const uint8_t* env_mask, void* workspace, hipStream_t stream) {
    const int w = big_waves(g);
    if (w <= 0) return hipErrorInvalidConfiguration;
    if (num_envs == 0) return hipSuccess;
    if (g.big_g == 16)
        launch_g<16>(g, w, p, s, num_envs, mode, action, reward, done, valid, env_mask, workspace, stream);
    else if (g.big_g == 32)
        launch_g<32>(g, w, p, s, num_envs, mode, action, reward, done, valid, env_mask, workspace, stream);
    else
        launch_g<64>(g, w, p, s, num_envs, mode, action, reward, done, valid, env_mask, workspace, stream);
    return hipGetLastError();
}

}  // namespace trx

// assign_quad.hip -- fused batched static traffic assignment, gfx950, v2.
//
// Same contract as assign_kernel.hip (src/env/repair_env.py:299-345, 207-237,
// 167-205), different mapping: each (env, origin) shortest-path tree is owned
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

#include "device_common.h"
#include "trx_internal.h"

namespace trx {

namespace {

constexpr int kQuad = 4;

struct SmemQ {
    float *flow, *cap, *dmg, *goal, *t, *aux, *dprev;  // [EPW*E]
    float* w;          // [EPW][NP(u)][4(j)][NP/4(i)]  cost of u -> 4i+j
    uint8_t* pred;     // [EPW*Z][NP]  per tree
    int16_t* eid;      // [NP*NP]
    float* dem;        // [Z*N]
    float* unas;       // [L]
    int* act;          // [EPW]
    double* red;       // [EPW*2]
    FibLane* heap;     // [L/64]
};

__host__ __device__ inline size_t align16q(size_t x) { return (x + 15) & ~size_t(15); }

__host__ __device__ inline size_t smemq_layout(int E, int N, int Z, int NP, int EPW, int L, SmemQ* s,
                                               unsigned char* base) {
    size_t off = 0;
    size_t el = (size_t)EPW * E * sizeof(float);
    float** arrs[7] = {s ? &s->flow : nullptr, s ? &s->cap : nullptr, s ? &s->dmg : nullptr, s ? &s->goal : nullptr,
                       s ? &s->t : nullptr,    s ? &s->aux : nullptr, s ? &s->dprev : nullptr};
    for (int i = 0; i < 7; ++i) {
        if (s) *arrs[i] = (float*)(base + off);
        off = align16q(off + el);
    }
    if (s) s->w = (float*)(base + off);
    off = align16q(off + (size_t)EPW * NP * NP * sizeof(float));
    if (s) s->pred = base + off;
    off = align16q(off + (size_t)EPW * Z * NP);
    if (s) s->eid = (int16_t*)(base + off);
    off = align16q(off + (size_t)NP * NP * sizeof(int16_t));
    if (s) s->dem = (float*)(base + off);
    off = align16q(off + (size_t)Z * N * sizeof(float));
    if (s) s->unas = (float*)(base + off);
    off = align16q(off + (size_t)L * sizeof(float));
    if (s) s->act = (int*)(base + off);
    off = align16q(off + (size_t)EPW * sizeof(int));
    if (s) s->red = (double*)(base + off);
    off = align16q(off + (size_t)EPW * 2 * sizeof(double));
    if (s) s->heap = (FibLane*)(base + off);
    off = align16q(off + (size_t)((L + 63) / 64) * sizeof(FibLane));
    return off;
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

template <int NP>
__global__ void __launch_bounds__(512) env_kernel_q(const DevGraph g, const trx_params p, const trx_state s, int B,
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
    SmemQ S;
    smemq_layout(E, N, Z, NP, EPW, L, &S, smem_raw);

    // ------------------------------------------------ per-env activation
    if (tid < EPW) {
        int gb = env0 + tid;
        int active = 0;
        if (gb < B) {
            if (mode == kModeStep) {
                int a = action[gb];
                active = s.damaged[(size_t)gb * E + a] != 0.0f;  // repair_env.py:210
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
    for (int i = tid; i < Z * N; i += L) S.dem[i] = g.dem[i];
    __syncthreads();

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
        S.t[i] = S.act[el] ? bpr_cost(fl, cp, g.t0[e], dm, p.bpr_alpha, p.bpr_beta) : 0.0f;
    }
    __syncthreads();

    // thread -> (tree = (env, origin zone), lane j of its quad)
    const int tree = tid / kQuad;
    const int j = tid & (kQuad - 1);
    const int lenv = tree / Z;
    const int zi = tree - lenv * Z;
    const bool tree_on = (lenv < EPW) && S.act[lenv];
    const int origin = tree_on ? g.origins[zi] : 0;
    float unassigned_lane = 0.0f;

    for (int it = 0; it < p.iters; ++it) {
        // ---------------- per-env cost rows in quad layout (LDS)
        for (int x = tid; x < EPW * NP * NP; x += L) {
            int el = x / (NP * NP), r = x - el * NP * NP;
            int u = r / NP, c = r - u * NP;  // c = jj * NPL + ii  ->  v = 4*ii + jj
            int v = kQuad * (c % NPL) + c / NPL;
            int e = S.eid[u * NP + v];
            S.w[x] = e >= 0 ? S.t[el * E + e] : kInfF;
        }
        __syncthreads();

        // ---------------- shortest-path tree per quad
        double d[NPL];
        bool amb_tree = false;
        if (tree_on) {
            const float* Wl = S.w + lenv * NP * NP;
            uint32_t info[NPL];  // pred | level << 8
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                d[i] = (kQuad * i + j == origin) ? 0.0 : kInfD;
                info[i] = kNoPred;
            }
            uint32_t scanned = 0u, amb = 0u, lev = 0u;
            double last = -1.0;
            for (int k = 0; k < N; ++k) {
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
                if (best > last) {
                    ++lev;
                    last = best;
                }
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
#pragma unroll
                for (int i = 0; i < NPL; ++i) {
                    double nd = __dadd_rn(best, (double)wv[i]);
                    bool uns = !((scanned >> i) & 1u) && (wv[i] < kInfF);
                    bool better = uns && nd < d[i];
                    bool tie = uns && !better && nd == d[i] && ((info[i] >> 8) == lev);
                    d[i] = better ? nd : d[i];
                    info[i] = better ? ((uint32_t)u | (lev << 8)) : info[i];
                    amb = better ? (amb & ~(1u << i)) : (tie ? (amb | (1u << i)) : amb);
                }
            }
            uint8_t* pr = S.pred + tree * NP;
#pragma unroll
            for (int i = 0; i < NPL; ++i) pr[kQuad * i + j] = (uint8_t)(info[i] & 0xFF);
            int a = amb != 0u;
            a |= qperm<0xB1>(a);
            a |= qperm<0x4E>(a);
            amb_tree = a != 0;
        }
        {
            // trees whose predecessor choice depends on scipy's heap order are
            // replayed exactly, one at a time per wave, by the quad's lane 0
            uint64_t pending = __ballot(tree_on && amb_tree && j == 0);
            FibLane* h = S.heap + (tid >> 6);
            while (pending) {
                int leader = __ffsll((unsigned long long)pending) - 1;
                if ((tid & 63) == leader) {
                    const float* Wl = S.w + lenv * NP * NP;
                    exact_sssp(
                        g, [&](int a_, int b_) { return Wl[a_ * NP + (b_ & 3) * NPL + (b_ >> 2)]; }, origin, h,
                        nullptr, S.pred + tree * NP, 1, 0);
                }
                pending &= pending - 1;
            }
        }
        __syncthreads();

        // ---------------- all-or-nothing: walk predecessor paths (repair_env.py:495-502)
        if (tree_on) {
            const uint8_t* pr = S.pred + tree * NP;
            const float* dm = S.dem + zi * N;
            float* aux = S.aux + lenv * E;
            float un = 0.0f;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int v = kQuad * i + j;
                if (v < N) {
                    float dv = dm[v];
                    bool reach = d[i] < kInfD && v != origin;
                    un += reach ? 0.0f : dv;  // unreachable or intrazonal (repair_env.py:708)
                    if (reach && dv != 0.0f) {
                        int cur = v;
                        for (int hop = 0; hop < N && cur != origin; ++hop) {
                            int pu = pr[cur];
                            atomicAdd(&aux[S.eid[pu * NP + cur]], dv);
                            cur = pu;
                        }
                    }
                }
            }
            unassigned_lane = un;
        }
        __syncthreads();

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
            S.t[i] = bpr_cost(nf, S.cap[i], g.t0[e], S.dmg[i], p.bpr_alpha, p.bpr_beta);
        }
        __syncthreads();
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
}

LaunchCfg quad_launch_cfg(const DevGraph& g, int num_envs) {
    LaunchCfg c{};
    c.np = g.NP;
    // envs per workgroup: fill up to 512 threads with whole envs (Z quads each)
    int per_env = g.Z * kQuad;
    int epw = 512 / per_env;
    if (epw < 1) epw = 1;
    if (epw > 4) epw = 4;  // 384 threads for SF: ~28 KB LDS, 5 workgroups/CU
    c.epw = epw;
    c.threads = ((epw * per_env + 63) / 64) * 64;
    c.smem = smemq_layout(g.E, g.N, g.Z, c.np, c.epw, c.threads, nullptr, nullptr);
    c.blocks = (num_envs + c.epw - 1) / c.epw;
    return c;
}

hipError_t launch_env_kernel_quad(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                  const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                  const uint8_t* env_mask, hipStream_t stream) {
    LaunchCfg c = quad_launch_cfg(g, num_envs);
    if (c.blocks == 0) return hipSuccess;
    if (c.threads > 512) return hipErrorInvalidConfiguration;
    dim3 grid(c.blocks), block(c.threads);
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

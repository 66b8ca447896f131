// assign_big.hip -- fused batched static traffic assignment for networks larger
// than the register-resident kernel takes (N > 32: Anaheim-sized, SURVEY.md
// §8(d) config #5), gfx950.
//
// Same contract as assign_quad.hip (src/env/repair_env.py:299-345 assignment,
// 207-237 step, 167-205 reset, 724-735 TSTT, 244-294 reward): one workgroup
// per env, the env's link arrays resident in LDS for the whole call, HBM
// touched only at the start and the end.  Each wave owns one shortest-path
// tree (env, origin zone) at a time:
//
//   labels   pull-based Bellman-Ford in float64 over LDS.  Node v is owned by
//            one lane; each lane walks its packed in-link list (nodes dealt to
//            lanes in contiguous chunks of a DFS order, so a sweep carries a
//            label along a whole chunk -- Gauss-Seidel inside the lane) and the
//            sweep direction alternates.  Rounded addition is monotone and
//            costs are > 0, so the least fixed point of
//                d[v] = min_u fl(d[u] + w(u,v)),  d[origin] = 0
//            is exactly the label set scipy's Dijkstra computes, whatever the
//            relaxation order.
//   preds    scipy records for v the first scanned tail achieving d[v], i.e.
//            the achieving tail with the smallest label.  A post pass picks it;
//            if two achieving tails share that label the heap order decides,
//            and the tree is replayed with the exact scipy Fibonacci heap
//            (device_common.h, per-wave scratch in the caller's workspace).
//   AON      the wave's lanes walk the tree's OD destinations back to the
//            origin by predecessor link and add the demand with LDS float
//            atomics: exact in any order (integral demands, total < 2^24).
//
// Algorithmic bytes per assignment: SURVEY.md §8(d) (bench.py roofline).
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "trx_internal.h"

namespace trx {

namespace {

constexpr int kBigMaxWaves = 8;

struct SmemB {
    uint32_t flow, cap, dmg, goal, t, aux, dprev;  // [E] f32
    uint32_t ent;                                  // [KMAX*64] uint2 {packed entry, weight bits}
    uint32_t lnk;                                  // [KMAX*64] i16 link id
    uint32_t lsrc;                                 // [E] i16 tail node of each link
    uint32_t dist;                                 // [W][N] f64 labels of the wave's tree
    uint32_t pe;                                   // [W][N] i16 predecessor link
    uint32_t unas;                                 // [W*64] f32
    uint32_t red;                                  // [2] f64
    uint32_t act;                                  // [1] i32
    uint32_t total;
};

__host__ __device__ inline uint32_t align16b(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline SmemB smemb_layout(int E, int N, int KMAX, int W) {
    SmemB o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t bytes) {
        uint32_t r = off;
        off = align16b(off + bytes);
        return r;
    };
    const uint32_t el = (uint32_t)(E * 4);
    o.flow = take(el);
    o.cap = take(el);
    o.dmg = take(el);
    o.goal = take(el);
    o.t = take(el);
    o.aux = take(el);
    o.dprev = take(el);
    o.ent = take((uint32_t)(KMAX * kBigLanes * 8));
    o.lnk = take((uint32_t)(KMAX * kBigLanes * 2));
    o.lsrc = take((uint32_t)(E * 2));
    o.dist = take((uint32_t)(W * N * 8));
    o.pe = take((uint32_t)(W * N * 2));
    o.unas = take((uint32_t)(W * 64 * 4));
    o.red = take(16);
    o.act = take(16);
    o.total = off;
    return o;
}

// per-wave FibBig scratch: val f64 | parent,left,right,child i16 | rank,state u8 | roots i16[32]
__host__ __device__ inline size_t fib_slot_bytes(int N) {
    size_t n = (size_t)((N + 7) & ~7);
    return ((n * 8 + n * 2 * 4 + n * 2 + 64) + 255) & ~(size_t)255;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

__global__ void __launch_bounds__(512) env_kernel_big(const DevGraph g, const trx_params p, const trx_state s, int B,
                                                      int mode, const int32_t* __restrict__ action,
                                                      double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                      uint8_t* __restrict__ valid_out,
                                                      const uint8_t* __restrict__ env_mask,
                                                      unsigned char* __restrict__ ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N, Z = g.Z, KMAX = g.KMAX;
    const int tid = threadIdx.x, L = blockDim.x;
    const int W = L / 64, wave = tid >> 6, lane = tid & 63;
    const int gb = blockIdx.x;
    const SmemB O = smemb_layout(E, N, KMAX, W);
    float* flow = (float*)(smem_raw + O.flow);
    float* cap = (float*)(smem_raw + O.cap);
    float* dmg = (float*)(smem_raw + O.dmg);
    float* goal = (float*)(smem_raw + O.goal);
    float* tt = (float*)(smem_raw + O.t);
    float* aux = (float*)(smem_raw + O.aux);
    float* dprev = (float*)(smem_raw + O.dprev);
    uint2* ent = (uint2*)(smem_raw + O.ent);
    int16_t* lnk = (int16_t*)(smem_raw + O.lnk);
    int16_t* lsrc = (int16_t*)(smem_raw + O.lsrc);
    double* dist = (double*)(smem_raw + O.dist) + (size_t)wave * N;
    int16_t* pe = (int16_t*)(smem_raw + O.pe) + (size_t)wave * N;
    float* unas = (float*)(smem_raw + O.unas);
    double* red = (double*)(smem_raw + O.red);
    int* act = (int*)(smem_raw + O.act);

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
        act[0] = active;
    }
    __syncthreads();
    if (!act[0]) return;  // workgroup-uniform

    // static in-link lists + link tails; state (repair_env.py:193-198, 215-216)
    for (int i = tid; i < KMAX * kBigLanes; i += L) {
        ent[i].x = g.blist[i];
        lnk[i] = g.blink[i];
    }
    const int a_step = mode == kModeStep ? action[gb] : -1;
    for (int e = tid; e < E; e += L) {
        lsrc[e] = (int16_t)g.src[e];
        size_t gi = (size_t)gb * E + e;
        float fl = 0.f, cp, dm, gl;
        if (mode == kModeReset) {
            dm = s.damaged[gi];
            cp = dm != 0.0f ? p.capacity_damage : g.cap0[e];
            gl = dm;
        } else {
            fl = s.flow[gi];
            cp = s.capacity[gi];
            dm = s.damaged[gi];
            gl = s.goal[gi];
            if (e == a_step) {
                dm = 0.0f;
                cp = g.cap0[e];
            }
        }
        flow[e] = fl;
        cap[e] = cp;
        dmg[e] = dm;
        goal[e] = gl;
        aux[e] = 0.0f;
        dprev[e] = 0.0f;
        tt[e] = bpr_cost(fl, cp, g.t0[e], dm, p.bpr_alpha, p.bpr_beta);
    }
    __syncthreads();

    FibBig fb;
    {
        const size_t slot = fib_slot_bytes(N);
        const size_t n = (size_t)((N + 7) & ~7);
        unsigned char* base = ws + ((size_t)blockIdx.x * W + wave) * slot;
        fb.val = (double*)base;
        fb.parent = (int16_t*)(base + n * 8);
        fb.left = fb.parent + n;
        fb.right = fb.left + n;
        fb.child = fb.right + n;
        fb.rank = (uint8_t*)(fb.child + n);
        fb.state = fb.rank + n;
        fb.roots = (int16_t*)(fb.state + n);
    }

    float unassigned_lane = 0.0f;
    for (int it = 0; it < p.iters; ++it) {
        // ---------------- per-entry link costs for this iteration
        for (int i = tid; i < KMAX * kBigLanes; i += L) {
            int e = lnk[i];
            ent[i].y = __float_as_uint(e >= 0 ? tt[e] : kInfF);
        }
        __syncthreads();

        float un = 0.0f;
        for (int zi = wave; zi < Z; zi += W) {
            const int origin = g.origins[zi];
            for (int v = lane; v < N; v += 64) dist[v] = v == origin ? 0.0 : kInfD;
            wave_sync();
            // ---------------- labels: alternating pull sweeps to the fixed point
            int dir = 0;
            for (int sweep = 0; sweep <= N; ++sweep) {
                bool changed = false;
                double m = kInfD;
                for (int kk = 0; kk < KMAX; ++kk) {
                    const int k = dir ? KMAX - 1 - kk : kk;
                    const uint2 en = ent[k * kBigLanes + lane];
                    const int u = en.x & 0xFFFF;
                    double nd = __dadd_rn(dist[u], (double)__uint_as_float(en.y));
                    m = nd < m ? nd : m;
                    const bool end = dir ? ((en.x >> 30) & 1u) : (en.x >> 31);
                    if (end) {
                        const int v = (en.x >> 16) & 0x3FFF;
                        if (m < dist[v]) {  // strict improvement
                            dist[v] = m;
                            changed = true;
                        }
                        m = kInfD;
                    }
                }
                wave_sync();
                if (__ballot(changed) == 0) break;
                dir ^= 1;
            }
            // ---------------- predecessors: smallest-label achieving tail
            bool amb = false;
            {
                double mdu = kInfD;
                int cnt = 0, best = -1;
                for (int k = 0; k < KMAX; ++k) {
                    const uint2 en = ent[k * kBigLanes + lane];
                    if ((en.x >> 30) & 1u) {
                        mdu = kInfD;
                        cnt = 0;
                        best = -1;
                    }
                    const int u = en.x & 0xFFFF, v = (en.x >> 16) & 0x3FFF;
                    const double du = dist[u], dv = dist[v];
                    const double nd = __dadd_rn(du, (double)__uint_as_float(en.y));
                    if (nd == dv && dv < kInfD) {
                        if (du < mdu) {
                            mdu = du;
                            cnt = 1;
                            best = lnk[k * kBigLanes + lane];
                        } else if (du == mdu) {
                            ++cnt;
                        }
                    }
                    if (en.x >> 31) {
                        const bool real = v != origin && dv < kInfD;
                        pe[v] = (int16_t)(real ? best : -1);
                        amb |= real && cnt > 1;
                    }
                }
            }
            wave_sync();
            if (__ballot(amb) != 0) {  // equal-label tie: scipy's heap order decides
                if (lane == 0) {
                    const int32_t* ce = g.csr_eid;
                    exact_sssp_links(
                        N, g.indptr, g.indices, ce, [tt, ce](int j) { return tt[ce[j]]; }, origin, &fb, pe);
                }
                wave_sync();
            }
            // ---------------- all-or-nothing by path walks (repair_env.py:490-502, 707-722)
            for (int q = g.od_ptr[zi] + lane; q < g.od_ptr[zi + 1]; q += 64) {
                const int d = g.od_dst[q];
                const float dm = g.od_dem[q];
                if (d == origin || pe[d] < 0) {
                    un += dm;  // intrazonal or unreachable (708-709)
                    continue;
                }
                int v = d;
                for (int h = 0; h < N && v != origin; ++h) {
                    const int e = pe[v];
                    if (e < 0) break;
                    atomicAdd(&aux[e], dm);
                    v = lsrc[e];
                }
            }
            wave_sync();
        }
        unassigned_lane = un;
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
            tt[e] = bpr_cost(nf, cap[e], g.t0[e], dmg[e], p.bpr_alpha, p.bpr_beta);
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
        double base = (double)pairwise_rec<7>(aux, E);
        double td = g.total_demand > 1.0 ? g.total_demand : 1.0;
        double tstt = base / td + (un > 0 ? p.unassigned_penalty * (un / td) : 0.0);
        double prev = s.tstt[gb];
        s.tstt[gb] = tstt;
        s.unassigned[gb] = un;
        if (mode == kModeReset) s.initial_tstt[gb] = tstt;
        if (mode == kModeStep) {
            float rem = 0.0f;
            for (int e = 0; e < E; ++e) rem += __fmul_rn(goal[e], dmg[e]);
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
            s.damaged[gi] = dmg[e];
            s.goal[gi] = goal[e];
        }
    }
}

size_t big_smem_bytes(const DevGraph& g, int waves) { return smemb_layout(g.E, g.N, g.KMAX, waves).total; }

int big_waves(const DevGraph& g) {
    int w = kBigMaxWaves;
    while (w > 0 && big_smem_bytes(g, w) > 160 * 1024) --w;
    return w;
}

size_t big_workspace_bytes(const DevGraph& g, int num_envs) {
    int w = big_waves(g);
    return (size_t)(num_envs > 0 ? num_envs : 0) * (size_t)(w > 0 ? w : 1) * fib_slot_bytes(g.N);
}

hipError_t launch_env_kernel_big(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                 const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                 const uint8_t* env_mask, void* workspace, hipStream_t stream) {
    const int w = big_waves(g);
    if (w <= 0) return hipErrorInvalidConfiguration;
    if (num_envs == 0) return hipSuccess;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(env_kernel_big),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(env_kernel_big, dim3(num_envs), dim3(w * 64), big_smem_bytes(g, w), stream, g, p, s, num_envs,
                       mode, action, reward, done, valid, env_mask, static_cast<unsigned char*>(workspace));
    return hipGetLastError();
}

}  // namespace trx

// gp_kernel.hip -- path-based (gradient-projection style) assignment,
// RepairEnv(assignment_method="gp") (src/env/repair_env.py:351-419), for B
// envs of a small network (N <= 32, E <= 128) on gfx950.
//
// One workgroup per env.  Per iteration:
//   1. one lane per origin zone replays scipy's dijkstra(indices=origin)
//      exactly (Fibonacci heap, device_common.h) on the current costs;
//   2. one lane per OD key (keys grouped by origin, dict order inside an
//      origin) extracts its shortest path, appends it to the key's path set if
//      new, prices every path with numpy's float32 pairwise sum over the
//      path's links, moves gp_step of every other path's flow to the cheapest
//      (float64, first minimum), and prunes to gp_keep_paths by a stable cost
//      order with the reference's renormalisation;
//   3. one lane per link reloads the link flow from the path flows in the
//      reference's order -- keys in insertion order, paths in list order --
//      rounding each path flow to float32 before the float32 add (NEP 50), so
//      fractional path flows (gp_step != 1) match bit for bit;
//   4. BPR, then TSTT / reward / done as in the other env kernels.
// The per-env path sets (RepairEnv.od_paths / od_path_flows) persist in the
// caller's trx_state.gp rows between calls; trx_reset clears them.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "trx_internal.h"

namespace trx {

namespace {

constexpr int kGpThreads = 256;

struct SmemG {
    uint32_t flow, cap, t;  // [E] f32
    uint32_t dmg;           // [E] u8
    uint32_t eid;           // [NP*NP] i16
    uint32_t pred;          // [NP][Z] u8 (scipy predecessor node per tree)
    uint32_t heap;          // [Z] FibLane
    uint32_t keyzone;       // [P] u8
    uint32_t newf;          // [P] u8
    uint32_t pbuf;          // [kGpMaxHops][kGpThreads] u8 path scratch
    uint32_t unas;          // [kGpThreads] f32
    uint32_t misc;          // [4] i32
    uint32_t total;
};

__host__ __device__ inline uint32_t a16g(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline SmemG smemg_layout(int E, int NP, int Z, int P) {
    SmemG o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t b) {
        uint32_t r = off;
        off = a16g(off + b);
        return r;
    };
    o.flow = take(E * 4);
    o.cap = take(E * 4);
    o.t = take(E * 4);
    o.dmg = take(E);
    o.eid = take(NP * NP * 2);
    o.pred = take(NP * Z);
    o.heap = take(Z * (uint32_t)sizeof(FibLane));
    o.keyzone = take(P);
    o.newf = take(P);
    o.pbuf = take(kGpMaxHops * kGpThreads);
    o.unas = take(kGpThreads * 4);
    o.misc = take(16);
    o.total = off;
    return o;
}

// numpy pairwise_sum (float32) of t over the path's links in path order
// (_path_cost, repair_env.py:346-349: float(np.sum(t[list(path)])))
__device__ float path_cost(const uint8_t* __restrict__ edges, int n, const float* t) {
    if (n < 8) {
        float r = 0.0f;
        for (int i = 0; i < n; ++i) r = __fadd_rn(r, t[edges[i]]);
        return r;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = t[edges[j]];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], t[edges[i + j]]);
    }
    float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                          __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
    for (; i < n; ++i) res = __fadd_rn(res, t[edges[i]]);
    return res;
}

struct GpRow {  // typed views of one env's path-set row
    int32_t* nkeys;
    int16_t* ord;
    uint8_t* np;
    double* flow;  // [P][KP]
    uint4* mask;   // [P][KP]
    uint8_t* len;  // [P][KP]
    uint8_t* edges;  // [P][KP][kGpMaxHops]
};

__device__ inline GpRow gp_row(unsigned char* base, int P, int keep) {
    const GpLayout L = gp_layout(P, keep);
    GpRow r;
    r.nkeys = (int32_t*)(base + L.nkeys);
    r.ord = (int16_t*)(base + L.ord);
    r.np = base + L.np;
    r.flow = (double*)(base + L.flow);
    r.mask = (uint4*)(base + L.mask);
    r.len = base + L.len;
    r.edges = base + L.edges;
    return r;
}

__device__ inline void swap_slots(GpRow& R, int q, int KP, int a, int b) {
    if (a == b) return;
    const size_t ia = (size_t)q * KP + a, ib = (size_t)q * KP + b;
    double f = R.flow[ia];
    R.flow[ia] = R.flow[ib];
    R.flow[ib] = f;
    uint4 m = R.mask[ia];
    R.mask[ia] = R.mask[ib];
    R.mask[ib] = m;
    uint8_t l = R.len[ia];
    R.len[ia] = R.len[ib];
    R.len[ib] = l;
    uint8_t* ea = R.edges + ia * kGpMaxHops;
    uint8_t* eb = R.edges + ib * kGpMaxHops;
    for (int i = 0; i < kGpMaxHops; ++i) {
        uint8_t x = ea[i];
        ea[i] = eb[i];
        eb[i] = x;
    }
}

}  // namespace

__global__ void __launch_bounds__(kGpThreads) gp_kernel(const DevGraph g, const trx_params p, const trx_state s,
                                                        int B, int mode, const int32_t* __restrict__ action,
                                                        double* __restrict__ reward_out,
                                                        uint8_t* __restrict__ done_out,
                                                        uint8_t* __restrict__ valid_out,
                                                        const uint8_t* __restrict__ env_mask) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N, NP = g.NP, Z = g.Z, P = g.P;
    const int tid = threadIdx.x, L = blockDim.x;
    const int gb = blockIdx.x;
    const int keep = p.gp_keep_paths, KP = keep + 1;
    const SmemG O = smemg_layout(E, NP, Z, P);
    float* flow = (float*)(smem_raw + O.flow);
    float* cap = (float*)(smem_raw + O.cap);
    float* tt = (float*)(smem_raw + O.t);
    uint8_t* dmg = smem_raw + O.dmg;
    int16_t* eid = (int16_t*)(smem_raw + O.eid);
    uint8_t* pred = smem_raw + O.pred;
    FibLane* heap = (FibLane*)(smem_raw + O.heap);
    uint8_t* keyzone = smem_raw + O.keyzone;
    uint8_t* newf = smem_raw + O.newf;
    uint8_t* pbuf = smem_raw + O.pbuf;
    float* unas = (float*)(smem_raw + O.unas);
    int* misc = (int*)(smem_raw + O.misc);

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

    GpRow R = gp_row(static_cast<unsigned char*>(s.gp) + (size_t)gb * gp_layout(P, keep).total, P, keep);
    const int a_step = mode == kModeStep ? action[gb] : -1;
    for (int e = tid; e < E; e += L) {
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
        tt[e] = bpr_cost(fl, cp, g.t0[e], dm, p.bpr_alpha, p.bpr_beta);
    }
    for (int i = tid; i < NP * NP; i += L) eid[i] = g.eid_of[i];
    for (int z = tid; z < Z; z += L)
        for (int q = g.od_ptr[z]; q < g.od_ptr[z + 1]; ++q) keyzone[q] = (uint8_t)z;
    if (mode == kModeReset) {  // reset(): od_paths = {} (repair_env.py:199-200, 354-356)
        for (int q = tid; q < P; q += L) R.np[q] = 0;
        if (tid == 0) *R.nkeys = 0;
    }
    __syncthreads();

    float unassigned_lane = 0.0f;
    for (int it = 0; it < p.iters; ++it) {
        const double step = p.gp_step > 0.0 ? p.gp_step : 1.0 / (it + 1.0);
        // ---------------- 1. scipy dijkstra(indices=origin) per origin zone
        if (tid < Z) {
            const int origin = g.origins[tid];
            exact_sssp(
                N, g.indptr, g.indices, [eid, tt, NP](int a_, int b_) { return tt[eid[a_ * NP + b_]]; }, origin,
                heap + tid, nullptr, pred, Z, tid);
        }
        __syncthreads();
        // ---------------- 2. per OD key: path set update (repair_env.py:366-404)
        float un = 0.0f;
        for (int q = tid; q < P; q += L) {
            newf[q] = 0;
            const int z = keyzone[q], origin = g.origins[z], d = g.od_dst[q];
            const float dem_f = g.od_dem[q];
            const double demand = (double)dem_f;
            if (d == origin || pred[d * Z + z] == kNoPred) {
                un += dem_f;  // no path: unassigned (368-371)
                continue;
            }
            // shortest path origin -> d, links in path order + link bitmask
            int nh = 0;
            for (int v = d; v != origin && nh < kGpMaxHops; ++nh) v = pred[v * Z + z];
            uint4 mk = make_uint4(0, 0, 0, 0);
            {
                int v = d;
                for (int h = nh - 1; h >= 0; --h) {
                    const int u = pred[v * Z + z];
                    const int e = eid[u * NP + v];
                    pbuf[h * L + tid] = (uint8_t)e;
                    const uint32_t bit = 1u << (e & 31);
                    if (e < 32) mk.x |= bit;
                    else if (e < 64) mk.y |= bit;
                    else if (e < 96) mk.z |= bit;
                    else mk.w |= bit;
                    v = u;
                }
            }
            int n = R.np[q];
            if (n == 0) {  // first path of a new key: all demand on it (374-377)
                const size_t i0 = (size_t)q * KP;
                R.flow[i0] = demand;
                R.mask[i0] = mk;
                R.len[i0] = (uint8_t)nh;
                for (int h = 0; h < nh; ++h) R.edges[i0 * kGpMaxHops + h] = pbuf[h * L + tid];
                R.np[q] = 1;
                newf[q] = 1;
                continue;
            }
            bool found = false;
            for (int i = 0; i < n; ++i) {
                const uint4 m2 = R.mask[(size_t)q * KP + i];
                found |= m2.x == mk.x && m2.y == mk.y && m2.z == mk.z && m2.w == mk.w;
            }
            if (!found) {  // append with zero flow (378-380)
                const size_t ia = (size_t)q * KP + n;
                R.flow[ia] = 0.0;
                R.mask[ia] = mk;
                R.len[ia] = (uint8_t)nh;
                for (int h = 0; h < nh; ++h) R.edges[ia * kGpMaxHops + h] = pbuf[h * L + tid];
                ++n;
            }
            double cost[kGpMaxPaths];
            int best = 0;
            for (int i = 0; i < n; ++i) {
                const size_t ia = (size_t)q * KP + i;
                cost[i] = (double)path_cost(R.edges + ia * kGpMaxHops, R.len[ia], tt);
                if (cost[i] < cost[best]) best = i;  // np.argmin: first minimum
            }
            if (n > 1) {  // move step x flow of every other path to the cheapest (384-392)
                double moved = 0.0;
                for (int i = 0; i < n; ++i) {
                    if (i == best) continue;
                    double& fi = R.flow[(size_t)q * KP + i];
                    const double tr = __dmul_rn(step, fi);
                    fi = __dsub_rn(fi, tr);
                    moved = __dadd_rn(moved, tr);
                }
                double& fb = R.flow[(size_t)q * KP + best];
                fb = __dadd_rn(fb, moved);
            }
            if (keep > 0 && n > keep) {  // prune to the keep cheapest, renormalise (393-404)
                int idx[kGpMaxPaths];
                for (int i = 0; i < n; ++i) idx[i] = i;
                for (int i = 1; i < n; ++i) {  // stable insertion sort by cost (numpy small-n argsort)
                    const int x = idx[i];
                    int j = i - 1;
                    while (j >= 0 && cost[idx[j]] > cost[x]) {
                        idx[j + 1] = idx[j];
                        --j;
                    }
                    idx[j + 1] = x;
                }
                int where[kGpMaxPaths], at[kGpMaxPaths];  // slot of original path i / path at slot j
                for (int i = 0; i < n; ++i) where[i] = at[i] = i;
                for (int j = 0; j < keep; ++j) {
                    const int src = where[idx[j]];
                    swap_slots(R, q, KP, j, src);
                    const int pj = at[j];
                    at[src] = pj;
                    where[pj] = src;
                    at[j] = idx[j];
                    where[idx[j]] = j;
                }
                double tot = 0.0;
                for (int j = 0; j < keep; ++j) tot = __dadd_rn(tot, R.flow[(size_t)q * KP + j]);
                for (int j = 0; j < keep; ++j) {
                    double& fj = R.flow[(size_t)q * KP + j];
                    fj = tot > 0.0 ? __ddiv_rn(__dmul_rn(fj, demand), tot) : (j == 0 ? demand : 0.0);
                }
                n = keep;
            }
            R.np[q] = (uint8_t)n;
        }
        unassigned_lane = un;
        __syncthreads();
        // new keys enter the dict in (origin, dict) order
        if (tid == 0) {
            int nk = *R.nkeys;
            for (int q = 0; q < P; ++q)
                if (newf[q]) R.ord[nk++] = (int16_t)q;
            *R.nkeys = nk;
        }
        __syncthreads();
        // ---------------- 3. link flows from path flows in dict order (406-413)
        const int nkeys = *R.nkeys;
        for (int e = tid; e < E; e += L) {
            const uint32_t bit = 1u << (e & 31);
            float acc = 0.0f;
            for (int k = 0; k < nkeys; ++k) {
                const int q = R.ord[k];
                const int n = R.np[q];
                for (int i = 0; i < n; ++i) {
                    const size_t ia = (size_t)q * KP + i;
                    const double f = R.flow[ia];
                    if (!(f > 0.0)) continue;
                    const uint4 m = R.mask[ia];
                    const uint32_t w = e < 32 ? m.x : e < 64 ? m.y : e < 96 ? m.z : m.w;
                    if (w & bit) acc = __fadd_rn(acc, (float)f);
                }
            }
            flow[e] = acc;
            tt[e] = bpr_cost(acc, cap[e], g.t0[e], dmg[e] ? 1.0f : 0.0f, p.bpr_alpha, p.bpr_beta);
        }
        __syncthreads();
    }

    // ---------------- TSTT, reward, done (repair_env.py:724-735, 220-236)
    unas[tid] = unassigned_lane;
    float* prod = (float*)(smem_raw + O.pbuf);  // path scratch is free now (>= E floats)
    for (int e = tid; e < E; e += L) prod[e] = __fmul_rn(flow[e], tt[e]);
    __syncthreads();
    if (tid == 0) {
        double un = 0.0;
        for (int x = 0; x < L; ++x) un += (double)unas[x];
        double base = (double)pairwise_sum(prod, E);
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

hipError_t launch_gp_kernel(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                            const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                            const uint8_t* env_mask, hipStream_t stream) {
    if (num_envs == 0) return hipSuccess;
    const size_t smem = smemg_layout(g.E, g.NP, g.Z, g.P).total;
    if (smem > 160 * 1024) return hipErrorInvalidConfiguration;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gp_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(gp_kernel, dim3(num_envs), dim3(kGpThreads), smem, stream, g, p, s, num_envs, mode, action,
                       reward, done, valid, env_mask);
    return hipGetLastError();
}

}  // namespace trx

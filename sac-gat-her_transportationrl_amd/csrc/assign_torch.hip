// assign_torch.hip -- the reference's configured shortest-path rule
// (sp_backend="torch": src/env/repair_env.py:520-573) as its own kernel, one
// env per wavefront.
//
// _all_or_nothing_torch: float32 all-pairs Floyd-Warshall (dist = 1e12, diag
// 0, link costs; for k ascending dist = where(dist[:,k] + dist[k,:] < dist,
// ..), next_hop likewise from next_hop[:,k]), then per OD pair a next-hop walk
// of at most N hops; a walk that misses its destination leaves the demand
// unassigned, intrazonal pairs are skipped.
//
// Mapping: lane (r, c) = (lane / 8, lane % 8) owns the BS x BS block of
// dist/next_hop (BS = NP / 8) at rows BS*r.., columns BS*c.. in registers.
// Step k needs column k and row k as they stand after step k-1 (step k
// changes neither: dist[k][k] = 0); every lane fetches its BS column-k values
// (with next_hop[:, k]) from lane (r, k / BS) and its BS row-k values from
// lane (k / BS, c) with ds_bpermute, and updates its block -- no matrix and no
// store + wave sync per step (round 5: 0.98 -> 0.80 ms per 4096-env MSA-30
// step with the k loop unrolled by BS, so the owners' column / row is a fixed
// register, and three walks in flight per lane).
// The walks then run over a [NP][NP] table of (next hop | link id << 8) and
// add the integer demand with LDS atomics (exact: integral demands, total <
// 2^24); a failed walk subtracts what it added.
#include <hip/hip_runtime.h>

#include <cmath>

#include "device_common.h"
#include "trx_internal.h"

namespace trx {

namespace {


constexpr int kRep = 8;  // copies of the link-load array the walks add into

struct SmemT {
    uint32_t flow, cap, dmg, goal, t, aux, dprev;  // [E] f32
    uint32_t he;                                   // [NP*NP] u16: next hop | link id << 8 (0xFFFF: none)
    uint32_t red;                                  // [2] f64 (CFW)
    uint32_t od;                                   // [P] u16 origin | destination << 8 (demands: global)
    uint32_t rep;                                  // [kRep][E | 1] u32 link-load copies (integral demands)
    uint32_t total;
};

__host__ __device__ inline uint32_t al16t(uint32_t x) { return (x + 15u) & ~15u; }

// LDS per env is what limits residency (one wave per workgroup): the link-id
// table and the OD demands are read from the graph in global memory (cached;
// once per iteration / walk), OD entries are u16, the CFW direction is
// allocated only for CFW.
__host__ __device__ inline SmemT smemt_layout(int E, int NP, int P, bool cfw) {
    SmemT o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t bytes) {
        const uint32_t r = off;
        off = al16t(off + bytes);
        return r;
    };
    const uint32_t el = (uint32_t)E * 4u;
    o.flow = take(el);
    o.cap = take(el);
    o.dmg = take(el);
    o.goal = take(el);
    o.t = take(el);
    o.aux = take(el);
    o.dprev = take(cfw ? el : 0u);
    o.he = take((uint32_t)(NP * NP * 2));
    o.red = take(16u);
    o.od = take((uint32_t)P * 2u);
    o.rep = take((uint32_t)(kRep * (E | 1)) * 4u);
    o.total = off;
    return o;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

bool torch_kernel_ok(const DevGraph& g) {
    return g.N <= kSmallMaxNodes && g.E <= 255 && g.NP % 8 == 0 && smemt_layout(g.E, g.NP, g.P, true).total <= 64 * 1024;
}

template <int NP>
__global__ void __launch_bounds__(64) env_kernel_t(const DevGraph g, const trx_params p, const trx_state s, int B,
                                                   int P, int mode, const int32_t* __restrict__ action,
                                                   double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                   uint8_t* __restrict__ valid_out,
                                                   const uint8_t* __restrict__ env_mask) {
    constexpr int BS = NP / 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N;
    const int lane = threadIdx.x;
    const int gb = blockIdx.x;
    if (gb >= B) return;
    const bool cfw = p.method == TRX_METHOD_CFW;
    const SmemT O = smemt_layout(E, NP, P, cfw);
    float* const sflow = (float*)(smem_raw + O.flow);
    float* const scap = (float*)(smem_raw + O.cap);
    float* const sdmg = (float*)(smem_raw + O.dmg);
    float* const sgoal = (float*)(smem_raw + O.goal);
    float* const st = (float*)(smem_raw + O.t);
    float* const saux = (float*)(smem_raw + O.aux);
    float* const sdprev = (float*)(smem_raw + O.dprev);
    uint16_t* const she = (uint16_t*)(smem_raw + O.he);
    const int16_t* const geid = g.eid_of;  // [NP*NP] link id of (u, v), -1: none (global, cached)
    double* const sred = (double*)(smem_raw + O.red);
    uint16_t* const sod = (uint16_t*)(smem_raw + O.od);
    uint32_t* const srep = (uint32_t*)(smem_raw + O.rep);
    const int EP = E | 1;  // odd row stride: a link's copies sit in different banks

    // ------------------------------------------------ activation (wave-uniform)
    int active;
    if (mode == kModeStep) {
        const int a = action[gb];
        // out-of-range ids (check=False) are memory-safe no-ops, like an already-repaired link (208-212)
        active = (unsigned)a < (unsigned)E && s.damaged[(size_t)gb * E + a] != 0.0f;
        if (!active) {
            if (lane == 0) {
                reward_out[gb] = -1.0;
                done_out[gb] = 0;
                valid_out[gb] = 0;
            }
            return;
        }
    } else {
        active = env_mask ? (env_mask[gb] != 0) : 1;
        if (!active) return;
    }

    // ------------------------------------------------------- load state
    const int act_e = mode == kModeStep ? action[gb] : -1;
    for (int e = lane; e < E; e += 64) {
        const size_t gi = (size_t)gb * E + e;
        float fl = 0.f, cp, dm, gl;
        if (mode == kModeReset) {
            dm = s.damaged[gi];  // repair_env.py:193-198
            cp = dm != 0.0f ? p.capacity_damage : g.cap0[e];
            gl = dm;
        } else {
            fl = s.flow[gi];
            cp = s.capacity[gi];
            dm = s.damaged[gi];
            gl = s.goal[gi];
            if (e == act_e) {  // repair_env.py:215-216
                dm = 0.0f;
                cp = g.cap0[e];
            }
        }
        sflow[e] = fl;
        scap[e] = cp;
        sdmg[e] = dm;
        sgoal[e] = gl;
        saux[e] = 0.0f;
        if (cfw) sdprev[e] = 0.0f;
        st[e] = bpr_cost(fl, cp, g.t0[e], dm, p.bpr_alpha, p.bpr_beta);
    }
    // OD entries (origin | destination << 8, demand), zone-major (od_ptr)
    for (int zi = 0; zi < g.Z; ++zi) {
        const int q0 = g.od_ptr[zi], q1 = g.od_ptr[zi + 1], o = g.origins[zi];
        for (int q = q0 + lane; q < q1; q += 64) {
            sod[q] = (uint16_t)(o | (g.od_dst[q] << 8));
        }
    }
    wave_sync();

    const int r = lane >> 3, c = lane & 7;
    float unassigned_lane = 0.0f;
    for (int it = 0; it < p.iters; ++it) {
        // ---------------- Floyd-Warshall (repair_env.py:524-542)
        float d[BS][BS];
        uint32_t h[BS][BS];
#pragma unroll
        for (int a = 0; a < BS; ++a)
#pragma unroll
            for (int b = 0; b < BS; ++b) {
                const int i = BS * r + a, j = BS * c + b;
                const int e = geid[i * NP + j];
                // dist = 1e12, diag 0, then dist[row, col] = t per link (524-535); padding never improves
                d[a][b] = e >= 0 ? st[e] : (i == j ? 0.0f : 1e12f);
                h[a][b] = e >= 0 ? (uint32_t)j : 0xFFu;
            }
        // step k = BS * kb + ks, ks unrolled: the owners' column / row ks is a fixed register
        for (int kb = 0; kb * BS < N; ++kb) {
#pragma unroll
            for (int ks = 0; ks < BS; ++ks) {
                if (kb * BS + ks >= N) break;  // wave-uniform
                // column k (with next_hop[:, k]) and row k as they are after step k-1, straight
                // from their owners' registers: lane (r, kb) holds column k of rows BS*r..,
                // lane (kb, c) row k of columns BS*c.. (ds_bpermute: no LDS store + wave sync)
                const int src_col = (r * 8 + kb) * 4, src_row = (kb * 8 + c) * 4;
                float ck[BS], rk[BS];
                uint32_t hk[BS];
#pragma unroll
                for (int a = 0; a < BS; ++a) {
                    ck[a] = __int_as_float(__builtin_amdgcn_ds_bpermute(src_col, __float_as_int(d[a][ks])));
                    hk[a] = (uint32_t)__builtin_amdgcn_ds_bpermute(src_col, (int)h[a][ks]);
                }
#pragma unroll
                for (int b = 0; b < BS; ++b)
                    rk[b] = __int_as_float(__builtin_amdgcn_ds_bpermute(src_row, __float_as_int(d[ks][b])));
#pragma unroll
                for (int a = 0; a < BS; ++a)
#pragma unroll
                    for (int b = 0; b < BS; ++b) {
                        const float alt = __fadd_rn(ck[a], rk[b]);
                        const bool better = alt < d[a][b];  // strict <
                        d[a][b] = better ? alt : d[a][b];
                        h[a][b] = better ? hk[a] : h[a][b];
                    }
            }
        }
        // ---------------- next-hop table with the link ids of the hops
#pragma unroll
        for (int a = 0; a < BS; ++a)
#pragma unroll
            for (int b = 0; b < BS; ++b) {
                const int i = BS * r + a, j = BS * c + b;
                const uint32_t hv = h[a][b];
                she[i * NP + j] = hv == 0xFFu ? (uint16_t)0xFFFF : (uint16_t)(hv | ((uint32_t)geid[i * NP + hv] << 8));
            }
        wave_sync();
        // ---------------- next_hop walks (repair_env.py:548-568)
        // Each lane walks two OD pairs at a time (independent LDS chains in
        // flight) and adds into one of kRep copies of the link loads (fewer
        // lanes on one address per atomic); the copies are summed afterwards
        // (integers: exact in any order).
        for (int x = lane; x < kRep * EP; x += 64) srep[x] = 0u;
        wave_sync();
        uint32_t* const myrep = srep + (lane & (kRep - 1)) * EP;
        float un = 0.0f;
        constexpr int WW = 3;  // independent walks in flight per lane (2: +2 %, 4: +15 % step time)
        for (int q = lane; q < P; q += 64 * WW) {
            int o[WW], dd[WW], cu[WW], hop[WW];
            uint32_t m[WW];  // integral demands: u32 atomics (native, exact)
            bool live[WW], run[WW];
#pragma unroll
            for (int w = 0; w < WW; ++w) {
                const int qi = q + 64 * w;
                o[w] = dd[w] = 0;
                m[w] = 0;
                if (qi < P) {
                    const uint32_t odm = sod[qi];
                    o[w] = odm & 0xFF;
                    dd[w] = (odm >> 8) & 0xFF;
                    m[w] = (uint32_t)g.od_dem[qi];  // zone-major like sod (global, cached)
                }
                live[w] = qi < P && o[w] != dd[w];  // origin == dest: skipped (551-552)
                cu[w] = o[w];
                hop[w] = 0;
                run[w] = live[w];
            }
            for (;;) {
                bool any = false;
#pragma unroll
                for (int w = 0; w < WW; ++w) any |= run[w];
                if (!any) break;
                uint32_t hv[WW];
#pragma unroll
                for (int w = 0; w < WW; ++w) hv[w] = run[w] ? (uint32_t)she[cu[w] * NP + dd[w]] : 0u;
#pragma unroll
                for (int w = 0; w < WW; ++w) {
                    if (run[w]) {
                        if (hv[w] == 0xFFFFu) {
                            run[w] = false;
                        } else {
                            atomicAdd(&myrep[hv[w] >> 8], m[w]);
                            cu[w] = hv[w] & 0xFF;
                            ++hop[w];
                            run[w] = cu[w] != dd[w] && hop[w] < N;
                        }
                    }
                }
            }
            // a walk that missed its destination: unassigned, partial path dropped (564-566)
#pragma unroll
            for (int w = 0; w < WW; ++w) {
                if (live[w] && cu[w] != dd[w]) {
                    un += (float)m[w];
                    int c2 = o[w];
                    for (int t2 = 0; t2 < hop[w]; ++t2) {
                        const uint32_t h2 = she[c2 * NP + dd[w]];
                        atomicAdd(&myrep[h2 >> 8], 0u - m[w]);
                        c2 = h2 & 0xFF;
                    }
                }
            }
        }
        unassigned_lane = un;
        wave_sync();
        for (int e = lane; e < E; e += 64) {
            uint32_t ax = 0;
#pragma unroll
            for (int rr = 0; rr < kRep; ++rr) ax += srep[rr * EP + e];
            saux[e] = (float)ax;  // exact: < 2^24
        }
        wave_sync();

        // ---------------- flow update + BPR (repair_env.py:317-342)
        if (cfw) {
            if (lane == 0) {
                double num = 0.0, den = 0.0;
                for (int e = 0; e < E; ++e) {
                    const float dfw = __fsub_rn(saux[e], sflow[e]);
                    num += (double)__fmul_rn(dfw, __fsub_rn(dfw, sdprev[e]));
                    den += (double)__fmul_rn(sdprev[e], sdprev[e]);
                }
                sred[0] = num;
                sred[1] = den;
            }
            wave_sync();
        }
        const double stepd = (p.method == TRX_METHOD_MSA) ? 1.0 / (it + 1.0) : 2.0 / (it + 2.0);
        const float s32 = (float)stepd, om32 = (float)(1.0 - stepd);
        for (int e = lane; e < E; e += 64) {
            const float fl = sflow[e];
            const float ax = saux[e];
            float nf;
            if (cfw) {
                const float dfw = __fsub_rn(ax, fl);
                float dir;
                if (it == 0) {
                    dir = dfw;
                } else {
                    const float num = (float)sred[0];
                    const double den = (double)(float)sred[1] + 1e-12;
                    double bb = (double)num / den;
                    bb = bb < 0.0 ? 0.0 : bb;
                    dir = __fadd_rn(dfw, __fmul_rn((float)bb, sdprev[e]));
                }
                nf = __fadd_rn(fl, __fmul_rn(s32, dir));
                nf = nf > 0.0f ? nf : 0.0f;
                sdprev[e] = dir;
            } else {
                nf = __fadd_rn(__fmul_rn(om32, fl), __fmul_rn(s32, ax));
            }
            if (nf != nf) nf = 0.0f;  // nan_to_num guard (repair_env.py:338-340)
            sflow[e] = nf;
            saux[e] = 0.0f;
            st[e] = bpr_cost(nf, scap[e], g.t0[e], sdmg[e], p.bpr_alpha, p.bpr_beta);
        }
        wave_sync();
    }

    // ---------------- TSTT (repair_env.py:724-735), reward, store
    double un = (double)unassigned_lane;  // integers: exact in any order
    for (int o = 32; o > 0; o >>= 1) un += __shfl_xor(un, o);
    for (int e = lane; e < E; e += 64) saux[e] = __fmul_rn(sflow[e], st[e]);
    wave_sync();
    if (lane == 0) {
        const double base = (double)pairwise_sum(saux, E);
        const double td = g.total_demand > 1.0 ? g.total_demand : 1.0;
        const double tstt = base / td + (un > 0 ? p.unassigned_penalty * (un / td) : 0.0);
        const double prev = s.tstt[gb];
        s.tstt[gb] = tstt;
        s.unassigned[gb] = un;
        if (mode == kModeReset) s.initial_tstt[gb] = tstt;
        if (mode == kModeStep) {
            float rem = 0.0f;
            for (int e = 0; e < E; ++e) rem += __fmul_rn(sgoal[e], sdmg[e]);
            const bool complete = rem == 0.0f;  // is_goal_complete (293-294)
            reward_out[gb] = reward_fn(p, prev, tstt, s.initial_tstt[gb], complete);
            done_out[gb] = complete ? 1 : 0;
            valid_out[gb] = 1;
        }
    }
    for (int e = lane; e < E; e += 64) {
        const size_t gi = (size_t)gb * E + e;
        s.flow[gi] = sflow[e];
        if (s.t) s.t[gi] = st[e];
        if (mode != kModeAssign) {
            s.capacity[gi] = scap[e];
            s.damaged[gi] = sdmg[e];
            s.goal[gi] = sgoal[e];
        }
    }
}

hipError_t launch_env_kernel_torch(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                   const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                   const uint8_t* env_mask, hipStream_t stream) {
    if (num_envs <= 0) return hipSuccess;
    const int num_od = g.P;
    const size_t smem = smemt_layout(g.E, g.NP, num_od, p.method == TRX_METHOD_CFW).total;
    const dim3 grid(num_envs), block(64);
    switch (g.NP) {
        case 8:
            hipLaunchKernelGGL(env_kernel_t<8>, grid, block, smem, stream, g, p, s, num_envs, num_od, mode, action,
                               reward, done, valid, env_mask);
            break;
        case 16:
            hipLaunchKernelGGL(env_kernel_t<16>, grid, block, smem, stream, g, p, s, num_envs, num_od, mode, action,
                               reward, done, valid, env_mask);
            break;
        case 24:
            hipLaunchKernelGGL(env_kernel_t<24>, grid, block, smem, stream, g, p, s, num_envs, num_od, mode, action,
                               reward, done, valid, env_mask);
            break;
        case 32:
            hipLaunchKernelGGL(env_kernel_t<32>, grid, block, smem, stream, g, p, s, num_envs, num_od, mode, action,
                               reward, done, valid, env_mask);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace trx

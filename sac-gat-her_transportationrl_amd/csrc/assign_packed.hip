// assign_packed.hip -- fused batched static traffic assignment, gfx950, v3
// ("packed-key" kernel).  Same contract as assign_quad.hip's env_kernel_q
// (src/env/repair_env.py:167-205 reset, 207-237 step, 299-345 assignment,
// scipy branch of _all_or_nothing 481-503 + 707-722, compute_tstt 724-735),
// same quad-of-lanes Dijkstra, rebuilt around one exactness property:
//
//   Every path label is an EXACT float64 sum of float32 link costs.
//   Costs are >= t_min > 0 (BPR only raises t0; damaged links cost 1e6), so
//   each cost is a multiple of g = ulp(t_min) and every label is a multiple of
//   g below (N-1)*t_max.  When (N-1)*t_max < 2^(log2 g + 48) -- checked on the
//   host per launch (packed_ok below; Sioux Falls: g = 2^-22, bound 2.3e7 <
//   2^26) -- a label's float64 mantissa ends in >= 5 zero bits.
//
// Consequences used here:
//  * the node id rides in those 5 low bits: key = bits(label) | id is one u64
//    whose unsigned order is (label, id) order, so the Dijkstra argmin and the
//    DPP quad reduction are single 64-bit compares, branch-free;
//  * a scanned node gets the key's sign bit: as u64 it is never the minimum
//    again, as i64 it is never improved (relaxation compares signed);
//  * labels are order-independent exact sums, so a shortest-path tie needs two
//    in-links of one node with bit-identical costs and equal tail labels: the
//    per-env list of such "tie candidate" link pairs (costs compared once per
//    iteration) decides which trees need scipy's heap-order replay, instead of
//    a post-pass over every in-link of every tree with labels staged in LDS;
//  * AON loading walks each destination's predecessor chain (preds in LDS) and
//    adds the integer demand with LDS float atomics (exact, order-free).
// Barriers per MSA/FW iteration: 3 (Dijkstra+AON | flow update+BPR+costs | tie candidates).
#include <hip/hip_runtime.h>

#include <cmath>

#include "device_common.h"
#include "trx_internal.h"

#ifdef TRX_PHASE_STAMPS
// Diagnostic build only (make stamps): per-phase cycle totals of thread 0 of
// each workgroup.  Never compiled into the shipped library.
__device__ unsigned long long trx_phase_cycles_p[8];
#define TRX_PSTAMP(slot)                                                    \
    do {                                                                    \
        if (threadIdx.x == 0) {                                             \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
            atomicAdd(&trx_phase_cycles_p[slot], now_ - stamp_prev_);        \
            stamp_prev_ = now_;                                             \
        }                                                                   \
    } while (0)
extern "C" int trx_debug_phase_cycles_p(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_phase_cycles_p), sizeof(unsigned long long) * 8) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(trx_phase_cycles_p), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define TRX_PSTAMP(slot) \
    do {                 \
    } while (0)
#endif

#ifndef TRX_PACKED_WAVES
#define TRX_PACKED_WAVES 6  // waves/SIMD the register budget targets (A/B builds override)
#endif

namespace trx {

namespace {

constexpr int kQ = 4;
constexpr uint64_t kInfKey = 0x7FF0000000000000ull;  // bits(+inf): unreached
constexpr uint32_t kSign = 0x80000000u;

struct SmemP {
    uint32_t flow, cap, dmg, goal, t, aux, dprev;  // [EPW*E] f32 (dprev: CFW only)
    uint32_t w;      // [EPW][NP(u)][4(j)][NP/4(i)] f32: cost of u -> 4i+j
    uint32_t pred;   // [EPW*Z][NP] u16 per tree: pred node | in-link id << 5 (0xFFFF: none)
    uint32_t ord;    // [EPW*Z][NP] u8 scan order per tree
    uint32_t sacc;   // [EPW*Z][NP] f32 subtree demand per tree
    uint32_t eid;    // [NP*NP] u8 link id of (u, v) (0xFF: none; the packed kernel takes E <= 255)
    uint32_t dem;    // [Z*N] f32
    uint32_t t0;     // [E] f32
    uint32_t ldst;   // [E] u8 head node of each link
    uint32_t pairs;  // [npairs] uint2 tie-candidate link pairs {e1 | e2 << 16, u1 | u2 << 8 | v << 16}
    uint32_t cand;   // [2][EPW][CW] u32 candidate masks (double buffered)
    uint32_t unas;   // [EPW] f32
    uint32_t act;    // [EPW] i32
    uint32_t red;    // [EPW*2] f64
    uint32_t heap;   // [waves] FibLane
    uint32_t rpred;  // [waves][32] u8 predecessors of a replayed tree
    uint32_t total;
};

__host__ __device__ inline uint32_t al16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline SmemP smemp_layout(int E, int N, int Z, int NP, int EPW, int L, int npairs, bool cfw) {
    SmemP o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t bytes) {
        uint32_t r = off;
        off = al16(off + bytes);
        return r;
    };
    const uint32_t el = (uint32_t)(EPW * E * 4);
    const int CW = (npairs + 31) / 32;
    o.flow = take(el);
    o.cap = take(el);
    o.dmg = take(el);
    o.goal = take(el);
    o.t = take(el);
    o.aux = take(el);
    o.dprev = take(cfw ? el : 0u);
    o.w = take((uint32_t)(EPW * NP * NP * 4));
    o.pred = take((uint32_t)(EPW * Z * NP * 2));
    o.ord = take((uint32_t)(EPW * Z * NP));
    o.sacc = take((uint32_t)(EPW * Z * NP * 4));
    o.eid = take((uint32_t)(NP * NP));
    o.dem = take((uint32_t)(Z * N * 4));
    o.t0 = take((uint32_t)(E * 4));
    o.ldst = take((uint32_t)E);
    o.pairs = take((uint32_t)(npairs * 8));
    o.cand = take((uint32_t)(2 * EPW * CW * 4));
    o.unas = take((uint32_t)(EPW * 4));
    o.act = take((uint32_t)(EPW * 4));
    o.red = take((uint32_t)(EPW * 2 * 8));
    // the replay scratch of wave w (FibLane heap + 32 pred bytes) lives in the
    // subtree-sum rows of that wave's trees, which are filled only after it
    const uint32_t per_wave_sacc = (uint32_t)(16 * NP * 4);
    if (per_wave_sacc >= (uint32_t)sizeof(FibLane) + 32u) {
        o.heap = o.sacc;
        o.rpred = o.sacc + (uint32_t)sizeof(FibLane);
    } else {
        o.heap = take((uint32_t)(((L + 63) / 64) * sizeof(FibLane)));
        o.rpred = take((uint32_t)(((L + 63) / 64) * 32));
    }
    o.total = off;
    return o;
}

// DPP quad_perm: xor 1 = [1,0,3,2] (0xB1), xor 2 = [2,3,0,1] (0x4E)
template <int CTRL>
__device__ __forceinline__ uint32_t qp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t qp64(uint64_t x) {
    return ((uint64_t)qp<CTRL>((uint32_t)(x >> 32)) << 32) | qp<CTRL>((uint32_t)x);
}
__device__ __forceinline__ uint64_t dbits(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double bitsd(uint64_t b) { return __longlong_as_double((long long)b); }

// key of quad node slot `s` held by lane `l` of this lane's quad (s, l quad-uniform)
template <int NPL>
__device__ __forceinline__ uint64_t quad_key(const uint64_t (&key)[NPL], int s, int l) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < NPL; ++i) v = (i == s) ? key[i] : v;
    const int src = ((int)(threadIdx.x & ~3u) + l) << 2;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// The exact scipy-heap replay of one ambiguous tree (rare: kept out of line so
// the Dijkstra loop's registers are not sized for it).
template <int NP>
__device__ __noinline__ void replay_tree(int N, const int32_t* __restrict__ indptr, const int32_t* __restrict__ indices,
                                         const float* Wl, int origin, FibLane* h, uint8_t* tmp, uint16_t* pl,
                                         const uint8_t* seid, uint8_t* ol) {
    constexpr int NPL = NP / kQ;
    exact_sssp(N, indptr, indices, [Wl](int a_, int b_) { return Wl[a_ * NP + (b_ & 3) * NPL + (b_ >> 2)]; }, origin,
               h, ol, tmp, 1, 0);
    for (int v = 0; v < N; ++v) {
        const int p = tmp[v];
        pl[v] = p != kNoPred ? (uint16_t)(p | (seid[p * NP + v] << 5)) : (uint16_t)0xFFFF;
    }
}

}  // namespace

bool packed_ok(const DevGraph& g, const trx_params& p) {
    // exact-label headroom (see the file comment)
    if (!(g.min_t0 > 0.0f) || p.bpr_alpha < 0.0f || g.npairs > kMaxTiePairs || g.E > 255) return false;
    int ex = 0;
    std::frexp((double)g.min_t0, &ex);          // min_t0 = m * 2^ex, m in [0.5, 1)
    const double gran = std::ldexp(1.0, ex - 1 - 23);  // ulp of the smallest float32 cost
    const double tmax = std::fmax(1e6, (double)g.max_t0 * (1.0 + (double)p.bpr_alpha * std::pow(10.0, p.bpr_beta)));
    const double bound = (double)(g.N - 1) * tmax * 1.0001;
    return bound < std::ldexp(gran, 48);
}

template <int NP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TRX_PACKED_WAVES))) env_kernel_p(const DevGraph g, const trx_params p, const trx_state s, int B,
                                                    int EPW, int mode, const int32_t* __restrict__ action,
                                                    double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                    uint8_t* __restrict__ valid_out,
                                                    const uint8_t* __restrict__ env_mask) {
    constexpr int NPL = NP / kQ;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N, Z = g.Z;
    const int L = blockDim.x;
    const int tid = threadIdx.x;
    const int EL = EPW * E;
    const int env0 = blockIdx.x * EPW;
    const int NPR = g.npairs;
    const int CW = (NPR + 31) / 32;
    const bool cfw = p.method == TRX_METHOD_CFW;
    const SmemP O = smemp_layout(E, N, Z, NP, EPW, L, NPR, cfw);
    float* const sflow = (float*)(smem_raw + O.flow);
    float* const scap = (float*)(smem_raw + O.cap);
    float* const sdmg = (float*)(smem_raw + O.dmg);
    float* const sgoal = (float*)(smem_raw + O.goal);
    float* const st = (float*)(smem_raw + O.t);
    float* const saux = (float*)(smem_raw + O.aux);
    float* const sdprev = (float*)(smem_raw + O.dprev);
    float* const sw = (float*)(smem_raw + O.w);
    uint16_t* const spred = (uint16_t*)(smem_raw + O.pred);
    uint8_t* const sord = smem_raw + O.ord;
    float* const sacc = (float*)(smem_raw + O.sacc);
    uint8_t* const seid = smem_raw + O.eid;
    float* const sdem = (float*)(smem_raw + O.dem);
    float* const st0 = (float*)(smem_raw + O.t0);
    uint8_t* const sdst = smem_raw + O.ldst;
    uint2* const spairs = (uint2*)(smem_raw + O.pairs);
    uint32_t* const scand = (uint32_t*)(smem_raw + O.cand);
    float* const sunas = (float*)(smem_raw + O.unas);
    int* const sact = (int*)(smem_raw + O.act);
    double* const sred = (double*)(smem_raw + O.red);
#ifdef TRX_PHASE_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif

    // ------------------------------------------------ per-env activation
    if (tid < EPW) {
        const int gb = env0 + tid;
        int active = 0;
        if (gb < B) {
            if (mode == kModeStep) {
                const int a = action[gb];
                // out-of-range ids (check=False) are memory-safe no-ops, like an
                // already-repaired link (repair_env.py:208-212)
                active = (unsigned)a < (unsigned)E && s.damaged[(size_t)gb * E + a] != 0.0f;
                if (!active) {
                    reward_out[gb] = -1.0;
                    done_out[gb] = 0;
                    valid_out[gb] = 0;
                }
            } else {
                active = env_mask ? (env_mask[gb] != 0) : 1;
            }
        }
        sact[tid] = active;
        sunas[tid] = 0.0f;
    }
    for (int i = tid; i < NP * NP; i += L) seid[i] = (uint8_t)g.eid_of[i];
    int16_t* const wpos_tmp = reinterpret_cast<int16_t*>(sw);  // [E] scratch in the cost-table region
    for (int i = tid; i < E; i += L) wpos_tmp[i] = -1;
    for (int i = tid; i < Z * N; i += L) sdem[i] = g.dem[i];
    for (int i = tid; i < E; i += L) st0[i] = g.t0[i];
    for (int i = tid; i < E; i += L) sdst[i] = (uint8_t)g.dst[i];
    for (int i = tid; i < NPR; i += L) {
        const uint32_t pe = g.tie_pairs[i];
        const int e1 = pe & 0xFFFF, e2 = pe >> 16;
        spairs[i] = make_uint2(pe, (uint32_t)g.src[e1] | ((uint32_t)g.src[e2] << 8) | ((uint32_t)g.dst[e1] << 16));
    }
    for (int i = tid; i < 2 * EPW * CW; i += L) scand[i] = 0u;
    __syncthreads();
    for (int i = tid; i < NP * NP; i += L) {
        const int e = seid[i];
        if (e != 0xFF) {
            const int u = i / NP, v = i - u * NP;
            wpos_tmp[e] = (int16_t)(u * NP + (v & (kQ - 1)) * NPL + (v >> 2));
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
    for (int x = tid; x < EPW * NP * NP; x += L) sw[x] = kInfF;
    __syncthreads();

    // ------------------------------------------------------- load state
    for (int i = tid; i < EL; i += L) {
        const int el = i / E, e = i - el * E;
        const int gb = env0 + el;
        float fl = 0.f, cp = 0.f, dm = 0.f, gl = 0.f;
        if (sact[el]) {
            const size_t gi = (size_t)gb * E + e;
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
        sflow[i] = fl;
        scap[i] = cp;
        sdmg[i] = dm;
        sgoal[i] = gl;
        saux[i] = 0.0f;
        if (cfw) sdprev[i] = 0.0f;
        const float tv = sact[el] ? bpr_cost(fl, cp, st0[e], dm, p.bpr_alpha, p.bpr_beta) : 0.0f;
        st[i] = tv;
        if (wpos_reg && my_wpos >= 0) sw[my_wpos] = tv;  // EL <= L: i == tid
    }
    __syncthreads();
    if (!wpos_reg) {  // generic path: rebuild link entries from the eid table
        for (int x = tid; x < EPW * NP * NP; x += L) {
            const int el = x / (NP * NP), r = x - el * NP * NP;
            const int u = r / NP, c = r - u * NP;
            const int v = kQ * (c % NPL) + c / NPL;
            const int e = seid[u * NP + v];
            sw[x] = e != 0xFF ? st[el * E + e] : kInfF;
        }
    }
    __syncthreads();
    // tie candidates for the first iteration (buffer 0)
    for (int x = tid; x < EPW * NPR; x += L) {
        const int el = x / NPR, q = x - el * NPR;
        const uint32_t pr = spairs[q].x;
        if (st[el * E + (pr & 0xFFFF)] == st[el * E + (pr >> 16)]) atomicOr(&scand[el * CW + (q >> 5)], 1u << (q & 31));
    }
    __syncthreads();

    // thread -> (tree = (env, origin zone), lane j of its quad)
    const int tree = tid / kQ;
    const int j = tid & (kQ - 1);
    const int lenv = tree / Z;
    const int zi = tree - lenv * Z;
    const bool tree_on = (lenv < EPW) && sact[lenv];
    const int origin = tree_on ? g.origins[zi] : 0;
    float unassigned_lane = 0.0f;
    TRX_PSTAMP(0);

    for (int it = 0; it < p.iters; ++it) {
        const int cb = it & 1;  // candidate-mask buffer read this iteration
        // the other buffer was last read in the previous iteration's Dijkstra
        // phase (two barriers ago); it is filled after this iteration's update
        for (int x = tid; x < EPW * CW; x += L) scand[(cb ^ 1) * EPW * CW + x] = 0u;
        // ---------------- shortest-path tree per quad (Dijkstra on packed keys)
        if (tree_on) {
            const float* Wl = sw + lenv * NP * NP;
            uint64_t key[NPL];
            uint32_t pr[NPL];
            int jo = j;
            asm volatile("" : "+v"(jo));  // keep the key set-up inside the loop (no hoist + spill)
            uint8_t* const ol = sord + tree * NP;
            int nscan = 0;
#ifndef TRX_EXP_DIJ_REPS  // diagnostic timing builds repeat the Dijkstra (never shipped)
#define TRX_EXP_DIJ_REPS 1
#endif
            for (int rep = 0; rep < TRX_EXP_DIJ_REPS; ++rep) {
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int v = kQ * i + jo;
                key[i] = v >= N ? ~0ull : (v == origin ? (uint64_t)v : (kInfKey | (uint64_t)v));
                pr[i] = kNoPred;
            }
            for (int k = 0; k < N; ++k) {
                // argmin over the lane's slots (pairwise: short dependency chain)
                uint64_t m[NPL];
#pragma unroll
                for (int i = 0; i < NPL; ++i) m[i] = key[i];
#pragma unroll
                for (int w = 1; w < NPL; w *= 2)
#pragma unroll
                    for (int i = 0; i + w < NPL; i += 2 * w) m[i] = m[i + w] < m[i] ? m[i + w] : m[i];
                uint64_t best = m[0];
                uint64_t o = qp64<0xB1>(best);
                best = o < best ? o : best;
                o = qp64<0x4E>(best);
                best = o < best ? o : best;
                if (best >= kInfKey) break;  // quad-uniform: the rest is unreachable
                const uint32_t u = (uint32_t)best & 31u;
                ol[k] = (uint8_t)u;  // the quad's 4 lanes store the same byte
                nscan = k + 1;
                const uint32_t bh = (uint32_t)(best >> 32) | kSign;
#pragma unroll
                for (int i = 0; i < NPL; ++i)  // mark the extracted node scanned
                    key[i] = key[i] == best ? (((uint64_t)bh << 32) | (uint32_t)key[i]) : key[i];
                const double bl = bitsd(best & ~31ull);
                const float* row = Wl + u * NP + j * NPL;
                float wv[NPL];
                if constexpr (NPL % 2 == 0) {
#pragma unroll
                    for (int q = 0; q < NPL / 2; ++q) {
                        const float2 w2 = reinterpret_cast<const float2*>(row)[q];
                        wv[2 * q] = w2.x;
                        wv[2 * q + 1] = w2.y;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < NPL; ++q) wv[q] = row[q];
                }
                // strict improvement (scipy `current_node.val > next_val`)
#pragma unroll
                for (int i = 0; i < NPL; ++i) {
                    const uint64_t nk = dbits(__dadd_rn(bl, (double)wv[i])) | (uint64_t)(kQ * i + j);
                    const bool better = (int64_t)nk < (int64_t)key[i];
                    key[i] = better ? nk : key[i];
                    pr[i] = better ? u : pr[i];
                }
            }
            }  // rep
            TRX_PSTAMP(1);
            // predecessor table: pred node | id of the link pred -> v << 5
            uint16_t* pl = spred + tree * NP;
            {
                int lk[NPL];
#pragma unroll
                for (int i = 0; i < NPL; ++i) lk[i] = seid[(pr[i] & 31u) * NP + kQ * i + j];  // all reads in flight
#pragma unroll
                for (int i = 0; i < NPL; ++i)
                    pl[kQ * i + j] = pr[i] != kNoPred ? (uint16_t)(pr[i] | (lk[i] << 5)) : (uint16_t)0xFFFF;
            }
            // ---------------- tie check on the candidate link pairs of this env
            // ambiguous iff some node v has two in-links of equal cost whose
            // tails have equal labels reaching v's label (scipy's heap order
            // then picks the predecessor): replay that tree exactly.
            int amb = 0;
            const uint32_t* cm = scand + (cb * EPW + lenv) * CW;
            for (int wd = 0; wd < CW; ++wd) {
                uint32_t bits = cm[wd];
                while (bits) {  // quad-uniform (env-uniform) loop
                    const int q = wd * 32 + __ffs(bits) - 1;
                    bits &= bits - 1;
                    const uint2 pq = spairs[q];
                    const int u1 = pq.y & 31, u2 = (pq.y >> 8) & 31, v = (pq.y >> 16) & 31;
                    const uint64_t k1 = quad_key<NPL>(key, u1 >> 2, u1 & 3) & 0x7FFFFFFFFFFFFFE0ull;
                    const uint64_t k2 = quad_key<NPL>(key, u2 >> 2, u2 & 3) & 0x7FFFFFFFFFFFFFE0ull;
                    const uint64_t kv = quad_key<NPL>(key, v >> 2, v & 3) & 0x7FFFFFFFFFFFFFE0ull;
                    const double w = (double)st[lenv * E + (pq.x & 0xFFFF)];
                    amb |= k1 == k2 && kv < kInfKey && v != origin && dbits(__dadd_rn(bitsd(k1), w)) == kv;
                }
            }
            amb |= (int)qp<0xB1>((uint32_t)amb);
            amb |= (int)qp<0x4E>((uint32_t)amb);
            const uint64_t need = __ballot(amb != 0 && j == 0);
            uint64_t pending = need;
            const bool heap_in_sacc = O.heap == O.sacc;
            const uint32_t wave_off = heap_in_sacc ? (uint32_t)((tid >> 6) * 16 * NP * 4)
                                                   : (uint32_t)((tid >> 6) * sizeof(FibLane));
            FibLane* h = reinterpret_cast<FibLane*>(smem_raw + O.heap + wave_off);
            uint8_t* rp = smem_raw + O.rpred + (heap_in_sacc ? wave_off : (uint32_t)((tid >> 6) * 32));
            while (pending) {  // wave-uniform: rare
                const int leader = __ffsll((unsigned long long)pending) - 1;
                if ((tid & 63) == leader)
                    replay_tree<NP>(N, g.indptr, g.indices, Wl, origin, h, rp, pl, seid, ol);
                pending &= pending - 1;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            TRX_PSTAMP(2);
            // ---------------- all-or-nothing (repair_env.py:490-502, 707-722), part 1:
            // subtree demand sums S(v) per tree.  In reverse scan order each
            // node's sum is added to its parent's (one lane per tree, plain LDS
            // read-modify-write: no other lane touches the tree's row).  Part 2
            // (after the barrier) gathers the link loads from these rows.
            // Integral demands make every float sum exact in any order.
            const float* dm = sdem + zi * N;
            float* sa = sacc + tree * NP;
            float un = 0.0f;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int v = kQ * i + j;
                const float dv = v < N ? dm[v] : 0.0f;
                const bool reach = v < N && pr[i] != kNoPred;   // (a replayed tree keeps its reachable set)
                un += (dv > 0.0f && !(reach && v != origin)) ? dv : 0.0f;  // intrazonal or unreachable (708)
                sa[kQ * i + j] = (reach && v != origin) ? dv : 0.0f;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifndef TRX_EXP_AON_REPS  // diagnostic timing builds repeat the AON (wrong results; never shipped)
#define TRX_EXP_AON_REPS 1
#endif
            for (int rep = 0; rep < TRX_EXP_AON_REPS; ++rep)
            if (j == 0) {
                uint32_t ow[NP / 4];  // the scan order in registers
#pragma unroll
                for (int q = 0; q < NP / 4; ++q) ow[q] = reinterpret_cast<const uint32_t*>(ol)[q];
#pragma unroll
                for (int k = NP - 1; k >= 1; --k) {
                    if (k < nscan) {  // quad-uniform
                        const int v = (ow[k >> 2] >> (8 * (k & 3))) & 0xFF;
                        const int pv = pl[v] & 31u;
                        sa[pv] = sa[pv] + sa[v];
                    }
                }
            }
            unassigned_lane = un;
            TRX_PSTAMP(3);
        }
        __syncthreads();
        TRX_PSTAMP(4);

        // ---------------- flow update + BPR + next cost entries (repair_env.py:317-342)
        // ---------------- all-or-nothing, part 2: link load = the sum over the
        // env's trees whose predecessor link of dst(e) is e of S(dst(e))
        for (int i = tid; i < EL; i += L) {
            const int el = i / E, e = i - el * E;
            if (!sact[el]) continue;
            const int v = sdst[e];
            float ax = 0.0f;
            const uint16_t* pz = spred + el * Z * NP + v;
            const float* sz = sacc + el * Z * NP + v;
            for (int z = 0; z < Z; ++z) ax += (pz[z * NP] >> 5) == (uint32_t)e ? sz[z * NP] : 0.0f;
            saux[i] = ax;
        }
        if (cfw) {  // the conjugate direction needs every link's load of the env
            __syncthreads();
            if (tid < EPW && sact[tid]) {
                double num = 0.0, den = 0.0;
                const float* fl = sflow + tid * E;
                const float* ax = saux + tid * E;
                const float* dp = sdprev + tid * E;
                for (int e = 0; e < E; ++e) {
                    const float dfw = __fsub_rn(ax[e], fl[e]);
                    num += (double)__fmul_rn(dfw, __fsub_rn(dfw, dp[e]));
                    den += (double)__fmul_rn(dp[e], dp[e]);
                }
                sred[2 * tid] = num;
                sred[2 * tid + 1] = den;
            }
            __syncthreads();
        }
        const double stepd = (p.method == TRX_METHOD_MSA) ? 1.0 / (it + 1.0) : 2.0 / (it + 2.0);
        const float s32 = (float)stepd, om32 = (float)(1.0 - stepd);
        for (int i = tid; i < EL; i += L) {
            const int el = i / E, e = i - el * E;
            if (!sact[el]) continue;
            const float fl = sflow[i];
            const float ax = saux[i];
            float nf;
            if (cfw) {
                const float dfw = __fsub_rn(ax, fl);
                float dir;
                if (it == 0) {
                    dir = dfw;
                } else {
                    const float num = (float)sred[2 * el];
                    const double den = (double)(float)sred[2 * el + 1] + 1e-12;
                    double b = (double)num / den;
                    b = b < 0.0 ? 0.0 : b;
                    dir = __fadd_rn(dfw, __fmul_rn((float)b, sdprev[i]));
                }
                nf = __fadd_rn(fl, __fmul_rn(s32, dir));
                nf = nf > 0.0f ? nf : 0.0f;
                sdprev[i] = dir;
            } else {
                nf = __fadd_rn(__fmul_rn(om32, fl), __fmul_rn(s32, ax));
            }
            if (nf != nf) nf = 0.0f;  // nan_to_num guard (repair_env.py:338-340)
            sflow[i] = nf;
            const float tv = bpr_cost(nf, scap[i], st0[e], sdmg[i], p.bpr_alpha, p.bpr_beta);
            st[i] = tv;
            if (wpos_reg && my_wpos >= 0) sw[my_wpos] = tv;
        }
        __syncthreads();
        TRX_PSTAMP(5);
        if (!wpos_reg) {
            for (int x = tid; x < EPW * NP * NP; x += L) {
                const int el = x / (NP * NP), r = x - el * NP * NP;
                const int u = r / NP, c = r - u * NP;
                const int v = kQ * (c % NPL) + c / NPL;
                const int e = seid[u * NP + v];
                sw[x] = e != 0xFF ? st[el * E + e] : kInfF;
            }
        }
        // tie candidates of the next iteration: in-link pairs with identical costs
        for (int x = tid; x < EPW * NPR; x += L) {
            const int el = x / NPR, q = x - el * NPR;
            const uint32_t pr2 = spairs[q].x;
            if (st[el * E + (pr2 & 0xFFFF)] == st[el * E + (pr2 >> 16)])
                atomicOr(&scand[((cb ^ 1) * EPW + el) * CW + (q >> 5)], 1u << (q & 31));
        }
        __syncthreads();
        TRX_PSTAMP(6);
    }

    // ---------------- per-env unassigned (last iteration; exact integers)
    if (tree_on) atomicAdd(&sunas[lenv], unassigned_lane);
    for (int i = tid; i < EL; i += L) saux[i] = __fmul_rn(sflow[i], st[i]);
    __syncthreads();

    if (tid < EPW && sact[tid]) {
        const int gb = env0 + tid;
        const double un = (double)sunas[tid];
        const double base = (double)pairwise_sum(saux + tid * E, E);
        const double td = g.total_demand > 1.0 ? g.total_demand : 1.0;
        const double tstt = base / td + (un > 0 ? p.unassigned_penalty * (un / td) : 0.0);  // repair_env.py:724-735
        const double prev = s.tstt[gb];
        s.tstt[gb] = tstt;
        s.unassigned[gb] = un;
        if (mode == kModeReset) s.initial_tstt[gb] = tstt;
        if (mode == kModeStep) {
            float rem = 0.0f;
            for (int e = 0; e < E; ++e) rem += __fmul_rn(sgoal[tid * E + e], sdmg[tid * E + e]);
            const bool complete = rem == 0.0f;  // is_goal_complete (293-294)
            reward_out[gb] = reward_fn(p, prev, tstt, s.initial_tstt[gb], complete);
            done_out[gb] = complete ? 1 : 0;
            valid_out[gb] = 1;
        }
    }
    for (int i = tid; i < EL; i += L) {
        const int el = i / E;
        if (!sact[el]) continue;
        const size_t gi = (size_t)(env0 + el) * E + (i - el * E);
        s.flow[gi] = sflow[i];
        if (s.t) s.t[gi] = st[i];
        if (mode != kModeAssign) {
            s.capacity[gi] = scap[i];
            s.damaged[gi] = sdmg[i];
            s.goal[gi] = sgoal[i];
        }
    }
}

LaunchCfg packed_launch_cfg(const DevGraph& g, int num_envs, int method) {
    LaunchCfg c{};
    c.np = g.NP;
    const int per_env = g.Z * kQ;
    static const int epw_env = [] {
        const char* e = getenv("TRX_EPW");  // tuning knob (A/B runs)
        return e ? atoi(e) : 0;
    }();
    int epw = epw_env > 0 ? epw_env : 2;
    while (epw > 1 && epw * per_env > 256) --epw;
    c.epw = epw;
    c.threads = ((epw * per_env + 63) / 64) * 64;
    c.smem = smemp_layout(g.E, g.N, g.Z, c.np, c.epw, c.threads, g.npairs, method == TRX_METHOD_CFW).total;
    c.blocks = (num_envs + c.epw - 1) / c.epw;
    return c;
}

hipError_t launch_env_kernel_packed(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs,
                                   int mode, const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                   const uint8_t* env_mask, hipStream_t stream) {
    const LaunchCfg c = packed_launch_cfg(g, num_envs, p.method);
    if (c.blocks == 0) return hipSuccess;
    if (c.threads > 256) return hipErrorInvalidConfiguration;
    const dim3 grid(c.blocks), block(c.threads);
    switch (c.np) {
        case 8:
            hipLaunchKernelGGL(env_kernel_p<8>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
        case 16:
            hipLaunchKernelGGL(env_kernel_p<16>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
        case 24:
            hipLaunchKernelGGL(env_kernel_p<24>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
        default:
            hipLaunchKernelGGL(env_kernel_p<32>, grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, action,
                               reward, done, valid, env_mask);
            break;
    }
    return hipGetLastError();
}

}  // namespace trx

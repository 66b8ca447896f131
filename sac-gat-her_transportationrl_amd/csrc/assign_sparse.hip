// assign_sparse.hip -- fused batched static traffic assignment, gfx950, v4
// ("sparse-relaxation" kernel).  Same contract and the same exact-label
// packed keys as the round-2 packed kernel (src/env/repair_env.py:167-205 reset,
// 207-237 step, 299-345 assignment, scipy branch of _all_or_nothing 481-503 +
// 707-722, compute_tstt 724-735); the Dijkstra is reorganised around where
// the packed kernel spent its VALU issue:
//
//  * the keys (bits(label) | node id, scanned = sign bit) live in LDS, one
//    [NP] u64 row per shortest-path tree.  Each step the tree's quad reads
//    the row (NP/4 keys per lane, ds_read_b128), takes the (label, id)
//    minimum and relaxes ONLY the extracted node's out-links: lane j of the
//    quad takes out-link slots j, j+4, .. of u from a per-env sparse cost
//    table [NP][DS] and applies a signed 64-bit LDS atomic min (scanned keys
//    are negative: never improved; scipy's strict `>`: an equal key is the
//    same key).  The packed kernel relaxed all NP/4 slots of every lane
//    against a dense [NP][NP] cost matrix (~3 of 24 entries finite).
//  * predecessors come from the atomic's returned old key: a strict
//    improvement makes u the predecessor (scipy's `>`).  Labels are exact
//    sums, so an EQUAL returned key means v already holds this label from the
//    tail pl[v]; scipy scans that tail first unless both tails have the same
//    label -- then its heap order, which our (label, id) order does not
//    follow, decides, and the tree is replayed with the exact Fibonacci heap
//    (device_common.h exact_sssp).  This replaces the packed kernel's
//    tie-candidate link pairs (their per-iteration masks, one barrier).
//  * the all-or-nothing loads come straight out of the subtree-demand pass
//    (reverse scan order): each final S(v) is added to v's predecessor link
//    with a u32 LDS atomic (integral demands: exact), so there is no pass
//    over (link, tree) pairs; subtree sums, the replay heap and the
//    link-position scratch alias the key rows.
// Barriers per MSA/FW iteration: 2 (trees | gather + flow update + BPR +
// cost table).  Exactness preconditions: exact_label_ok() plus out-degree <= 16
// (sparse_ok(); graphs outside them run env_kernel_q, assign_quad.hip).
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>

#include "device_common.h"
#include "trx_internal.h"

#ifdef TRX_PHASE_STAMPS
// Diagnostic build only (make stamps): per-phase cycle totals of thread 0 of
// each workgroup.  Never compiled into the shipped library.
__device__ unsigned long long trx_phase_cycles_s[8];
#define TRX_SSTAMP(slot)                                                    \
    do {                                                                    \
        if (threadIdx.x == 0) {                                             \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
            atomicAdd(&trx_phase_cycles_s[slot], now_ - stamp_prev_);        \
            stamp_prev_ = now_;                                             \
        }                                                                   \
    } while (0)
// per-workgroup wall cycles (thread 0, kernel start -> end) of the last launch
__device__ unsigned long long trx_wg_cycles_s[1 << 16];
extern "C" int trx_debug_wg_cycles_s(unsigned long long* out, int n) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (n > (1 << 16)) n = 1 << 16;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_wg_cycles_s), sizeof(unsigned long long) * n) != hipSuccess)
        return -2;
    return 0;
}
extern "C" int trx_debug_phase_cycles_s(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_phase_cycles_s), sizeof(unsigned long long) * 8) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(trx_phase_cycles_s), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define TRX_SSTAMP(slot) \
    do {                 \
    } while (0)
#endif

#ifndef TRX_SPARSE_WAVES
// waves/SIMD the register budget targets (72 VGPRs; some spills outside the Dijkstra
// loop).  LDS then allows 9 workgroups (27 waves) per CU for Sioux Falls: 0.92 ->
// 0.84 ms per 4096-env step against the 6-wave (80 VGPR, 24 waves) build.
#define TRX_SPARSE_WAVES 7
#endif

namespace trx {

namespace {

constexpr int kQs = 4;
// Key encoding (64 bits, read as a double by the argmin and as a signed integer by
// the relaxation's atomic min):
//   reached, unscanned: bits(label) | id -- a positive double, ordered by (label, id)
//   unreached:          0x7FF8000000000000 | id -- a quiet NaN, the largest positive integer
//   scanned:            high word 0xFFF80000, low word = the scan step at which the node's
//                       equal-label run began -- a quiet NaN, a negative integer
//   padding node:       all ones -- a quiet NaN, a negative integer
// v_min_f64 (IEEE minNum) ignores quiet NaNs, so the argmin sees only reached,
// unscanned nodes; the signed min never improves a scanned key.
constexpr uint64_t kUnreached = 0x7FF8000000000000ull;
constexpr uint32_t kScannedHi = 0xFFF80000u;
constexpr int kMaxDeg = 16;   // out-degree (out-slot rounds of 4: 1, 2, 4)


struct SmemS {
    uint32_t flow, cap, dmg, goal, t, aux, dprev;  // [EPW*E] f32 (dprev: CFW only); aux: u32 AON link
                                                   // loads while an iteration runs, f32 after
    uint32_t ocost;  // [EPW][NP][DS] f32 cost of out-link slot s of u (+inf: none)
    uint32_t ov;     // [NP][DS] u8 head node of out-link slot s of u (empty: u itself)
    uint32_t keys;   // [rows][NP] u64 keys per tree; aliased: subtree sums (f32, first NP of each row),
                     // per-wave replay heap, link-position scratch at start-up
    uint32_t pred;   // [EPW*Z][NP] u8 predecessor node per tree (0xFF: none)
    uint32_t ord;    // [EPW*Z][NP] u8 scan order per tree
    uint32_t eid;    // [NP*NP] u8 link id of (u, v) (0xFF: none; the kernel takes E <= 255)
    uint32_t unas;   // [EPW] f32
    uint32_t act;    // [EPW] i32
    uint32_t red;    // [EPW*2] f64
    uint32_t total;
};

__host__ __device__ inline uint32_t al16s(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline SmemS smems_layout(int E, int N, int Z, int NP, int EPW, int L, int DS,
                                             bool cfw) {
    SmemS o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t bytes) {
        uint32_t r = off;
        off = al16s(off + bytes);
        return r;
    };
    const uint32_t el = (uint32_t)(EPW * E * 4);
    const int rows = ((L + 63) / 64) * 16;  // 16 trees per wave: every wave's heap lies in its own rows
    o.flow = take(el);
    o.cap = take(el);
    o.dmg = take(el);
    o.goal = take(el);
    o.t = take(el);
    o.aux = take(el);
    o.dprev = take(cfw ? el : 0u);
    o.ocost = take((uint32_t)(EPW * NP * DS * 4));
    o.ov = take((uint32_t)(NP * DS));
    o.keys = take((uint32_t)(rows * NP * 8));
    o.pred = take((uint32_t)(EPW * Z * NP));
    o.ord = take((uint32_t)(EPW * Z * NP));
    o.eid = take((uint32_t)(NP * NP));
    o.unas = take((uint32_t)(EPW * 4));
    o.act = take((uint32_t)(EPW * 4));
    o.red = take((uint32_t)(EPW * 2 * 8));
    o.total = off;
    return o;
}

template <int CTRL>
__device__ __forceinline__ uint32_t qps(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t qps64(uint64_t x) {
    return ((uint64_t)qps<CTRL>((uint32_t)(x >> 32)) << 32) | qps<CTRL>((uint32_t)x);
}
__device__ __forceinline__ uint64_t dbits_s(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double bitsd_s(uint64_t b) { return __longlong_as_double((long long)b); }

// v_min_f64 without the compiler's sNaN canonicalisation of the inputs (all NaN
// keys are quiet by construction)
__device__ __forceinline__ double vmin_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ void wave_sync_s() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The lane's NPL consecutive keys of a tree row (16-byte LDS reads).
template <int NPL>
__device__ __forceinline__ void read_keys(const uint64_t* row, uint64_t (&m)[NPL]) {
    const uint4* r4 = reinterpret_cast<const uint4*>(row);
#pragma unroll
    for (int q = 0; q < NPL / 2; ++q) {
        const uint4 w = r4[q];
        m[2 * q] = ((uint64_t)w.y << 32) | w.x;
        m[2 * q + 1] = ((uint64_t)w.w << 32) | w.z;
    }
}

// The exact scipy-heap replay of one ambiguous tree, run by the whole wave in
// lockstep with the heap held in registers: lane x keeps node x's heap fields
// (value, parent, left, right, child, rank, state) and roots[x]; a field of
// node i is read with v_readlane and written by a lane select (i is
// wave-uniform: the heap walk is sequential), so device_common.h's Fibonacci
// heap runs unchanged on register proxies instead of pointer-chasing LDS or
// global memory (~10x shorter per replay: a tie that persists through every
// MSA iteration of a step no longer holds the launch).
__device__ __forceinline__ int lane_put(int old, int x, int i) {  // lane i's copy := x
    return (int)(threadIdx.x & 63) == i ? x : old;
}
struct LaneI {  // one int per lane: lane i holds entry i
    int v;
    struct Ref {
        int* p;
        int i;
        __device__ __forceinline__ operator int() const { return __builtin_amdgcn_readlane(*p, i); }
        __device__ __forceinline__ Ref& operator=(int x) {
            *p = lane_put(*p, x, i);
            return *this;
        }
        __device__ __forceinline__ Ref& operator=(const Ref& o) { return *this = (int)o; }
        __device__ __forceinline__ Ref& operator+=(int d) { return *this = (int)*this + d; }
        __device__ __forceinline__ Ref& operator-=(int d) { return *this = (int)*this - d; }
    };
    __device__ __forceinline__ Ref operator[](int i) { return Ref{&v, i}; }
};
struct LaneD {  // one double per lane (two 32-bit halves)
    int lo, hi;
    struct Ref {
        LaneD* p;
        int i;
        __device__ __forceinline__ operator double() const {
            const uint32_t l = (uint32_t)__builtin_amdgcn_readlane(p->lo, i);
            const uint32_t h = (uint32_t)__builtin_amdgcn_readlane(p->hi, i);
            return __longlong_as_double((long long)(((uint64_t)h << 32) | l));
        }
        __device__ __forceinline__ Ref& operator=(double x) {
            const uint64_t b = (uint64_t)__double_as_longlong(x);
            p->lo = lane_put(p->lo, (int)(uint32_t)b, i);
            p->hi = lane_put(p->hi, (int)(uint32_t)(b >> 32), i);
            return *this;
        }
    };
    __device__ __forceinline__ Ref operator[](int i) { return Ref{this, i}; }
};
struct WaveHeap {
    using idx_t = int;
    LaneD val;
    LaneI parent, left, right, child, rank, state, roots;
};

// device_common.h exact_sssp's loop on the wave heap, with the adjacency and
// the costs read from the workgroup's LDS tables: u's k-th out-link (scipy CSR
// order) sits in slot (k % 4) * R + k / 4 of row u of the sparse tables (head
// node in `ov`, cost in `oc`; empty slots name u itself and come after the
// real ones).  Every lane runs it; lane 0 writes the scan order and the
// predecessors.
template <int NP, int R>
__device__ __forceinline__ void replay_tree_wave(int N, const uint8_t* ov, const float* oc, int origin, uint8_t* ol,
                                                 uint8_t* pl) {
    constexpr int DS = 4 * R;
    const int lane = (int)(threadIdx.x & 63);
    WaveHeap hh;
    hh.val.lo = hh.val.hi = 0;
    hh.parent.v = hh.left.v = hh.right.v = hh.child.v = -1;
    hh.rank.v = hh.state.v = 0;
    hh.roots.v = -1;
    if (lane < N) pl[lane] = kNoPred;
    Heap<WaveHeap> H{&hh, -1};
    WaveHeap* const h = &hh;
    fh_insert(H, origin);
    int k = 0;
    while (H.min >= 0) {
        const int v = fh_remove_min(H);
        h->state[v] = 2;
        if (lane == 0) ol[k] = (uint8_t)v;
        ++k;
        const double vv = h->val[v];
        for (int q = 0; q < DS; ++q) {
            const int slot = v * DS + (q & 3) * R + (q >> 2);
            const int jc = __builtin_amdgcn_readfirstlane((int)ov[slot]);
            if (jc == v) break;  // no more out-links
            const int st = h->state[jc];
            if (st != 2) {
                const double nv = vv + (double)oc[slot];
                if (st == 0) {
                    h->state[jc] = 1;
                    h->val[jc] = nv;
                    fh_insert(H, jc);
                    if (lane == 0) pl[jc] = (uint8_t)v;
                } else if (h->val[jc] > nv) {
                    fh_decrease(H, jc, nv);
                    if (lane == 0) pl[jc] = (uint8_t)v;
                }
            }
        }
    }
}

// Fibonacci-heap storage of one replay sized for NP nodes, carved from the
// wave's key rows in LDS (dead between the Dijkstra and the subtree pass).
template <int NPX>
struct FibSmall {
    using idx_t = int8_t;
    double val[NPX];
    int8_t parent[NPX], left[NPX], right[NPX], child[NPX];
    uint8_t rank[NPX], state[NPX];
    int8_t roots[32];
};

// The exact scipy-heap replay of one ambiguous tree (rare: out of line so the
// Dijkstra loop's registers are not sized for it); writes scan order and preds.
// device_common.h exact_sssp's loop, with the adjacency and the costs read from
// the workgroup's LDS tables instead of the graph in global memory: u's k-th
// out-link (scipy CSR order) sits in slot (k % 4) * R + k / 4 of row u of the
// sparse tables (head node in `ov`, cost in `oc`; empty slots name u itself and
// come after the real ones).
template <int NP, int R>
__device__ __noinline__ void replay_tree_s(int N, const uint8_t* ov, const float* oc, int origin, FibSmall<NP>* h,
                                           uint8_t* ol, uint8_t* pl) {
    constexpr int DS = 4 * R;
    for (int k = 0; k < N; ++k) {
        h->val[k] = 0.0;
        h->parent[k] = h->left[k] = h->right[k] = h->child[k] = -1;
        h->rank[k] = 0;
        h->state[k] = 0;
        pl[k] = kNoPred;
    }
    Heap<FibSmall<NP>> H{h, -1};
    fh_insert(H, origin);
    int k = 0;
    while (H.min >= 0) {
        const int v = fh_remove_min(H);
        h->state[v] = 2;
        ol[k++] = (uint8_t)v;
        const double vv = h->val[v];
        for (int q = 0; q < DS; ++q) {
            const int slot = v * DS + (q & 3) * R + (q >> 2);
            const int jc = ov[slot];
            if (jc == v) break;  // no more out-links
            const int st = h->state[jc];
            if (st != 2) {
                const double nv = vv + (double)oc[slot];
                if (st == 0) {
                    h->state[jc] = 1;
                    h->val[jc] = nv;
                    fh_insert(H, jc);
                    pl[jc] = (uint8_t)v;
                } else if (h->val[jc] > nv) {
                    fh_decrease(H, jc, nv);
                    pl[jc] = (uint8_t)v;
                }
            }
        }
    }
}

// out-slot rounds of 4 (the kernel is instantiated for 1, 2 and 4)
int sparse_rounds(const DevGraph& g) {
    const int r = (g.max_out_deg + kQs - 1) / kQs;
    return r <= 1 ? 1 : (r == 2 ? 2 : 4);
}

}  // namespace

// Exact-label headroom: every path label is an exact float64 sum of float32
// link costs, each a multiple of g = ulp(smallest float32 cost); when
// (N-1) * t_max < 2^48 g the label's mantissa ends in >= 5 zero bits, which
// carry the node id of the key.  t_max bounds the BPR cost at the v/c clip
// (10) and the damaged-link cost 1e6 (repair_env.py:667-677).
bool exact_label_ok(const DevGraph& g, const trx_params& p) {
    if (!(g.min_t0 > 0.0f) || p.bpr_alpha < 0.0f || g.E > 255) return false;
    int ex = 0;
    std::frexp((double)g.min_t0, &ex);                 // min_t0 = m * 2^ex, m in [0.5, 1)
    const double gran = std::ldexp(1.0, ex - 1 - 23);  // ulp of the smallest float32 cost
    const double tmax = std::fmax(1e6, (double)g.max_t0 * (1.0 + (double)p.bpr_alpha * std::pow(10.0, p.bpr_beta)));
    const double bound = (double)(g.N - 1) * tmax * 1.0001;
    return bound < std::ldexp(gran, 48);
}

bool sparse_ok(const DevGraph& g, const trx_params& p) {
    if (g.N > kSmallMaxNodes || !exact_label_ok(g, p) || g.max_out_deg > kMaxDeg || g.NP % 8 != 0) return false;
    // the launch budget launch_env_kernel_sparse enforces, checked here so that
    // selection falls through to env_kernel_q instead of failing the step
    const LaunchCfg c = sparse_launch_cfg(g, 1, p.method);
    return c.threads <= 256 && c.smem <= 64 * 1024;
}

template <int NP, int R>  // R = out-slot rounds per extracted node (DS = 4R slots)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TRX_SPARSE_WAVES)))
env_kernel_s(const DevGraph g, const trx_params p, const trx_state s, int B, int EPW, int mode,
             const int32_t* __restrict__ action, double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
             uint8_t* __restrict__ valid_out, const uint8_t* __restrict__ env_mask, unsigned char* __restrict__ ws) {
    constexpr int NPL = NP / kQs;
    constexpr int DS = R * kQs;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N, Z = g.Z;
    const int L = blockDim.x;
    const int tid = threadIdx.x;
    const int EL = EPW * E;
    const int env0 = blockIdx.x * EPW;
    const bool cfw = p.method == TRX_METHOD_CFW;
    const SmemS O = smems_layout(E, N, Z, NP, EPW, L, DS, cfw);
    float* const sflow = (float*)(smem_raw + O.flow);
    float* const scap = (float*)(smem_raw + O.cap);
    float* const sdmg = (float*)(smem_raw + O.dmg);
    float* const sgoal = (float*)(smem_raw + O.goal);
    float* const st = (float*)(smem_raw + O.t);
    float* const saux = (float*)(smem_raw + O.aux);
    float* const sdprev = (float*)(smem_raw + O.dprev);
    float* const socost = (float*)(smem_raw + O.ocost);
    uint8_t* const sov = smem_raw + O.ov;
    uint64_t* const skeys = (uint64_t*)(smem_raw + O.keys);
    uint8_t* const spred = smem_raw + O.pred;
    uint8_t* const sord = smem_raw + O.ord;
    uint8_t* const seid = smem_raw + O.eid;
    uint32_t* const sload = reinterpret_cast<uint32_t*>(saux);  // AON link loads (integral demands)
    const float* const gdem = g.dem;  // [Z*N] demands and [E] free-flow times: read from the graph
    const float* const gt0 = g.t0;    // (global, cached) -- LDS per workgroup bounds residency
    float* const sunas = (float*)(smem_raw + O.unas);
    int* const sact = (int*)(smem_raw + O.act);
    double* const sred = (double*)(smem_raw + O.red);
    const int DSP = DS;  // row stride of the out-slot tables (padded rows measured neutral, round 3)
    const int NDS = NP * DSP;
#ifdef TRX_PHASE_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
    const unsigned long long wg_start_ = stamp_prev_;
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
    // static tables: sparse out-adjacency (scipy CSR order), in-adjacency
    int16_t* const opos_tmp = reinterpret_cast<int16_t*>(skeys);  // [E] scratch in the key rows
    // padding entries are harmless no-ops, so the loops below need no validity
    // tests: an empty out-slot of u targets u itself (scanned before its
    // relaxation: never improved) at cost +inf; an empty in-slot of v names v
    // itself as tail over link 0 (label(v) + cost > label(v): never achieving)
    for (int i = tid; i < NDS; i += L) sov[i] = (uint8_t)(i / DSP);
    for (int i = tid; i < NP * NP; i += L) seid[i] = (uint8_t)g.eid_of[i];
    for (int i = tid; i < EPW * NDS; i += L) socost[i] = kInfF;
    for (int u = tid; u < N; u += L) {
        const int a0 = g.indptr[u], a1 = g.indptr[u + 1];
        for (int a = a0; a < a1; ++a) {
            // out-link k of u -> lane k % 4, round k / 4: each lane's R slots are contiguous
            const int pos = u * DSP + ((a - a0) & (kQs - 1)) * R + (a - a0) / kQs;
            sov[pos] = (uint8_t)g.indices[a];
            opos_tmp[g.csr_eid[a]] = (int16_t)pos;
        }
    }
    __syncthreads();
    const bool opos_reg = EL <= L;  // one (env, link) per thread: its cost-table slot in a register
    int my_opos = -1;
    if (opos_reg && tid < EL) {
        const int el = tid / E, e = tid - el * E;
        my_opos = el * NDS + opos_tmp[e];
    }
    __syncthreads();  // the scratch is overwritten by the key rows below

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
        const float tv = sact[el] ? bpr_cost(fl, cp, gt0[e], dm, p.bpr_alpha, p.bpr_beta) : 0.0f;
        st[i] = tv;
        if (my_opos >= 0) socost[my_opos] = tv;  // opos_reg: i == tid
    }
    __syncthreads();
    if (!opos_reg) {  // generic path: cost-table entries from the static out-adjacency
        for (int x = tid; x < EPW * NDS; x += L) {
            const int el = x / NDS, r = x - el * NDS;
            const int u = r / DSP, v = sov[r];
            socost[x] = v != u ? st[el * E + g.eid_of[u * NP + v]] : kInfF;
        }
    }
    __syncthreads();

    // thread -> (tree = (env, origin zone), lane j of its quad)
    const int tree = tid / kQs;
    const int j = tid & (kQs - 1);
    const int lenv = tree / Z;
    const int zi = tree - lenv * Z;
    const bool tree_on = (lenv < EPW) && sact[lenv];
    const int origin = tree_on ? g.origins[zi] : 0;
    float unassigned_lane = 0.0f;
    TRX_SSTAMP(0);

    for (int it = 0; it < p.iters; ++it) {
        // ---------------- shortest-path tree per quad (Dijkstra, sparse relaxation)
        if (tree_on) {
            uint64_t* const kt = skeys + tree * NP;
            uint32_t* const kt32 = reinterpret_cast<uint32_t*>(kt);
            const float* const oc = socost + lenv * NDS;
            uint8_t* const ol = sord + tree * NP;
            uint8_t* const pl = spred + tree * NP;
            int jo = j;
            asm volatile("" : "+v"(jo));  // keep the key set-up inside the loop (no hoist + spill)
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int v = NPL * jo + i;
                kt[NPL * j + i] = v >= N ? ~0ull : (v == origin ? (uint64_t)v : (kUnreached | (uint64_t)v));
                pl[NPL * j + i] = kNoPred;
            }
            wave_sync_s();
            int nscan = 0;
            int amb = 0;
            // equal-label runs of the scan order: labels come out non-decreasing, so two
            // scanned nodes have equal labels iff they belong to the same run (run = the
            // scan step at which the run began, stored in the scanned key's low word)
            int run = 0;
            uint64_t prev_lb = ~0ull;
            uint64_t m[NPL];
            read_keys<NPL>(kt + NPL * j, m);
            for (int k = 0; k < N; ++k) {
                // argmin over the lane's keys (pairwise v_min_f64), then over the quad (DPP)
                double d[NPL];
#pragma unroll
                for (int i = 0; i < NPL; ++i) d[i] = bitsd_s(m[i]);
#pragma unroll
                for (int w = 1; w < NPL; w *= 2)
#pragma unroll
                    for (int i = 0; i + w < NPL; i += 2 * w) d[i] = vmin_f64(d[i], d[i + w]);
                double bd = vmin_f64(d[0], bitsd_s(qps64<0xB1>(dbits_s(d[0]))));
                bd = vmin_f64(bd, bitsd_s(qps64<0x4E>(dbits_s(bd))));
                if (!(bd < kInfD)) break;  // quad-uniform: the rest is unreachable (NaN or +inf: all ignored)
                const uint64_t best = dbits_s(bd);
                const uint32_t u = (uint32_t)best & 31u;
                const uint64_t lb = best & ~31ull;
                if (lb != prev_lb) {  // quad-uniform
                    run = k;
                    prev_lb = lb;
                }
                // one lane of the quad stores the scan order and the scanned mark (+ run)
                if (j == 0) {
                    ol[k] = (uint8_t)u;
                    kt[u] = ((uint64_t)kScannedHi << 32) | (uint32_t)run;
                }
                nscan = k + 1;
                const double bl = bitsd_s(lb);
                uint32_t v[R];
                float c[R];
                {  // lane j's R slots of u: one read each for heads and costs
                    const int sl = (int)u * DSP + j * R;
                    if constexpr (R == 1) {
                        v[0] = sov[sl];
                        c[0] = oc[sl];
                    } else if constexpr (R == 2) {
                        const uint32_t hv = *reinterpret_cast<const uint16_t*>(sov + sl);
                        const float2 cv = *reinterpret_cast<const float2*>(oc + sl);
                        v[0] = hv & 0xFFu;
                        v[1] = hv >> 8;
                        c[0] = cv.x;
                        c[1] = cv.y;
                    } else {
                        const uint32_t hv = *reinterpret_cast<const uint32_t*>(sov + sl);
                        const float4 cv = *reinterpret_cast<const float4*>(oc + sl);
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = (hv >> (8 * r)) & 0xFFu;
                        c[0] = cv.x;
                        c[1] = cv.y;
                        c[2] = cv.z;
                        c[3] = cv.w;
                    }
                }
                long long nk[R], was[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {  // the atomics back to back; empty slots (v == u) skip theirs
                    nk[r] = (long long)(dbits_s(__dadd_rn(bl, (double)c[r])) | v[r]);
                    was[r] = LLONG_MIN;
                    if (v[r] != u)
                        was[r] = __hip_atomic_fetch_min(reinterpret_cast<long long*>(kt + v[r]), nk[r],
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                // next step's keys: issued behind the mark and the atomics (a wave's LDS
                // operations complete in order), before waiting on the atomics' results
                read_keys<NPL>(kt + NPL * j, m);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    // scipy's strict improvement: u becomes v's predecessor.  An equal key
                    // means v already holds this label from the tail pl[v] (scanned before
                    // u); scipy's order between the two is its heap's iff the tails' labels
                    // are equal, i.e. iff pl[v] is in u's equal-label run (exact: no false
                    // positives, so warm-started steps never replay on integral labels)
                    if (nk[r] < was[r]) pl[v[r]] = (uint8_t)u;
                    if (nk[r] == was[r]) amb |= kt32[2 * pl[v[r]]] == (uint32_t)run;
                }
            }
            wave_sync_s();
            TRX_SSTAMP(1);
            amb |= (int)qps<0xB1>((uint32_t)amb);
            amb |= (int)qps<0x4E>((uint32_t)amb);
            const uint64_t need = __ballot(amb != 0 && j == 0);
            wave_sync_s();
            TRX_SSTAMP(2);
#ifdef TRX_PHASE_STAMPS
            if (tid == 0) atomicAdd(&trx_phase_cycles_s[7], (unsigned long long)__popcll(need));  // replayed trees (wave 0)
#endif
            if (need) {  // wave-uniform: exact scipy-heap replays of the ambiguous trees
                if (__ballot(1) == ~0ull) {
                    // every lane of the wave is active: one tree at a time by the whole wave,
                    // the heap in registers (replay_tree_wave)
                    uint64_t pend = need;
                    while (pend) {
                        const int bit = __builtin_ctzll(pend);
                        pend &= pend - 1;
                        const int t = (int)(tid >> 6) * 16 + (bit >> 2);  // the tree of quad leader `bit`
                        const int le = t / Z, zt = t - le * Z;
                        replay_tree_wave<NP, R>(N, sov, socost + le * NDS, g.origins[zt], sord + t * NP,
                                                spred + t * NP);
                    }
                    wave_sync_s();
                } else {  // an inactive env leaves lanes of the wave off: per-lane heaps in LDS
                    // the ambiguous trees' quad leaders replay their trees concurrently, each with
                    // its own heap in LDS: the wave's 16 key rows (16 * NP * 8 bytes, dead until the
                    // subtree pass re-initialises them) hold kSlots heaps, so up to kSlots trees per
                    // round.  (A heap in global memory cost ~1 ms of dependent misses per replay,
                    // and a single replay held the whole launch.)
                    constexpr int kHeapBytes = (int)((sizeof(FibSmall<NP>) + 7) & ~(size_t)7);
                    constexpr int kSlots = (16 * NP * 8) / kHeapBytes;
                    static_assert(kSlots >= 1, "replay heap does not fit the wave's key rows");
                    unsigned char* const area = reinterpret_cast<unsigned char*>(skeys + (size_t)(tid >> 6) * 16 * NP);
                    const int lane = tid & 63;
                    uint64_t pend = need;
                    while (pend) {  // wave-uniform
                        uint64_t batch = 0, m = pend;
                        for (int c = 0; c < kSlots && m; ++c) {
                            const uint64_t b = m & (~m + 1);
                            batch |= b;
                            m ^= b;
                        }
                        pend &= ~batch;
                        if ((batch >> lane) & 1ull) {
                            const int slot = __popcll(batch & ((1ull << lane) - 1ull));
                            FibSmall<NP>* const h = reinterpret_cast<FibSmall<NP>*>(area + slot * kHeapBytes);
                            replay_tree_s<NP, R>(N, sov, oc, origin, h, ol, pl);
                        }
                        wave_sync_s();
                    }
                }
            }
            // ---------------- all-or-nothing (repair_env.py:490-502, 707-722): subtree
            // demand sums S(v) per tree in reverse scan order, once final added to
            // the load of v's predecessor link (u32 LDS atomics; integral demands:
            // exact in any order).  The quad's four lanes take the scan slots four
            // at a time (group = one scan-order word, lane j slot 4G + 3 - j, so
            // lane 0 is the latest scanned): each lane reads its S(v) -- complete
            // but for children scanned in the same group -- adds those over three
            // quad broadcasts (lane m's S is final after round m), then adds S(v)
            // to v's link load and, unless v's predecessor is in the group (it has
            // taken S(v) already), to the predecessor's S (u32 LDS atomic: two
            // lanes may share a predecessor).
            const float* dm = gdem + zi * N;
            uint32_t* const sa = reinterpret_cast<uint32_t*>(kt);
            float un = 0.0f;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int v = NPL * j + i;
                const float dv = v < N ? dm[v] : 0.0f;
                const bool load = v < N && pl[v] != kNoPred;  // reached, not the origin
                un += (dv > 0.0f && !load) ? dv : 0.0f;      // intrazonal or unreachable (708)
                sa[v] = load ? (uint32_t)dv : 0u;             // exact: integral demands < 2^24
            }
            wave_sync_s();
            {
                uint32_t* const ll = sload + lenv * E;
                constexpr int QH = NP / 8;  // scan-order words per half: two halves keep 2*QH VGPRs live
#pragma unroll
                for (int half = 1; half >= 0; --half) {
                    uint32_t ow[QH], pw[QH];  // scan order and predecessors of this half, in registers
#pragma unroll
                    for (int q = 0; q < QH; ++q) ow[q] = reinterpret_cast<const uint32_t*>(ol)[half * QH + q];
#pragma unroll
                    for (int q = 0; q < QH; ++q) {
                        uint32_t w = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            w |= (4 * (half * QH + q) + b < nscan ? (uint32_t)pl[(ow[q] >> (8 * b)) & 0xFF] : 0u)
                                 << (8 * b);
                        pw[q] = w;
                    }
#pragma unroll
                    for (int q = QH - 1; q >= 0; --q) {
                        const int kb = 4 * (half * QH + q);  // the group's first scan slot
                        if (kb >= nscan) continue;           // quad-uniform
                        const int sh = 8 * (3 - j);          // my slot kb + 3 - j
                        const bool valid = kb + 3 - j >= 1 && kb + 3 - j < nscan;
                        const int v = (ow[q] >> sh) & 0xFF, pv = (pw[q] >> sh) & 0xFF;
                        uint32_t S = valid ? sa[v] : 0u;
                        const int e = valid ? seid[pv * NP + v] : 0;
                        auto take = [&](const uint32_t Sm, const int m) {  // lane m's final S, to its parent
                            const int km = kb + 3 - m, pvm = (pw[q] >> (8 * (3 - m))) & 0xFF;
                            const bool vm = km >= 1 && km < nscan;
                            S += (j > m && vm && valid && pvm == v) ? Sm : 0u;
                        };
                        take((uint32_t)__builtin_amdgcn_update_dpp(0, (int)S, 0x00, 0xf, 0xf, false), 0);
                        take((uint32_t)__builtin_amdgcn_update_dpp(0, (int)S, 0x55, 0xf, 0xf, false), 1);
                        take((uint32_t)__builtin_amdgcn_update_dpp(0, (int)S, 0xAA, 0xf, 0xf, false), 2);
                        bool parent_here = false;  // v's predecessor scanned in this group, after v
#pragma unroll
                        for (int m = 1; m < 4; ++m) {
                            const int km = kb + 3 - m, vmn = (ow[q] >> (8 * (3 - m))) & 0xFF;
                            parent_here |= m > j && km >= 1 && km < nscan && vmn == pv;
                        }
                        if (valid) {
                            atomicAdd(ll + e, S);
                            if (!parent_here) atomicAdd(sa + pv, S);
                        }
                    }
                }
            }
            unassigned_lane = un;
            TRX_SSTAMP(3);
        }
        __syncthreads();
        TRX_SSTAMP(4);

        // ---------------- flow update + BPR + next cost table (repair_env.py:317-342)
        const double stepd = (p.method == TRX_METHOD_MSA) ? 1.0 / (it + 1.0) : 2.0 / (it + 2.0);
        const float s32 = (float)stepd, om32 = (float)(1.0 - stepd);
        if (cfw) {  // the conjugate direction needs every link's load of the env
            for (int i = tid; i < EL; i += L) saux[i] = (float)sload[i];  // exact: < 2^24
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
        for (int i = tid; i < EL; i += L) {
            const int el = i / E, e = i - el * E;
            if (!sact[el]) continue;
            const float fl = sflow[i];
            const float ax = cfw ? saux[i] : (float)sload[i];  // exact: integral, < 2^24
            sload[i] = 0u;                                       // the next iteration's loads
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
            const float tv = bpr_cost(nf, scap[i], gt0[e], sdmg[i], p.bpr_alpha, p.bpr_beta);
            st[i] = tv;
            if (my_opos >= 0) socost[my_opos] = tv;
        }
        __syncthreads();
        if (!opos_reg) {
            for (int x = tid; x < EPW * NDS; x += L) {
                const int el = x / NDS, r = x - el * NDS;
                const int u = r / DSP, v = sov[r];
                if (v != u) socost[x] = st[el * E + g.eid_of[u * NP + v]];
            }
            __syncthreads();
        }
    }

    TRX_SSTAMP(5);
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
    TRX_SSTAMP(6);
#ifdef TRX_PHASE_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < (1u << 16)) trx_wg_cycles_s[blockIdx.x] = __builtin_amdgcn_s_memtime() - wg_start_;
#endif
}

size_t sparse_workspace_bytes(const DevGraph& g, int num_envs) {
    const LaunchCfg c = sparse_launch_cfg(g, num_envs, TRX_METHOD_MSA);
    return (size_t)c.blocks * (size_t)(c.threads / 4) * sizeof(FibLane);  // one exact heap per tree (quad)
}

LaunchCfg sparse_launch_cfg(const DevGraph& g, int num_envs, int method) {
    LaunchCfg c{};
    c.np = g.NP;
    const int per_env = g.Z * kQs;
    static const int epw_env = [] {
        const char* e = getenv("TRX_EPW");  // tuning knob (A/B runs)
        return e ? atoi(e) : 0;
    }();
    int epw = epw_env > 0 ? epw_env : 2;
    while (epw > 1 && epw * per_env > 256) --epw;
    c.epw = epw;
    c.threads = ((epw * per_env + 63) / 64) * 64;
    c.smem = smems_layout(g.E, g.N, g.Z, c.np, c.epw, c.threads, sparse_rounds(g) * kQs,
                          method == TRX_METHOD_CFW).total;
    c.blocks = (num_envs + c.epw - 1) / c.epw;
    return c;
}

hipError_t launch_env_kernel_sparse(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs,
                                    int mode, const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                    const uint8_t* env_mask, void* ws, hipStream_t stream) {
    const LaunchCfg c = sparse_launch_cfg(g, num_envs, p.method);
    if (c.blocks == 0) return hipSuccess;
    if (c.threads > 256 || c.smem > 64 * 1024) return hipErrorInvalidConfiguration;
    const int R = sparse_rounds(g);
    const dim3 grid(c.blocks), block(c.threads);
#define TRX_SPARSE_LAUNCH(NPV, RV)                                                                              \
    hipLaunchKernelGGL((env_kernel_s<NPV, RV>), grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, \
                       action, reward, done, valid, env_mask, static_cast<unsigned char*>(ws))
#define TRX_SPARSE_NP(NPV)             \
    if (R == 1)                        \
        TRX_SPARSE_LAUNCH(NPV, 1);     \
    else if (R == 2)                   \
        TRX_SPARSE_LAUNCH(NPV, 2);     \
    else                               \
        TRX_SPARSE_LAUNCH(NPV, 4)
    switch (c.np) {
        case 8:
            TRX_SPARSE_NP(8);
            break;
        case 16:
            TRX_SPARSE_NP(16);
            break;
        case 24:
            TRX_SPARSE_NP(24);
            break;
        default:
            TRX_SPARSE_NP(32);
            break;
    }
#undef TRX_SPARSE_NP
#undef TRX_SPARSE_LAUNCH
    return hipGetLastError();
}

}  // namespace trx

// assign_pair.hip -- fused batched static traffic assignment, gfx950, v5
// ("pair" kernel, env_kernel_pair<NP, RS, FULL>): one shortest-path tree per
// PAIR of lanes.  Same contract, key encoding and exactness argument as the
// quad kernel env_kernel_s (assign_sparse.hip; reset repair_env.py:167-205, step
// 207-237, assignment 299-345, scipy branch of _all_or_nothing 481-503 +
// 707-722, compute_tstt 724-735); reorganised around VALU issue, which bounds
// env_kernel_s (VALU busy 0.71, 53 K VALU instructions per wave for 16 trees):
//
//  * two lanes per tree instead of four.  Every Dijkstra step costs a fixed
//    number of wave instructions (key reads, argmin, extraction, relaxation,
//    predecessor / tie tests); a wave now carries 32 trees instead of 16, so
//    each tree pays about half the issue.  Lane j owns the 2-key chunks
//    4q + 2j of its tree's key row (12 keys for Sioux Falls: 6 ds_read_b128,
//    11 v_min_f64, one DPP swap); the row stride NP + 4 keys puts the 16 lanes
//    of every ds_read_b128 lane group on distinct bank quads (conflict-free);
//  * the out-slot table holds each slot's cost as a float64 with the head node
//    in its low 5 bits (a float32 widened to float64 has 29 zero low bits): one
//    8-byte read per slot yields both, and at step 0 (the origin, label 0) the
//    entry IS the relaxed key;
//  * the steps are unrolled over NP: the scan-order store takes its slot as an
//    immediate offset, and on graphs where every origin reaches every node
//    and N == NP (FULL; reachability is checked at trx_graph_create) there is
//    no exit test, no predecessor reset, and the last step relaxes nothing
//    (every head is scanned);
//  * equal-label tails need no run tracking: labels are exact sums, so when v
//    receives a key EQUAL to its current one from u, label(pl[v]) + c(pl[v], v)
//    == label(u) + c(u, v) exactly, and the two tails' labels are equal (scipy's
//    heap order decides: exact replay) iff the two link costs are equal;
//  * the subtree pass takes the scan slots two at a time (lane 0 the later one):
//    lane 1 adds lane 0's final sum over one DPP broadcast when lane 0's node is
//    its child, so each tree's dependent LDS chain is NP/2 round trips.
// Barriers per MSA/FW iteration: 2, as env_kernel_s.  Exactness preconditions:
// exact_label_ok() plus out-degree <= 8 (pair_ok()); graphs outside them run
// env_kernel_s / env_kernel_q.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>

#include "device_common.h"
#include "trx_internal.h"

#ifdef TRX_PHASE_STAMPS
// Diagnostic build only (make stamps): per-phase cycle totals of thread 0 of
// each workgroup.  Never compiled into the shipped library.
__device__ unsigned long long trx_phase_cycles_w[8];
#define TRX_WSTAMP(slot)                                                    \
    do {                                                                    \
        if (threadIdx.x == 0) {                                             \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
            atomicAdd(&trx_phase_cycles_w[slot], now_ - stamp_prev_);        \
            stamp_prev_ = now_;                                             \
        }                                                                   \
    } while (0)
// per-workgroup wall cycles (thread 0, kernel start -> end) of the last launch
__device__ unsigned long long trx_wg_cycles_w[1 << 16];
extern "C" int trx_debug_wg_cycles_w(unsigned long long* out, int n) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (n > (1 << 16)) n = 1 << 16;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_wg_cycles_w), sizeof(unsigned long long) * n) != hipSuccess)
        return -2;
    return 0;
}
extern "C" int trx_debug_phase_cycles_w(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_phase_cycles_w), sizeof(unsigned long long) * 8) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(trx_phase_cycles_w), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define TRX_WSTAMP(slot) \
    do {                 \
    } while (0)
#endif

namespace trx {

namespace {

// key encoding: env_kernel_s's (assign_sparse.hip).  Scanned keys carry no run here.
constexpr uint64_t kUnreachedW = 0x7FF8000000000000ull;  // | id: quiet NaN, largest positive integers
constexpr uint64_t kScannedW = 0xFFF8000000000000ull;    // quiet NaN, negative integer
constexpr int kPairMaxDeg = 8;                           // out-slots per node: 2 lanes x RS rounds
constexpr uint32_t kEidBytes = 32 * 32;                  // (u, v) -> link id table at LDS offset 0
#ifndef TRX_PAIR_WAVE_REPLAYS
#define TRX_PAIR_WAVE_REPLAYS 2
#endif
// ambiguous trees of a wave up to which the whole wave replays them one at a time
// (heap in registers); above it every pair leader replays its own tree at once
constexpr int kWaveReplays = TRX_PAIR_WAVE_REPLAYS;

struct SmemW {
    uint32_t flow, cap, dmg, goal, t, aux, dprev;  // [EPW*E] f32 (aux: u32 AON link loads during an iteration)
    uint32_t opos;   // [E] u32: link's entry in an env's out-slot table | head << 16
    uint32_t oc;     // [EPW][NP][2][RS] u64 out-slot entries: bits(double(cost)) | head
    uint32_t keys;   // [rows][NP + 4] u64 keys per tree; aliased after the Dijkstra: subtree sums (u32 [NP])
    uint32_t pred;   // [rows][NP] u8 predecessor node (0xFF: none)
    uint32_t ord;    // [rows][NP] u8 scan order
    uint32_t unas;   // [EPW] f32
    uint32_t act;    // [EPW] i32
    uint32_t red;    // [EPW*2] f64 (CFW)
    uint32_t total;
};

__host__ __device__ inline uint32_t al16w(uint32_t x) { return (x + 15u) & ~15u; }

// rows = threads / 2 (one per lane pair of the block, idle pairs included)
__host__ __device__ inline SmemW smemw_layout(int E, int NP, int RS, int EPW, int rows, bool cfw) {
    SmemW o{};
    uint32_t off = kEidBytes;  // the (u, v) -> link table sits at offset 0: its address is (u << 5) + v
    auto take = [&off](uint32_t bytes) {
        uint32_t r = off;
        off = al16w(off + bytes);
        return r;
    };
    const uint32_t el = (uint32_t)(EPW * E * 4);
    o.flow = take(el);
    o.cap = take(el);
    o.dmg = take(el);
    o.goal = take(el);
    o.t = take(el);
    o.aux = take(el);
    o.dprev = take(cfw ? el : 0u);
    o.opos = take((uint32_t)(E * 4));
    o.oc = take((uint32_t)(EPW * NP * 2 * RS * 8));
    o.keys = take((uint32_t)(rows * (NP + 4) * 8));
    o.pred = take((uint32_t)(rows * NP));
    o.ord = take((uint32_t)(rows * NP));
    o.unas = take((uint32_t)(EPW * 4));
    o.act = take((uint32_t)(EPW * 4));
    o.red = take((uint32_t)(EPW * 2 * 8));
    o.total = off;
    return o;
}

template <int CTRL>
__device__ __forceinline__ uint32_t wdpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t dbits_w(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double bitsd_w(uint64_t b) { return __longlong_as_double((long long)b); }

// v_min_f64 without the compiler's sNaN canonicalisation of the inputs (all NaN
// keys are quiet by construction)
__device__ __forceinline__ double vmin_w(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ void wave_sync_w() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// out-slot entry: the link cost widened to float64 (29 zero low bits) with the
// head node in the low 5 bits
__device__ __forceinline__ uint64_t slot_entry(float c, uint32_t head) { return dbits_w((double)c) | head; }

// lane j's keys: the 2-key chunks 4q + 2j of the row (NQ = NP / 4 ds_read_b128)
template <int NQ>
__device__ __forceinline__ void read_keys_w(const uint64_t* rowj, uint64_t (&m)[2 * NQ]) {
    const uint4* r4 = reinterpret_cast<const uint4*>(rowj);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const uint4 w = r4[2 * q];
        m[2 * q] = ((uint64_t)w.y << 32) | w.x;
        m[2 * q + 1] = ((uint64_t)w.w << 32) | w.z;
    }
}

// The exact scipy-heap replay of one ambiguous tree by the whole wave, the heap
// in registers (assign_sparse.hip replay_tree_wave's storage), adjacency and
// costs from the env's out-slot table: u's k-th out-link in scipy CSR order is
// entry (u * 2 + k % 2) * RS + k / 2 (empty slots name u itself and come after
// the real ones).  Every lane of the wave runs it; lane 0 writes the scan
// order and the predecessors.
struct LaneIW {
    int v;
    struct Ref {
        int* p;
        int i;
        __device__ __forceinline__ operator int() const { return __builtin_amdgcn_readlane(*p, i); }
        __device__ __forceinline__ Ref& operator=(int x) {
            *p = (int)(threadIdx.x & 63) == i ? x : *p;
            return *this;
        }
        __device__ __forceinline__ Ref& operator=(const Ref& o) { return *this = (int)o; }
        __device__ __forceinline__ Ref& operator+=(int d) { return *this = (int)*this + d; }
        __device__ __forceinline__ Ref& operator-=(int d) { return *this = (int)*this - d; }
    };
    __device__ __forceinline__ Ref operator[](int i) { return Ref{&v, i}; }
};
struct LaneDW {
    int lo, hi;
    struct Ref {
        LaneDW* p;
        int i;
        __device__ __forceinline__ operator double() const {
            const uint32_t l = (uint32_t)__builtin_amdgcn_readlane(p->lo, i);
            const uint32_t h = (uint32_t)__builtin_amdgcn_readlane(p->hi, i);
            return __longlong_as_double((long long)(((uint64_t)h << 32) | l));
        }
        __device__ __forceinline__ Ref& operator=(double x) {
            const uint64_t b = (uint64_t)__double_as_longlong(x);
            const bool me = (int)(threadIdx.x & 63) == i;
            p->lo = me ? (int)(uint32_t)b : p->lo;
            p->hi = me ? (int)(uint32_t)(b >> 32) : p->hi;
            return *this;
        }
    };
    __device__ __forceinline__ Ref operator[](int i) { return Ref{this, i}; }
};
struct WaveHeapW {
    using idx_t = int;
    LaneDW val;
    LaneIW parent, left, right, child, rank, state, roots;
};

template <int RS>
__device__ __forceinline__ void replay_tree_pair(int N, const uint64_t* oc, int origin, uint8_t* ol, uint8_t* pl) {
    const int lane = (int)(threadIdx.x & 63);
    WaveHeapW hh;
    hh.val.lo = hh.val.hi = 0;
    hh.parent.v = hh.left.v = hh.right.v = hh.child.v = -1;
    hh.rank.v = hh.state.v = 0;
    hh.roots.v = -1;
    if (lane < N) pl[lane] = kNoPred;
    Heap<WaveHeapW> H{&hh, -1};
    WaveHeapW* const h = &hh;
    fh_insert(H, origin);
    int k = 0;
    while (H.min >= 0) {
        const int v = fh_remove_min(H);
        h->state[v] = 2;
        if (lane == 0) ol[k] = (uint8_t)v;
        ++k;
        const double vv = h->val[v];
        for (int q = 0; q < 2 * RS; ++q) {
            const uint64_t en = oc[(v * 2 + (q & 1)) * RS + (q >> 1)];
            const int jc = __builtin_amdgcn_readfirstlane((int)((uint32_t)en & 31u));
            if (jc == v) break;  // no more out-links
            const int st = h->state[jc];
            if (st != 2) {
                const double nv = vv + bitsd_w(en & ~31ull);
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

// Fibonacci-heap storage of one per-lane replay sized for NPX nodes, carved from
// the wave's key rows in LDS (dead between the Dijkstra and the subtree pass).
template <int NPX>
struct FibSmallW {
    using idx_t = int8_t;
    double val[NPX];
    int8_t parent[NPX], left[NPX], right[NPX], child[NPX];
    uint8_t rank[NPX], state[NPX];
    int8_t roots[32];
};

// The exact scipy-heap replay of one ambiguous tree by ONE lane (its pair leader),
// the heap in LDS: many of a wave's trees replay concurrently (cold resets with
// random damage are tie-heavy), where replay_tree_pair takes them one at a time.
// Same loop, same adjacency and costs.
template <int NP, int RS>
__device__ __noinline__ void replay_tree_lane(int N, const uint64_t* oc, int origin, FibSmallW<NP>* h, uint8_t* ol,
                                              uint8_t* pl) {
    for (int k = 0; k < N; ++k) {
        h->val[k] = 0.0;
        h->parent[k] = h->left[k] = h->right[k] = h->child[k] = -1;
        h->rank[k] = 0;
        h->state[k] = 0;
        pl[k] = kNoPred;
    }
    Heap<FibSmallW<NP>> H{h, -1};
    fh_insert(H, origin);
    int k = 0;
    while (H.min >= 0) {
        const int v = fh_remove_min(H);
        h->state[v] = 2;
        ol[k++] = (uint8_t)v;
        const double vv = h->val[v];
        for (int q = 0; q < 2 * RS; ++q) {
            const uint64_t en = oc[(v * 2 + (q & 1)) * RS + (q >> 1)];
            const int jc = (int)((uint32_t)en & 31u);
            if (jc == v) break;  // no more out-links
            const int st = h->state[jc];
            if (st != 2) {
                const double nv = vv + bitsd_w(en & ~31ull);
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

}  // namespace

bool pair_ok(const DevGraph& g, const trx_params& p) {
    if (g.N > kSmallMaxNodes || !exact_label_ok(g, p) || g.max_out_deg > kPairMaxDeg || g.NP % 4 != 0) return false;
    const LaunchCfg c = pair_launch_cfg(g, 1, p.method);
    return c.threads <= 256 && c.smem <= 64 * 1024;
}

static int pair_rounds(const DevGraph& g) {  // out-slots per lane: ceil(max out-degree / 2) -> 1..4
    const int r = (g.max_out_deg + 1) / 2;
    return r < 1 ? 1 : r;
}

// 4 waves/SIMD of register budget (<= 128 VGPRs): the 3 waves of each of a CU's 4
// workgroups (Sioux Falls: 4 envs, 39.4 KB of LDS each) must find room on whichever
// SIMDs they are dealt to, so that B = 4096 runs in one round on 256 CUs
template <int NP, int RS, bool FULL>  // RS = out-slots per lane (2 RS per node); FULL: N == NP, every origin reaches every node
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
env_kernel_pair(const DevGraph g, const trx_params p, const trx_state s, int B, int EPW, int mode,
                const int32_t* __restrict__ action, double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                uint8_t* __restrict__ valid_out, const uint8_t* __restrict__ env_mask) {
    constexpr int KR = NP + 4;  // key row stride (u64): conflict-free ds_read_b128 lane groups
    constexpr int NQ = NP / 4;  // 2-key chunks per lane
    constexpr int KL = NP / 2;  // keys per lane
    constexpr int DSP = 2 * RS; // out-slots per node
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int E = g.E, N = g.N, Z = g.Z;
    const int L = blockDim.x;
    const int tid = threadIdx.x;
    const int EL = EPW * E;
    const int env0 = blockIdx.x * EPW;
    const bool cfw = p.method == TRX_METHOD_CFW;
    const SmemW O = smemw_layout(E, NP, RS, EPW, L / 2, cfw);
    uint8_t* const seid = smem_raw;  // [32][32] at offset 0
    float* const sflow = (float*)(smem_raw + O.flow);
    float* const scap = (float*)(smem_raw + O.cap);
    float* const sdmg = (float*)(smem_raw + O.dmg);
    float* const sgoal = (float*)(smem_raw + O.goal);
    float* const st = (float*)(smem_raw + O.t);
    float* const saux = (float*)(smem_raw + O.aux);
    float* const sdprev = (float*)(smem_raw + O.dprev);
    uint32_t* const sopos = (uint32_t*)(smem_raw + O.opos);
    uint64_t* const soc = (uint64_t*)(smem_raw + O.oc);
    uint64_t* const skeys = (uint64_t*)(smem_raw + O.keys);
    uint8_t* const spred = smem_raw + O.pred;
    uint8_t* const sord = smem_raw + O.ord;
    uint32_t* const sload = reinterpret_cast<uint32_t*>(saux);  // AON link loads (integral demands)
    const float* const gdem = g.dem;  // [Z*N] demands and [E] free-flow times: read from the graph
    const float* const gt0 = g.t0;    // (global, cached)
    float* const sunas = (float*)(smem_raw + O.unas);
    int* const sact = (int*)(smem_raw + O.act);
    double* const sred = (double*)(smem_raw + O.red);
    constexpr int ENV_SLOTS = NP * DSP;
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
    // static tables: (u, v) -> link id, each link's out-slot position and head;
    // every out-slot entry starts empty (head = its own node, never relaxed)
    for (int i = tid; i < (int)kEidBytes; i += L) {
        const int u = i >> 5, v = i & 31;
        seid[i] = (u < NP && v < NP) ? (uint8_t)g.eid_of[u * NP + v] : (uint8_t)0xFF;
    }
    for (int i = tid; i < EPW * ENV_SLOTS; i += L) soc[i] = (uint64_t)((i % ENV_SLOTS) / DSP);
    for (int u = tid; u < N; u += L) {
        const int a0 = g.indptr[u], a1 = g.indptr[u + 1];
        for (int a = a0; a < a1; ++a) {
            const int k = a - a0;  // out-link k of u (scipy CSR order) -> lane k % 2, round k / 2
            sopos[g.csr_eid[a]] = (uint32_t)((u * 2 + (k & 1)) * RS + (k >> 1)) | ((uint32_t)g.indices[a] << 16);
        }
    }
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
        const float tv = sact[el] ? bpr_cost(fl, cp, gt0[e], dm, p.bpr_alpha, p.bpr_beta) : 0.0f;
        st[i] = tv;
        const uint32_t op = sopos[e];
        soc[el * ENV_SLOTS + (op & 0xFFFFu)] = slot_entry(tv, op >> 16);
    }
    __syncthreads();

    // thread -> (tree = (env, origin zone), lane j of its pair)
    const int tree = tid >> 1;
    const int j = tid & 1;
    const int lenv = tree / Z;
    const int zi = tree - lenv * Z;
    const bool tree_on = (lenv < EPW) && sact[lenv];
    const int origin = tree_on ? g.origins[zi] : 0;
    uint64_t* const kt = skeys + tree * KR;
    uint8_t* const ol = sord + tree * NP;
    uint8_t* const pl = spred + tree * NP;
    const uint64_t* const oce = soc + (tree_on ? lenv : 0) * ENV_SLOTS + j * RS;  // lane j's slots of node 0
    const float* const stl = st + (tree_on ? lenv : 0) * E;
    float unassigned_lane = 0.0f;
    TRX_WSTAMP(0);

    for (int it = 0; it < p.iters; ++it) {
        int amb = 0;
        int nscan = 0;
        uint32_t ow[NQ];  // the tree's scan order, four nodes per word (pair-uniform)
        // ---------------- shortest-path tree per lane pair (Dijkstra, sparse relaxation)
        if (tree_on) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {  // lane j's chunks; the origin starts scanned (step 0 below)
                uint64_t kk[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int v = 4 * q + 2 * j + i;
                    kk[i] = (!FULL && v >= N) ? ~0ull : (v == origin ? kScannedW : (kUnreachedW | (uint64_t)v));
                }
                *reinterpret_cast<uint4*>(kt + 4 * q + 2 * j) =
                    make_uint4((uint32_t)kk[0], (uint32_t)(kk[0] >> 32), (uint32_t)kk[1], (uint32_t)(kk[1] >> 32));
                if constexpr (!FULL) {
                    pl[4 * q + 2 * j] = kNoPred;
                    pl[4 * q + 2 * j + 1] = kNoPred;
                }
            }
            ow[0] = (uint32_t)origin;
#pragma unroll
            for (int q = 1; q < NQ; ++q) ow[q] = 0u;
            wave_sync_w();
            uint64_t m[KL];
            // relax u's out-slots of lane j from label bl (FIRST: the origin, label 0:
            // the entry is the key), then issue the next step's key reads behind the
            // atomics (a wave's LDS operations complete in order)
            auto relax = [&](const uint32_t u, const double bl, const bool first, const bool reload) {
                const uint64_t* const er = oce + (int)u * DSP;
                uint64_t en[RS];
#pragma unroll
                for (int r = 0; r < RS; ++r) en[r] = er[r];
                long long nk[RS], was[RS];
                uint32_t hv[RS];
#pragma unroll
                for (int r = 0; r < RS; ++r) {  // the atomics back to back; empty slots (head == u) skip theirs
                    hv[r] = (uint32_t)en[r] & 31u;
                    nk[r] = first ? (long long)en[r]
                                  : (long long)(dbits_w(__dadd_rn(bl, bitsd_w(en[r] & ~31ull))) | hv[r]);
                    was[r] = LLONG_MIN;
                    if (hv[r] != u)
                        was[r] = __hip_atomic_fetch_min(reinterpret_cast<long long*>(kt + hv[r]), nk[r],
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if (reload) read_keys_w<NQ>(kt + 2 * j, m);
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    // scipy's strict improvement: u becomes v's predecessor.  An equal key:
                    // v holds this label from the tail pl[v] already; the tails' labels
                    // are equal (heap order decides: exact replay) iff the costs are
#ifndef TRX_PAIR_NOPRED  // diagnostic variant: predecessor stores left out (wrong results; timing only)
                    if (nk[r] < was[r]) pl[hv[r]] = (uint8_t)u;
#endif
                    if (nk[r] == was[r]) {
                        const int tail = pl[hv[r]];
                        const float ct = stl[seid[(tail << 5) + (int)hv[r]]];
                        amb |= (double)ct == bitsd_w(en[r] & ~31ull);
                    }
                }
            };
            relax((uint32_t)origin, 0.0, true, true);
            nscan = 1;
            bool alive = true;
#pragma unroll
            for (int k = 1; k < NP; ++k) {
                if (FULL || k < N) {  // uniform
                    // argmin over the lane's keys (pairwise v_min_f64), then over the pair (DPP swap)
                    double d[KL];
#pragma unroll
                    for (int i = 0; i < KL; ++i) d[i] = bitsd_w(m[i]);
#pragma unroll
                    for (int w = 1; w < KL; w *= 2)
#pragma unroll
                        for (int i = 0; i + w < KL; i += 2 * w) d[i] = vmin_w(d[i], d[i + w]);
                    const uint64_t b0 = dbits_w(d[0]);
                    const double bd = vmin_w(d[0], bitsd_w(((uint64_t)wdpp<0xB1>((uint32_t)(b0 >> 32)) << 32) |
                                                           wdpp<0xB1>((uint32_t)b0)));
                    // pair-uniform: the rest is unreachable (NaN / +inf: every key ignored)
                    if (!FULL) alive = alive && bd < kInfD;
                    if (FULL || alive) {
                        const uint64_t best = dbits_w(bd);
                        const uint32_t u = (uint32_t)best & 31u;
                        // scanned: the key's high word becomes 0xFFF80000 (a quiet NaN, negative);
                        // both lanes of the pair store the same word
                        reinterpret_cast<uint32_t*>(kt + u)[1] = (uint32_t)(kScannedW >> 32);
                        ow[k >> 2] |= u << (8 * (k & 3));
                        nscan = k + 1;
                        // FULL: the last step's heads are all scanned -- nothing to relax
                        if (FULL ? k + 1 < NP : true) relax(u, bitsd_w(best & ~31ull), false, FULL ? k + 1 < NP : k + 1 < N);
                    }
                }
            }
        }
        wave_sync_w();
        TRX_WSTAMP(1);
        // ---------------- exact scipy-heap replays of the ambiguous trees (every lane of
        // the wave takes part: the heap lives in the wave's registers)
        amb |= (int)wdpp<0xB1>((uint32_t)amb);
        const uint64_t need = __ballot(amb != 0 && j == 0);
#ifdef TRX_PHASE_STAMPS
        if (tid == 0) atomicAdd(&trx_phase_cycles_w[7], (unsigned long long)__popcll(need));  // replayed trees (wave 0)
#endif
        if (need) {  // wave-uniform: the scan orders go through LDS, where the replays rewrite theirs
            if (tree_on && j == 0) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) reinterpret_cast<uint32_t*>(ol)[q] = ow[q];
            }
            wave_sync_w();
            if (__popcll(need) <= kWaveReplays) {  // few: one at a time, the whole wave, heap in registers
                uint64_t pend = need;
                while (pend) {
                    const int bit = __builtin_ctzll(pend);
                    pend &= pend - 1;
                    const int t = (int)(tid >> 6) * 32 + (bit >> 1);  // the tree of pair leader `bit`
                    const int le = t / Z, zt = t - le * Z;
                    replay_tree_pair<RS>(N, soc + le * ENV_SLOTS, g.origins[zt], sord + t * NP, spred + t * NP);
                }
            } else {  // many: each pair leader replays its own tree, kSlots heaps at a time in the
                      // wave's key rows
                constexpr int kHeapBytes = (int)((sizeof(FibSmallW<NP>) + 15) & ~(size_t)15);
                constexpr int kSlots = (32 * KR * 8) / kHeapBytes;
                static_assert(kSlots >= 1, "replay heap does not fit the wave's key rows");
                unsigned char* const area = reinterpret_cast<unsigned char*>(skeys + (size_t)(tid >> 6) * 32 * KR);
                const int lane = tid & 63;
                uint64_t pend = need;
                while (pend) {  // wave-uniform
                    uint64_t batch = 0, mm = pend;
                    for (int c = 0; c < kSlots && mm; ++c) {
                        const uint64_t bb = mm & (~mm + 1);
                        batch |= bb;
                        mm ^= bb;
                    }
                    pend &= ~batch;
                    if ((batch >> lane) & 1ull) {  // my tree (I am its pair leader)
                        const int slot = __popcll(batch & ((1ull << lane) - 1ull));
                        replay_tree_lane<NP, RS>(N, soc + lenv * ENV_SLOTS, origin,
                                                 reinterpret_cast<FibSmallW<NP>*>(area + slot * kHeapBytes), ol, pl);
                    }
                    wave_sync_w();
                }
            }
            wave_sync_w();
            if (tree_on) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) ow[q] = reinterpret_cast<const uint32_t*>(ol)[q];
            }
        }
        TRX_WSTAMP(2);
        // ---------------- all-or-nothing (repair_env.py:490-502, 707-722): subtree demand
        // sums S(v) per tree in reverse scan order, each final S(v) added to the load of
        // v's predecessor link and to the predecessor's S (u32 LDS atomics; integral
        // demands: exact in any order).  The pair takes the scan slots two at a time:
        // lane 0 slot 2g + 1, lane 1 slot 2g; lane 0's S is final when read, lane 1 adds
        // it over a DPP broadcast when lane 0's node is its child.
#ifdef TRX_PAIR_NOSUB  // diagnostic variant: no subtree pass (wrong results; timing only)
        if (false) {
#else
        if (tree_on) {
#endif
            const float* dm = gdem + zi * N;
            uint32_t* const sa = reinterpret_cast<uint32_t*>(kt);  // the key row is dead
            float un = 0.0f;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                uint32_t sv[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int v = 4 * q + 2 * j + i;
                    const float dv = (FULL || v < N) ? dm[v] : 0.0f;
                    const bool load = FULL ? v != origin : (v < N && pl[v] != kNoPred);
                    un += (dv > 0.0f && !load) ? dv : 0.0f;  // intrazonal or unreachable (708)
                    sv[i] = load ? (uint32_t)dv : 0u;         // exact: integral demands < 2^24
                }
                *reinterpret_cast<uint2*>(sa + 4 * q + 2 * j) = make_uint2(sv[0], sv[1]);
            }
            unassigned_lane = un;
            const int ns = FULL ? NP : nscan;
            wave_sync_w();
            uint32_t* const ll = sload + lenv * E;
            const uint32_t sh0 = 8u * (1u - (uint32_t)j);  // my byte of a slot pair: slot 2g + 1 - j
#pragma unroll
            for (int gp = NP / 2 - 1; gp >= 0; --gp) {
                if (2 * gp >= ns) continue;  // pair-uniform (uniform when FULL)
                const int sl = 2 * gp + 1 - j;
                const bool valid = sl >= 1 && sl < ns;
                const bool valid0 = 2 * gp + 1 < ns;  // lane 0's slot
                const uint32_t v = (ow[gp >> 1] >> (sh0 + 16u * (uint32_t)(gp & 1))) & 0xFFu;
                const uint32_t pv = valid ? pl[v] : 0u;
                const uint32_t e = valid ? seid[(pv << 5) + v] : 0u;
                uint32_t S = valid ? sa[v] : 0u;
                const uint32_t S0 = wdpp<0xA0>(S), p0 = wdpp<0xA0>(pv), v1 = wdpp<0xF5>(v);
                if (j == 1 && valid0 && p0 == v) S += S0;             // lane 0's node is my child
                const bool parent_here = j == 0 && gp >= 1 && pv == v1;  // lane 1 takes my S
                if (valid) {
                    atomicAdd(ll + e, S);
                    if (!parent_here) atomicAdd(sa + pv, S);
                }
            }
        }
        __syncthreads();
        TRX_WSTAMP(3);

        // ---------------- flow update + BPR + next out-slot costs (repair_env.py:317-342)
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
            const uint32_t op = sopos[e];
            soc[el * ENV_SLOTS + (op & 0xFFFFu)] = slot_entry(tv, op >> 16);
        }
        __syncthreads();
        TRX_WSTAMP(4);
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
    TRX_WSTAMP(5);
#ifdef TRX_PHASE_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < (1u << 16)) trx_wg_cycles_w[blockIdx.x] = __builtin_amdgcn_s_memtime() - wg_start_;
#endif
}

LaunchCfg pair_launch_cfg(const DevGraph& g, int num_envs, int method) {
    LaunchCfg c{};
    c.np = g.NP;
    const int per_env = g.Z * 2;
    // envs per workgroup: the fewest idle lanes in the block's last wave, then the most
    // envs, among the configurations within 64 KB of LDS
    const int RS = pair_rounds(g);
    const bool cfw = method == TRX_METHOD_CFW;
    int best = 1;
    double best_util = -1.0;
    for (int epw = 1; epw * per_env <= 256; ++epw) {
        const int th = ((epw * per_env + 63) / 64) * 64;
        if (smemw_layout(g.E, g.NP, RS, epw, th / 2, cfw).total > 64 * 1024) break;
        const double util = (double)(epw * per_env) / th;
        if (util > best_util + 1e-9 || (util > best_util - 1e-9 && epw > best)) {
            best = epw;
            best_util = util;
        }
    }
    c.epw = best;
    c.threads = ((c.epw * per_env + 63) / 64) * 64;
    c.smem = smemw_layout(g.E, g.NP, RS, c.epw, c.threads / 2, cfw).total;
    c.blocks = (num_envs + c.epw - 1) / c.epw;
    return c;
}

hipError_t launch_env_kernel_pair(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                  const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                  const uint8_t* env_mask, hipStream_t stream) {
    const LaunchCfg c = pair_launch_cfg(g, num_envs, p.method);
    if (c.blocks == 0) return hipSuccess;
    if (c.threads > 256 || c.smem > 64 * 1024 || g.Z * 2 > 256) return hipErrorInvalidConfiguration;
    const int RS = pair_rounds(g);
    const bool full = g.reach_all != 0 && g.N == g.NP;
    const dim3 grid(c.blocks), block(c.threads);
#define TRX_PAIR_LAUNCH(NPV, RV, FV)                                                                                 \
    hipLaunchKernelGGL((env_kernel_pair<NPV, RV, FV>), grid, block, c.smem, stream, g, p, s, num_envs, c.epw, mode, \
                       action, reward, done, valid, env_mask)
#define TRX_PAIR_RS(NPV, FV)             \
    switch (RS) {                        \
        case 1:                          \
            TRX_PAIR_LAUNCH(NPV, 1, FV); \
            break;                       \
        case 2:                          \
            TRX_PAIR_LAUNCH(NPV, 2, FV); \
            break;                       \
        case 3:                          \
            TRX_PAIR_LAUNCH(NPV, 3, FV); \
            break;                       \
        default:                         \
            TRX_PAIR_LAUNCH(NPV, 4, FV); \
            break;                       \
    }
#define TRX_PAIR_NP(NPV)         \
    if (full) {                  \
        TRX_PAIR_RS(NPV, true)   \
    } else {                     \
        TRX_PAIR_RS(NPV, false)  \
    }
    switch (c.np) {
        case 8:
            TRX_PAIR_NP(8);
            break;
        case 16:
            TRX_PAIR_NP(16);
            break;
        case 24:
            TRX_PAIR_NP(24);
            break;
        default:
            TRX_PAIR_NP(32);
            break;
    }
#undef TRX_PAIR_NP
#undef TRX_PAIR_RS
#undef TRX_PAIR_LAUNCH
    return hipGetLastError();
}

}  // namespace trx

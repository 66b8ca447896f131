// gat_tail.hip -- the acting pass's tail on bf16 MFMA, gfx950: the last GATConv
// of GATEncoder (src/models/gat_encoder.py:22-25, 47-53: heads 1, concat False,
// LayerNorm, ELU, global mean|max pool) and the edge scorer of Actor/Critic
// (src/rl/sac.py:38-46, 69-78) in ONE kernel, four graphs per workgroup.
//
// Through the layer kernels (gat_infer.hip) this tail was 5 launches with four
// HBM round trips: xh = x @ W^T (hipBLASLt) -> trx_gat_layer_infer -> p = emb @
// W_nodes^T, c = ctx @ W_ctx^T (hipBLASLt) -> trx_edge_head_infer.  Here:
//   1. xh^T = W_lin . x^T on v_mfma_f32_16x16x32_bf16: the weights are the A
//      operand, read straight from global memory (a lane's 8 k-values of an
//      output channel are 16 contiguous bytes of the row-major [C, K] weight;
//      the 512 KB matrix stays in every XCD's L2), the graphs' x rows the B
//      operand, staged through LDS in 128-wide K chunks (double-buffered, row
//      stride == 8 dwords mod 64: conflict-free ds_read_b128 fragments).  The
//      transposed product leaves four consecutive channels of one node in a
//      lane, stored as one packed 8-byte bf16 write.
//   2. attention dots, edge softmax, aggregation, bias, LayerNorm, ELU, pool:
//      the arithmetic of gat_layer_infer_kernel, in its order (the pool sums
//      the graph's nodes in node order across the two waves of the graph).
//   3. c = bf16(bf16(ctx) @ W_ctx^T) + b1 and p = bf16(bf16(y) @ W_nodes^T) on
//      MFMA (p in four blocks of 64 hidden units, src and dst halves), each
//      block consumed by the edge scorer at once: one lane per link, the
//      per-hidden-unit terms of edge_head_infer_kernel and its summation tree
//      (4 units per partial, 16 partials per 64 units pairwise, the four
//      64-unit totals as (T0 + T1) + (T2 + T3)), then the masked softmax and
//      the categorical draw of edge_head_infer_kernel.
// Results equal the layer-kernel path except where hipBLASLt's and this
// kernel's fp32 GEMM accumulation orders round a bf16 output differently.
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kW = 64;
constexpr int kTG = 4;              // graphs per workgroup
constexpr int kTWaves = 8;
constexpr int kTThreads = kTWaves * kW;
constexpr int kTC = 256;            // channels of the last layer == hidden units of the edge MLP
constexpr int kKC = 128;            // GEMM1 K chunk
constexpr int kAS = kKC + 16;       // staged x row stride (bf16): 72 dwords == 8 (mod 64)
constexpr int kXS = kTC + 16;       // xh / emb row stride: 136 dwords == 8 (mod 64)
constexpr int kPS = 128 + 16;       // p block row stride: 64 src + 64 dst units
constexpr int kCS = 2 * kTC + 16;   // ctx row stride: 264 dwords == 8 (mod 64)
constexpr int kTED = 8;             // edge_dim <= 8

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float trx_f2t __attribute__((ext_vector_type(2)));
typedef __bf16 trx_b2t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
    const trx_f2t v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, trx_b2t));
}
__device__ __forceinline__ float bfr(float x) {
    return __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x) << 16);
}
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ bf16x8 ldg8(const uint16_t* p) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ bf16x8 lds8(const uint16_t* p) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

#define TRX_TDPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, false))
#define TRX_TDPPM(v, ctrl) \
    __int_as_float(__builtin_amdgcn_update_dpp((int)0xff800000, __float_as_int(v), ctrl, 0xf, 0xf, false))
// the reductions of gat_infer.hip (same trees, so the same sums)
__device__ __forceinline__ float t_row_sum16(float v) {
    v = v + TRX_TDPP(v, 0xB1);
    v = v + TRX_TDPP(v, 0x4E);
    v = v + TRX_TDPP(v, 0x141);
    v = v + TRX_TDPP(v, 0x140);
    return v;
}
__device__ __forceinline__ float t_wave_sum(float v) {
    v = t_row_sum16(v);
    return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
           (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}
__device__ __forceinline__ float t_wave_max(float v) {
    v = fmaxf(v, TRX_TDPPM(v, 0xB1));
    v = fmaxf(v, TRX_TDPPM(v, 0x4E));
    v = fmaxf(v, TRX_TDPPM(v, 0x141));
    v = fmaxf(v, TRX_TDPPM(v, 0x140));
    return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))),
                 fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48))));
}
#undef TRX_TDPP
#undef TRX_TDPPM

struct TailSmem {
    uint32_t U, X, as_, ad_, rp, cl, dlc, al, cs, wes, w2s, lg, mk, eal, lsd, tsum, bad, total;
};

__host__ __device__ inline uint32_t al16t(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline TailSmem tail_smem(int MT, int n, int E, int me) {
    const int R = 16 * MT;
    TailSmem o{};
    uint32_t off = 0;
    auto take = [&off](uint32_t b) {
        const uint32_t r = off;
        off = al16t(off + b);
        return r;
    };
    // U: GEMM1 staging | pool partials (odd-half y rows) + ctx rows | one p block
    uint32_t u = 2u * R * kAS * 2;
    const uint32_t ypart = (uint32_t)kTG * ((n + 1) / 2) * kTC * 4;
    const uint32_t pool = al16t(ypart) + 16u * kCS * 2;
    if (pool > u) u = pool;
    if ((uint32_t)R * kPS * 2 > u) u = (uint32_t)R * kPS * 2;
    o.U = take(u);
    o.X = take((uint32_t)R * kXS * 2);
    o.as_ = take((uint32_t)R * 4);
    o.ad_ = take((uint32_t)R * 4);
    o.rp = take((uint32_t)(R + 1) * 4);
    o.cl = take((uint32_t)kTG * me * 4);
    o.dlc = take((uint32_t)kTG * me * 4);
    o.al = take((uint32_t)kTG * me * 4);
    o.cs = take((uint32_t)kTG * kTC * 4);
    o.wes = take((uint32_t)kTC * kTED * 4);
    o.w2s = take((uint32_t)kTC * 4);
    o.lg = take((uint32_t)kTG * E * 4);
    o.mk = take((uint32_t)kTG * E * 4);
    o.eal = take((uint32_t)kTG * E * kTED * 4);
    o.lsd = take((uint32_t)kTG * E * 2 * 4);
    o.tsum = take((uint32_t)kTG * E * 4 * 4);
    o.bad = take((uint32_t)(kTG + 1) * 4);
    o.total = off;
    return o;
}

}  // namespace

#ifdef TRX_PHASE_STAMPS
// Diagnostic build only (make stamps): per-phase cycle totals of thread 0 of
// each workgroup (input, GEMM1, attention, aggregate+pool, ctx GEMM, p+scorer, outputs).
__device__ unsigned long long trx_tail_cycles[8];
#define TRX_TSTAMP(slot)                                                    \
    do {                                                                    \
        if (threadIdx.x == 0) {                                             \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
            atomicAdd(&trx_tail_cycles[slot], now_ - stamp_prev_);          \
            stamp_prev_ = now_;                                             \
        }                                                                   \
    } while (0)
extern "C" int trx_debug_tail_cycles(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_tail_cycles), sizeof(unsigned long long) * 8) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(trx_tail_cycles), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define TRX_TSTAMP(slot) \
    do {                 \
    } while (0)
#endif

// MT: 16-row node tiles per workgroup (4 graphs * nodes_per_graph <= 16 * MT)
template <int MT>
__global__ void __launch_bounds__(kTThreads) gat_tail_kernel(trx_gat_tail_args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int R = 16 * MT;
    const int n = a.nodes_per_graph, E = a.edges_per_graph, K = a.in_dim, D = a.edge_dim, me = a.max_graph_edges;
    const int tid = threadIdx.x, lane = tid & (kW - 1), wave = tid / kW;
    const int g0 = blockIdx.x * kTG;
    const int G = a.num_graphs - g0 < kTG ? a.num_graphs - g0 : kTG;
    const int nrow = G * n;
    const int64_t node0 = (int64_t)g0 * n;
    const TailSmem O = tail_smem(MT, n, E, me);
#ifdef TRX_PHASE_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif
    uint16_t* const As = reinterpret_cast<uint16_t*>(smem + O.U);
    uint16_t* const xs = reinterpret_cast<uint16_t*>(smem + O.X);
    float* const as_ = reinterpret_cast<float*>(smem + O.as_);
    float* const ad_ = reinterpret_cast<float*>(smem + O.ad_);
    int* const rp = reinterpret_cast<int*>(smem + O.rp);
    int* const cl = reinterpret_cast<int*>(smem + O.cl);
    int* const dlc = reinterpret_cast<int*>(smem + O.dlc);
    float* const al = reinterpret_cast<float*>(smem + O.al);
    float* const cs = reinterpret_cast<float*>(smem + O.cs);
    float* const wes = reinterpret_cast<float*>(smem + O.wes);
    float* const w2s = reinterpret_cast<float*>(smem + O.w2s);
    float* const lgs = reinterpret_cast<float*>(smem + O.lg);
    float* const mks = reinterpret_cast<float*>(smem + O.mk);
    int* const bad = reinterpret_cast<int*>(smem + O.bad);
    float* const eal = reinterpret_cast<float*>(smem + O.eal);   // [kTG][E][kTED] link features (fp32)
    int* const lsd = reinterpret_cast<int*>(smem + O.lsd);       // [kTG][E][2] workgroup-local endpoints
    float* const tsum = reinterpret_cast<float*>(smem + O.tsum); // [kTG][E][4] 64-unit row sums

    // ---------------------------------------------- small inputs (into LDS)
    const int ebeg = a.rowptr[node0];
    const int ne = a.rowptr[node0 + nrow] - ebeg;  // CSR positions of the workgroup's graphs
    if (tid <= kTG) bad[tid] = 0;
    for (int i = tid; i <= nrow; i += kTThreads) rp[i] = a.rowptr[node0 + i] - ebeg;
    const bool csr_ok = ne >= 0 && ne <= kTG * me;
    if (csr_ok)
        for (int p = tid; p < ne; p += kTThreads) {
            cl[p] = a.col[ebeg + p] - (int)node0;
            al[p] = a.a_edge[(size_t)(ebeg + p) * a.a_edge_stride + a.a_edge_offset];
        }
    for (int v = tid; v < kTC * kTED; v += kTThreads) {
        const int k = v / kTED, j = v - k * kTED;
        wes[v] = j < D ? a.we[k * D + j] : 0.0f;
    }
    for (int k = tid; k < kTC; k += kTThreads) w2s[k] = a.w2[k];
    __syncthreads();  // bad[] cleared
    for (int v = tid; v < G * E; v += kTThreads) {
        const int gl = v / E;
        const int64_t eg = (int64_t)g0 * E + v, base = (int64_t)(g0 + gl) * n;
        const int64_t s = a.src[eg] - base, d = a.dst[eg] - base;
        const bool okl = s >= 0 && s < n && d >= 0 && d < n;  // else: poison the graph, never read outside LDS
        if (!okl) atomicOr(&bad[gl], 1);
        lsd[2 * v] = okl ? gl * n + (int)s : 0;
        lsd[2 * v + 1] = okl ? gl * n + (int)d : 0;
#pragma unroll
        for (int j = 0; j < kTED; ++j) eal[kTED * v + j] = j < D ? a.ea[eg * D + j] : 0.0f;
    }

    TRX_TSTAMP(0);
    // ---------------------------------------------- 1. xh^T = W_lin . x^T (MFMA)
    constexpr int SU = R * 16 / kTThreads;  // 16-byte staging units per thread per chunk
    const uint16_t* const xg = static_cast<const uint16_t*>(a.x) + node0 * K;
    const uint16_t* const wl = static_cast<const uint16_t*>(a.w_lin);
    auto load_chunk = [&](u32x4 (&st)[SU], int s) {
#pragma unroll
        for (int j = 0; j < SU; ++j) {
            const int idx = tid + kTThreads * j, row = idx >> 4, un = idx & 15;
            st[j] = row < nrow ? *reinterpret_cast<const u32x4*>(xg + (size_t)row * K + s * kKC + un * 8)
                               : u32x4{0u, 0u, 0u, 0u};
        }
    };
    auto store_chunk = [&](const u32x4 (&st)[SU], int buf) {
#pragma unroll
        for (int j = 0; j < SU; ++j) {
            const int idx = tid + kTThreads * j, row = idx >> 4, un = idx & 15;
            *reinterpret_cast<u32x4*>(As + (size_t)buf * R * kAS + row * kAS + un * 8) = st[j];
        }
    };
    const int ot0 = 2 * wave;  // this wave's two 16-channel tiles
    const uint16_t* const wr0 = wl + (size_t)(16 * ot0 + (lane & 15)) * K + 8 * (lane >> 4);
    const uint16_t* const wr1 = wr0 + (size_t)16 * K;
    f32x4 acc[2][MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[0][m] = acc[1][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 wa[4][2], wnx[4][2];
    const int NS = K / kKC;
    u32x4 stA[SU], stB[SU];  // x chunks in flight: two ahead of the one being multiplied
    load_chunk(stA, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        wa[ks][0] = ldg8(wr0 + ks * 32);
        wa[ks][1] = ldg8(wr1 + ks * 32);
    }
    store_chunk(stA, 0);
    if (NS > 1) load_chunk(stA, 1);
    __syncthreads();
    // one K chunk: `cur` holds chunk s+1 (in flight since the previous chunk), chunk s+2 goes to `nxt`
    auto chunk = [&](int s, u32x4 (&cur)[SU], u32x4 (&nxt)[SU]) {
        const int buf = s & 1;
        const bool more = s + 1 < NS;
        if (s + 2 < NS) load_chunk(nxt, s + 2);
        if (more) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                wnx[ks][0] = ldg8(wr0 + (s + 1) * kKC + ks * 32);
                wnx[ks][1] = ldg8(wr1 + (s + 1) * kKC + ks * 32);
            }
        }
        const uint16_t* const ab = As + (size_t)buf * R * kAS + (lane & 15) * kAS + 8 * (lane >> 4);
        bf16x8 xb[2][MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) xb[0][m] = lds8(ab + 16 * m * kAS);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            if (ks + 1 < 4)
#pragma unroll
                for (int m = 0; m < MT; ++m) xb[(ks + 1) & 1][m] = lds8(ab + 16 * m * kAS + (ks + 1) * 32);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                acc[0][m] = mfma(wa[ks][0], xb[ks & 1][m], acc[0][m]);
                acc[1][m] = mfma(wa[ks][1], xb[ks & 1][m], acc[1][m]);
            }
        }
        if (more) {
            store_chunk(cur, buf ^ 1);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                wa[ks][0] = wnx[ks][0];
                wa[ks][1] = wnx[ks][1];
            }
        }
        __syncthreads();
    };
    for (int s = 0; s < NS; s += 2) {
        chunk(s, stA, stB);
        if (s + 1 < NS) chunk(s + 1, stB, stA);
    }
    // bf16 xh rows (the lin output's rounding point): lane = node, four channels
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const int node = 16 * m + (lane & 15), o = 16 * (ot0 + t) + 4 * (lane >> 4);
            uint2 u;
            u.x = pk2(acc[t][m][0], acc[t][m][1]);
            u.y = pk2(acc[t][m][2], acc[t][m][3]);
            *reinterpret_cast<uint2*>(xs + node * kXS + o) = u;
        }
    if (csr_ok)
        for (int i = tid; i < nrow; i += kTThreads) {
            // the aggregation keeps a node's in-edges one per lane: more than 64 poison the graph
            if (rp[i + 1] - rp[i] > kW) atomicOr(&bad[i / n], 1);
            for (int p = rp[i]; p < rp[i + 1]; ++p) dlc[p] = i;
        }
    __syncthreads();

    TRX_TSTAMP(1);
    // ---------------------------------------------- 2. attention (gat_infer.hip order)
    if (!csr_ok) {  // LDS was sized for max_graph_edges per graph: poison, never overrun
        for (int v = tid; v < G * E; v += kTThreads) {
            a.out[(size_t)g0 * E + v] = __builtin_nanf("");
            if (a.softmax && a.logits) a.logits[(size_t)g0 * E + v] = __builtin_nanf("");
        }
        if (a.softmax && a.u && tid < G) a.action[g0 + tid] = 0;
        return;
    }
    {   // <xh[i], att_src>, <xh[i], att_dst>: four nodes per wave at a time, lane owns channels 4*sl + 64*m
        const int sub = lane >> 4, sl = lane & 15;
        float4 sa[4], da[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            sa[m] = *reinterpret_cast<const float4*>(a.att_src + 4 * sl + 64 * m);
            da[m] = *reinterpret_cast<const float4*>(a.att_dst + 4 * sl + 64 * m);
        }
        for (int i0 = 4 * wave; i0 < nrow; i0 += 4 * kTWaves) {
            const int i = i0 + sub;
            const bool ok = i < nrow;
            float s1 = 0.0f, s2 = 0.0f;
            if (ok) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const uint2 u = *reinterpret_cast<const uint2*>(xs + i * kXS + 4 * sl + 64 * m);
                    const float v0 = lo_bf(u.x), v1 = hi_bf(u.x), v2 = lo_bf(u.y), v3 = hi_bf(u.y);
                    s1 += (v0 * sa[m].x + v1 * sa[m].y) + (v2 * sa[m].z + v3 * sa[m].w);
                    s2 += (v0 * da[m].x + v1 * da[m].y) + (v2 * da[m].z + v3 * da[m].w);
                }
            }
            s1 = t_row_sum16(s1);
            s2 = t_row_sum16(s2);
            if (ok && sl == 0) {
                as_[i] = s1;
                ad_[i] = s2;
            }
        }
    }
    __syncthreads();
    for (int p = tid; p < ne; p += kTThreads) {
        const float x = as_[cl[p]] + ad_[dlc[p]] + al[p];
        al[p] = x > 0.0f ? x : x * a.negative_slope;
    }
    __syncthreads();
    for (int i = tid; i < nrow; i += kTThreads) {
        const int p0 = rp[i], p1 = rp[i + 1];
        float m = -__builtin_huge_valf();
        for (int p = p0; p < p1; ++p) m = fmaxf(m, al[p]);
        float ssum = 0.0f;
        for (int p = p0; p < p1; ++p) {
            const float ex = __expf(al[p] - m);
            al[p] = ex;
            ssum += ex;
        }
        ad_[i] = ssum + 1e-16f;
    }
    __syncthreads();
    for (int p = tid; p < ne; p += kTThreads) al[p] = al[p] / ad_[dlc[p]];
    __syncthreads();

    TRX_TSTAMP(2);
    // ---------------------------------------------- 3. aggregation, LayerNorm, ELU, pool
    // graph gw = wave / 2; the even wave takes nodes [0, h), the odd one [h, n)
    const int gw = wave >> 1, par = wave & 1;
    const int h = (n + 1) / 2;
    const int i_lo = par ? h : 0, i_hi = par ? n : h;
    float* const ypart = reinterpret_cast<float*>(smem + O.U);  // [kTG][h][kTC] the odd waves' y rows
    const int f0 = 4 * lane;
    const float4 bias4 = *reinterpret_cast<const float4*>(a.bias + f0);
    const float4 lnw4 = *reinterpret_cast<const float4*>(a.ln_weight + f0);
    const float4 lnb4 = *reinterpret_cast<const float4*>(a.ln_bias + f0);
    const float bias_r[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
    const float lnw_r[4] = {lnw4.x, lnw4.y, lnw4.z, lnw4.w};
    const float lnb_r[4] = {lnb4.x, lnb4.y, lnb4.z, lnb4.w};
    constexpr int kMaxHalf = 16;  // nodes_per_graph <= 32
    float ysv[kMaxHalf][4];
    float psum[4] = {0.f, 0.f, 0.f, 0.f}, pmax[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pmax[r] = -__builtin_huge_valf();
    const bool gon = gw < G;
    // CSR metadata lane-parallel: lane j holds row start j of this wave's nodes;
    // per node the (source, weight) pairs sit one per lane, fetched a node ahead
    const int cnt = gon ? i_hi - i_lo : 0;
    const int nb = gw * n + i_lo;
    const int rpl = lane <= cnt ? rp[nb + lane] : 0;
    int mc = 0;
    float mw = 0.0f;
    if (cnt > 0) {
        const int q0 = __builtin_amdgcn_readlane(rpl, 0), q1 = __builtin_amdgcn_readlane(rpl, 1);
        mc = lane < q1 - q0 ? cl[q0 + lane] : 0;
        mw = lane < q1 - q0 ? al[q0 + lane] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < kMaxHalf; ++j) {  // compile-time trip count: ysv stays in registers
        if (j >= cnt) continue;
        const int node = nb + j;
        const int deg = min(__builtin_amdgcn_readlane(rpl, j + 1) - __builtin_amdgcn_readlane(rpl, j), kW);
        const int cc = mc;
        const float cw = mw;
        if (j + 1 < cnt) {
            const int q0 = __builtin_amdgcn_readlane(rpl, j + 1), q1 = __builtin_amdgcn_readlane(rpl, j + 2);
            mc = lane < q1 - q0 ? cl[q0 + lane] : 0;
            mw = lane < q1 - q0 ? al[q0 + lane] : 0.0f;
        }
        float acc4[4] = {0.f, 0.f, 0.f, 0.f};
        auto fma_row = [&](uint2 u, float w) {
            acc4[0] = __builtin_fmaf(w, lo_bf(u.x), acc4[0]);  // the layer kernel's fused multiply-adds
            acc4[1] = __builtin_fmaf(w, hi_bf(u.x), acc4[1]);
            acc4[2] = __builtin_fmaf(w, lo_bf(u.y), acc4[2]);
            acc4[3] = __builtin_fmaf(w, hi_bf(u.y), acc4[3]);
        };
        int e = 0;
        for (; e + 4 <= deg; e += 4) {  // four rows in flight, summed in CSR order
            uint2 u[4];
            float w[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int sn = __builtin_amdgcn_readlane(cc, e + t);
                w[t] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cw), e + t));
                u[t] = *reinterpret_cast<const uint2*>(xs + sn * kXS + f0);
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) fma_row(u[t], w[t]);
        }
        for (; e < deg; ++e) {
            const int sn = __builtin_amdgcn_readlane(cc, e);
            const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cw), e));
            fma_row(*reinterpret_cast<const uint2*>(xs + sn * kXS + f0), w);
        }
        float v[4];
        float s = 0.0f;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc4[r] + bias_r[r];
        s += (v[0] + v[1]) + (v[2] + v[3]);
        const float mean = t_wave_sum(s) / (float)kTC;
        float s2 = 0.0f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float d = v[r] - mean;
            s2 += d * d;
        }
        const float rstd = rsqrtf(t_wave_sum(s2) / (float)kTC + a.ln_eps);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float y = __builtin_fmaf(lnw_r[r], rstd * (v[r] - mean), lnb_r[r]);
            y = y <= 0.0f ? (expf(y) - 1.0f) : y;
            ysv[j][r] = y;
            if (!par) {
                psum[r] += y;
                pmax[r] = fmaxf(pmax[r], y);
            }
        }
        if (par)
            *reinterpret_cast<float4*>(ypart + ((size_t)gw * h + j) * kTC + f0) =
                make_float4(ysv[j][0], ysv[j][1], ysv[j][2], ysv[j][3]);
        (void)node;
    }
    __syncthreads();  // every xh read done; the odd halves' y rows are in LDS
    uint16_t* const ctxb = reinterpret_cast<uint16_t*>(smem + O.U + al16t((uint32_t)kTG * h * kTC * 4));
    if (gon && !par) {  // the pool in node order: own rows, then the odd wave's
        for (int j = 0; j < n - h; ++j) {
            const float4 y4 = *reinterpret_cast<const float4*>(ypart + ((size_t)gw * h + j) * kTC + f0);
            const float yv[4] = {y4.x, y4.y, y4.z, y4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                psum[r] += yv[r];
                pmax[r] = fmaxf(pmax[r], yv[r]);
            }
        }
        float mean4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) mean4[r] = psum[r] / (float)n;
        if (a.pool) {
            float* pg = a.pool + (size_t)(g0 + gw) * 2 * kTC;
            *reinterpret_cast<float4*>(pg + f0) = make_float4(mean4[0], mean4[1], mean4[2], mean4[3]);
            *reinterpret_cast<float4*>(pg + kTC + f0) = make_float4(pmax[0], pmax[1], pmax[2], pmax[3]);
        }
        uint2 u;
        u.x = pk2(mean4[0], mean4[1]);
        u.y = pk2(mean4[2], mean4[3]);
        *reinterpret_cast<uint2*>(ctxb + gw * kCS + f0) = u;
        u.x = pk2(pmax[0], pmax[1]);
        u.y = pk2(pmax[2], pmax[3]);
        *reinterpret_cast<uint2*>(ctxb + gw * kCS + kTC + f0) = u;
    }
    // emb = bf16(y) over the xh rows (LDS), and to HBM when asked
#pragma unroll
    for (int j = 0; j < kMaxHalf; ++j) {
        const int i = i_lo + j;
        if (!gon || i >= i_hi) continue;
        const int node = gw * n + i;
        uint2 u;
        u.x = pk2(ysv[j][0], ysv[j][1]);
        u.y = pk2(ysv[j][2], ysv[j][3]);
        *reinterpret_cast<uint2*>(xs + node * kXS + f0) = u;
        if (a.emb_bf16) *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.emb_bf16) + (node0 + node) * kTC + f0) = u;
    }
    __syncthreads();

    TRX_TSTAMP(3);
    // ---------------------------------------------- 4. c = bf16(bf16(ctx) @ W_ctx^T) + b1 (MFMA)
    {
        const uint16_t* const wc = static_cast<const uint16_t*>(a.w_ctx);  // [kTC][2*kTC]
        f32x4 cacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        const int gl = lane & 15;
        const uint16_t* const c0 = wc + (size_t)(16 * ot0 + gl) * 2 * kTC + 8 * (lane >> 4);
        const uint16_t* const c1 = c0 + (size_t)16 * 2 * kTC;
        const uint16_t* const xb = ctxb + gl * kCS + 8 * (lane >> 4);
#pragma unroll
        for (int ks = 0; ks < 2 * kTC / 32; ++ks) {
            const bf16x8 b = gl < G ? lds8(xb + 32 * ks) : __builtin_bit_cast(bf16x8, u32x4{0u, 0u, 0u, 0u});
            cacc[0] = mfma(ldg8(c0 + 32 * ks), b, cacc[0]);
            cacc[1] = mfma(ldg8(c1 + 32 * ks), b, cacc[1]);
        }
        if (gl < G)
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int k = 16 * (ot0 + t) + 4 * (lane >> 4) + i;
                    cs[gl * kTC + k] = bfr(cacc[t][i]) + a.b1[k];
                }
    }

    TRX_TSTAMP(4);
    // ---------------------------------------------- 5. p blocks (MFMA) + edge scorer
    // the edge scorer of edge_head_infer_kernel with its lane -> hidden-unit map:
    // a 16-lane row holds one link, lane sl the units 64b + 4sl .. +3 (its
    // weights in registers), and the row's DPP sum is that kernel's row sum;
    // a graph's two waves x four rows take 8 links per round
    uint16_t* const pb = reinterpret_cast<uint16_t*>(smem + O.U);  // [R][kPS] one block of p
    const uint16_t* const wnb = static_cast<const uint16_t*>(a.w_nodes);  // [2*kTC][kTC]
    // wave w: output tile w of the block (w < 4: src units 64b + 16w, else dst units)
    const int orow_base = (wave < 4 ? 0 : kTC) + 16 * (wave & 3) + (lane & 15);
    const int pcol = (wave < 4 ? 0 : 64) + 16 * (wave & 3) + 4 * (lane >> 4);
    const int r4 = lane >> 4, sl = lane & 15;
    const int nit = (E + 7) / 8;
    bf16x8 wv[kTC / 32];  // this block's W_nodes fragments, fetched during the previous block's scorer
#pragma unroll
    for (int ks = 0; ks < kTC / 32; ++ks) wv[ks] = ldg8(wnb + (size_t)orow_base * kTC + 8 * (lane >> 4) + 32 * ks);
    for (int b = 0; b < 4; ++b) {
        __syncthreads();  // previous block's p reads (and the ctx / ypart reads) done
        f32x4 pacc[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) pacc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
        const uint16_t* const eb = xs + (lane & 15) * kXS + 8 * (lane >> 4);
#pragma unroll
        for (int ks = 0; ks < kTC / 32; ++ks)
#pragma unroll
            for (int m = 0; m < MT; ++m) pacc[m] = mfma(wv[ks], lds8(eb + 16 * m * kXS + 32 * ks), pacc[m]);
        if (b + 1 < 4)
#pragma unroll
            for (int ks = 0; ks < kTC / 32; ++ks)
                wv[ks] = ldg8(wnb + (size_t)(orow_base + 64 * (b + 1)) * kTC + 8 * (lane >> 4) + 32 * ks);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const int node = 16 * m + (lane & 15);
            uint2 u;
            u.x = pk2(pacc[m][0], pacc[m][1]);
            u.y = pk2(pacc[m][2], pacc[m][3]);
            *reinterpret_cast<uint2*>(pb + node * kPS + pcol) = u;
        }
        __syncthreads();
        if (gon) {
            float we_r[4][kTED], w2_r[4], c_r[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = 64 * b + 4 * sl + r;
                const float4 w0 = *reinterpret_cast<const float4*>(wes + k * kTED);
                const float4 w1 = *reinterpret_cast<const float4*>(wes + k * kTED + 4);
                we_r[r][0] = w0.x; we_r[r][1] = w0.y; we_r[r][2] = w0.z; we_r[r][3] = w0.w;
                we_r[r][4] = w1.x; we_r[r][5] = w1.y; we_r[r][6] = w1.z; we_r[r][7] = w1.w;
                w2_r[r] = w2s[k];
                c_r[r] = cs[gw * kTC + k];
            }
            for (int it = 0; it < nit; ++it) {
                const int e = 8 * it + 4 * par + r4;
                const int v = gw * E + (e < E ? e : E - 1);
                const int2 ud = *reinterpret_cast<const int2*>(lsd + 2 * v);
                const float4 e0 = *reinterpret_cast<const float4*>(eal + kTED * v);
                const float4 e1 = *reinterpret_cast<const float4*>(eal + kTED * v + 4);
                const float ear[kTED] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
                const uint2 su = *reinterpret_cast<const uint2*>(pb + ud.x * kPS + 4 * sl);
                const uint2 du = *reinterpret_cast<const uint2*>(pb + ud.y * kPS + 64 + 4 * sl);
                const float psv[4] = {lo_bf(su.x), hi_bf(su.x), lo_bf(su.y), hi_bf(su.y)};
                const float pdv[4] = {lo_bf(du.x), hi_bf(du.x), lo_bf(du.y), hi_bf(du.y)};
                float part = 0.0f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float ew = 0.0f;  // edge_head_infer_kernel's fused multiply-adds, same order
#pragma unroll
                    for (int j = 0; j < kTED; ++j)
                        if (j < D) ew = __builtin_fmaf(ear[j], we_r[r][j], ew);
                    const float z = ((psv[r] + pdv[r]) + ew) + c_r[r];   // fp32 after the p GEMM
                    part = __builtin_fmaf(fmaxf(z, 0.0f), w2_r[r], part);
                }
                part = t_row_sum16(part);
                if (sl == 0 && e < E) tsum[4 * v + b] = part;
            }
        }
    }
    __syncthreads();
    for (int v = tid; v < G * E; v += kTThreads) {
        const float4 t = *reinterpret_cast<const float4*>(tsum + 4 * v);
        lgs[v] = ((t.x + t.y) + (t.z + t.w)) + a.b2[0];
    }
    __syncthreads();

    TRX_TSTAMP(5);
    // ---------------------------------------------- 6. outputs (edge_head_infer_kernel's tail)
    if (!gon || par) return;
    const int g = g0 + gw;
    float* const lg = lgs + gw * E;
    float* const mk = mks + gw * E;
    if (bad[gw]) {
        for (int x = lane; x < E; x += kW) {
            a.out[(int64_t)g * E + x] = __builtin_nanf("");
            if (a.softmax && a.logits) a.logits[(int64_t)g * E + x] = __builtin_nanf("");
        }
        if (a.softmax && a.u && lane == 0) a.action[g] = 0;
        return;
    }
    if (!a.softmax) {
        for (int x = lane; x < E; x += kW) a.out[(int64_t)g * E + x] = lg[x];
        return;
    }
    for (int x = lane; x < E; x += kW) lg[x] = a.mask[(int64_t)g * E + x] <= 0.0f ? -1e9f : lg[x];
    if (a.logits)
        for (int x = lane; x < E; x += kW) a.logits[(int64_t)g * E + x] = lg[x];
    float mx = -__builtin_huge_valf();
    for (int x0 = 0; x0 < E; x0 += kW) mx = fmaxf(mx, t_wave_max(x0 + lane < E ? lg[x0 + lane] : -__builtin_huge_valf()));
    float ssum = 0.0f;
    for (int x0 = 0; x0 < E; x0 += kW) {
        const int x = x0 + lane;
        const float ex = x < E ? expf(lg[x] - mx) : 0.0f;
        if (x < E) mk[x] = ex;
        ssum += t_wave_sum(ex);
    }
    const float denom = ssum + 1e-16f;
    for (int x = lane; x < E; x += kW) a.out[(int64_t)g * E + x] = mk[x] / denom;
    if (a.u) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) {
            const float target = a.u[g] * ssum;
            float accs = 0.0f;
            int pick = -1, last = 0;
            for (int x = 0; x < E; ++x) {
                const float ex = mk[x];
                if (ex > 0.0f) last = x;
                accs += ex;
                if (pick < 0 && accs > target) pick = x;
            }
            a.action[g] = pick >= 0 ? pick : last;
        }
    }
}

size_t gat_tail_smem(const trx_gat_tail_args& a) {
    const int MT = gat_tail_mtiles(a.nodes_per_graph);
    return tail_smem(MT, a.nodes_per_graph, a.edges_per_graph, a.max_graph_edges).total;
}

int gat_tail_mtiles(int nodes_per_graph) {
    const int rows = kTG * nodes_per_graph;
    return ((rows + 31) / 32) * 2;  // even: the staging deals R*16 units over 512 threads
}

template <int MT>
static hipError_t launch_tail(const trx_gat_tail_args& a, size_t smem, hipStream_t stream) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gat_tail_kernel<MT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const int blocks = (a.num_graphs + kTG - 1) / kTG;
    hipLaunchKernelGGL(gat_tail_kernel<MT>, dim3(blocks), dim3(kTThreads), smem, stream, a);
    return hipGetLastError();
}

hipError_t launch_gat_tail_infer(const trx_gat_tail_args& a, hipStream_t stream) {
    const size_t smem = gat_tail_smem(a);
    switch (gat_tail_mtiles(a.nodes_per_graph)) {
        case 2: return launch_tail<2>(a, smem, stream);
        case 4: return launch_tail<4>(a, smem, stream);
        case 6: return launch_tail<6>(a, smem, stream);
        default: return launch_tail<8>(a, smem, stream);
    }
}

}  // namespace trx

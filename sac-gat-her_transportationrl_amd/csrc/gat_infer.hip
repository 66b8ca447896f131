// gat_infer.hip -- fused GAT-SAC inference for acting on gfx950.
//
// The acting pass of the trainer evaluates the Actor (src/rl/sac.py:35-46:
// input LayerNorms -> GATEncoder -> edge scorer -> masked softmax) on 4096
// Sioux-Falls-sized graphs per step.  Through torch ops every GAT layer
// materialises ~10 [98304 x 1024] fp32 intermediates (lin output cast, the
// attention dot products, aggregate, + bias, LayerNorm, residual, ReLU, the
// cast for the next GEMM): HBM-bound at ~2 ms per layer.  Here each layer is
// one kernel, one workgroup per graph:
//   1. stage the graph's xh rows (n x H*C bf16, <= 64 KB) in LDS -- for layer 0
//      xh = bf16(x0 @ w0^T) is computed from the 4 raw features instead;
//   2. a_src / a_dst = <xh, att> per (node, head): one wave per pair;
//   3. attention softmax over each node's in-edges (lanes = edges), exactly
//      the arithmetic of gat_fwd_kernel (gat_kernel.hip);
//   4. aggregation from LDS (one wave per node, lane owns float4 columns),
//      + bias, LayerNorm (wave reductions), residual, ReLU/ELU, bf16 / fp32
//      stores, and on the last layer the global mean|max pool.
// HBM traffic per layer is one read of xh plus the output write.
//
// The edge scorer (second kernel) evaluates, per link, the factored first
// edge-MLP layer (see sac.py docstring), ReLU, the 256->1 projection and the
// per-graph masked softmax, without materialising the [E, 256] hidden.
// bf16 roundings are applied where the bf16-autocast torch path rounds, so
// the two paths agree to bf16 precision (tests/test_gat_infer.py).
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kWave = 64;
constexpr int kInferThreads = 256;
constexpr int kInferWaves = kInferThreads / kWave;

// Wave-wide reductions on DPP + readlane (no LDS round trips): quad butterflies
// (xor 1, xor 2), half-row and row mirrors give every lane its 16-lane row
// total; the four row totals are combined from lanes 0/16/32/48.
#define TRX_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, false))
__device__ __forceinline__ float wave_sum_f(float v) {
    v = v + TRX_DPP(v, 0xB1);   // quad_perm [1,0,3,2]
    v = v + TRX_DPP(v, 0x4E);   // quad_perm [2,3,0,1]
    v = v + TRX_DPP(v, 0x141);  // row_half_mirror
    v = v + TRX_DPP(v, 0x140);  // row_mirror
    return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
           (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}
// every lane gets the total of its 16-lane row
__device__ __forceinline__ float row_sum16_f(float v) {
    v = v + TRX_DPP(v, 0xB1);
    v = v + TRX_DPP(v, 0x4E);
    v = v + TRX_DPP(v, 0x141);
    v = v + TRX_DPP(v, 0x140);
    return v;
}
#define TRX_DPPM(v, ctrl) \
    __int_as_float(__builtin_amdgcn_update_dpp((int)0xff800000, __float_as_int(v), ctrl, 0xf, 0xf, false))
__device__ __forceinline__ float wave_max_f(float v) {
    v = fmaxf(v, TRX_DPPM(v, 0xB1));
    v = fmaxf(v, TRX_DPPM(v, 0x4E));
    v = fmaxf(v, TRX_DPPM(v, 0x141));
    v = fmaxf(v, TRX_DPPM(v, 0x140));
    return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))),
                 fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48))));
}
#undef TRX_DPP
#undef TRX_DPPM
__device__ __forceinline__ float leaky_f(float x, float slope) { return x > 0.0f ? x : x * slope; }

// fp32 -> bf16 bits, round to nearest even (torch's conversion): gfx950's
// v_cvt_pk_bf16_f32 (one instruction per pair) instead of integer arithmetic
typedef float trx_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 trx_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
    const trx_f2 v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, trx_b2));
}
__device__ __forceinline__ uint16_t f2bf(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ float bf16r(float x) { return bf2f(f2bf(x)); }
// native 16-byte vector: register arrays of HIP's struct uint4 are not promoted
// out of scratch when written conditionally, this one is
typedef unsigned int trx_u4 __attribute__((ext_vector_type(4)));

// Row elements of the staged xh / p tiles: bf16 bits (the autocast rounding
// points) or, in the exact mode (trx_*_args.exact), float32.
template <bool XF> struct XElem { typedef uint16_t T; };
template <> struct XElem<true> { typedef float T; };
// four consecutive row values as floats
template <bool XF>
__device__ __forceinline__ float4 xld4(const typename XElem<XF>::T* p) {
    if constexpr (XF) {
        return *reinterpret_cast<const float4*>(p);
    } else {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                           __uint_as_float(u.y & 0xffff0000u));
    }
}
template <bool XF>
__device__ __forceinline__ void xst4(typename XElem<XF>::T* p, float a, float b, float c, float d) {
    if constexpr (XF) {
        *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
    } else {
        uint2 u;
        u.x = pk_bf16(a, b);
        u.y = pk_bf16(c, d);
        *reinterpret_cast<uint2*>(p) = u;
    }
}

}  // namespace

#ifdef TRX_PHASE_STAMPS
// Diagnostic build only (make stamps): per-phase cycle totals of the layer
// kernel, thread 0 of each workgroup, rows 0 = layer 0, 1 = HC 1024, 2 = other;
// row 3 = the edge scorer (stage, links, softmax, draw).
__device__ unsigned long long trx_infer_cycles[4][8];
#define TRX_ISTAMP(slot)                                                      \
    do {                                                                      \
        if (threadIdx.x == 0) {                                               \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();            \
            atomicAdd(&trx_infer_cycles[IN > 0 ? 0 : (HC == 1024 ? 1 : 2)][slot], now_ - stamp_prev_); \
            stamp_prev_ = now_;                                               \
        }                                                                     \
    } while (0)
#define TRX_ESTAMP(slot)                                                      \
    do {                                                                      \
        if (threadIdx.x == 0) {                                               \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();            \
            atomicAdd(&trx_infer_cycles[3][slot], now_ - stamp_prev_);        \
            stamp_prev_ = now_;                                               \
        }                                                                     \
    } while (0)
extern "C" int trx_debug_infer_cycles(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(trx_infer_cycles), sizeof(unsigned long long) * 32) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(trx_infer_cycles), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define TRX_ISTAMP(slot) \
    do {                 \
    } while (0)
#define TRX_ESTAMP(slot) \
    do {                 \
    } while (0)
#endif

// ------------------------------------------------------------- layer kernel
// IN: 0 = xh given (layers >= 1), else the layer-0 input width (4).
// XF: the exact mode -- xh float32 (staged as float rows), no bf16 rounding.
template <int HC, int IN, int NT, bool XF>
__global__ void __launch_bounds__(NT) gat_layer_infer_kernel(const NetList<trx_gat_layer_args> nets) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const trx_gat_layer_args& a = nets.a[blockIdx.y];  // network blockIdx.y (*_multi launches)
    typedef typename XElem<XF>::T XE;
    constexpr int EV = 16 / sizeof(XE);  // row elements per 16-byte piece
    constexpr int kInferThreads = NT, kInferWaves = NT / kWave;  // this instance's workgroup
    constexpr int KC = HC / 256;  // float4 chunks per lane in a row
    const int g = blockIdx.x;
    const int n = a.nodes_per_graph, H = a.heads, C = a.channels;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
#ifdef TRX_PHASE_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif
    const int node0 = g * n;
    const int ebeg = a.rowptr[node0];
    const int ne = a.rowptr[node0 + n] - ebeg;
    // 0a. xh rows of the graph (layers >= 1): all loads of a batch in flight before the LDS stores
#ifndef TRX_STAGE_BATCH
#define TRX_STAGE_BATCH 12
#endif
    constexpr int kStageBatch = TRX_STAGE_BATCH;
    trx_u4 stg[kStageBatch];
    const int nq = IN == 0 ? n * HC / EV : 0;
    const trx_u4* xsrc = IN == 0 ? reinterpret_cast<const trx_u4*>(static_cast<const XE*>(a.xh) + (size_t)node0 * HC)
                                 : nullptr;
    if (IN == 0) {
#pragma unroll
        for (int j = 0; j < kStageBatch; ++j) {
            const int v = tid + kInferThreads * j;
            if (v < nq) stg[j] = xsrc[v];
        }
    }
    if (ne > a.max_graph_edges || ne < 0) {  // LDS was sized for max_graph_edges: poison, do not overrun
        for (int idx = tid; idx < n * HC; idx += kInferThreads) {
            if (a.out_f32) a.out_f32[(size_t)node0 * HC + idx] = __builtin_nanf("");
            if (a.out_bf16) static_cast<uint16_t*>(a.out_bf16)[(size_t)node0 * HC + idx] = 0x7fc0;
        }
        if (a.pool)
            for (int f = tid; f < 2 * HC; f += kInferThreads) a.pool[(size_t)g * 2 * HC + f] = __builtin_nanf("");
        return;
    }

    // xh rows padded by 16 B: the attention dots read four nodes' rows
    // per wave instruction, which an unpadded 2 KB stride puts on the same banks
    constexpr int XS = HC + EV;
    XE* xs = reinterpret_cast<XE*>(smem);                // [n][XS] bf16 (exact: float)
    float* as_ = reinterpret_cast<float*>(xs + n * XS);  // [n*H]
    float* ad_ = as_ + n * H;                            // [n*H]
    float* al = ad_ + n * H;        // [me*H] edge logits, then attention weights (in place)
    int* cl = reinterpret_cast<int*>(al + a.max_graph_edges * H);  // [me] source, graph-local
    int* rp = cl + a.max_graph_edges;                    // [n+1] graph-local row pointers
    int* dlc = rp + n + 1;                               // [me] graph-local destination per CSR position
    float* x0l = reinterpret_cast<float*>(dlc + a.max_graph_edges);  // [n*IN]
    float* yt = reinterpret_cast<float*>(smem + ((reinterpret_cast<char*>(x0l + n * IN) - smem + 15) &
                                                 ~(ptrdiff_t)15));  // [n][HC] (pool only), 16-byte aligned

    // 0b. graph-local CSR slice, this layer's edge logits, layer-0 inputs: every
    //     load of the phase issued before the first LDS store (one HBM round trip)
    const int rpv = tid <= n ? a.rowptr[node0 + tid] : 0;
    const int clv = tid < ne ? a.col[ebeg + tid] : 0;  // ne <= max_graph_edges <= 256
    constexpr int kAlRegs = 4;
    float alv[kAlRegs];
#pragma unroll
    for (int j = 0; j < kAlRegs; ++j) {
        const int v = tid + kInferThreads * j, e = v / H, h = v - (v / H) * H;
        alv[j] = v < ne * H ? a.a_edge[(size_t)(ebeg + e) * a.a_edge_stride + a.a_edge_offset + h] : 0.0f;
    }
    const float x0v = IN > 0 && tid < n * IN ? a.x0[(size_t)node0 * IN + tid] : 0.0f;  // n*IN <= 128
    if (tid <= n) rp[tid] = rpv - ebeg;
    if (tid < ne) cl[tid] = clv - node0;
#pragma unroll
    for (int j = 0; j < kAlRegs; ++j) {
        const int v = tid + kInferThreads * j;
        if (v < ne * H) al[v] = alv[j];
    }
    for (int v = tid + kInferThreads * kAlRegs; v < ne * H; v += kInferThreads) {
        const int e = v / H, h = v - e * H;
        al[v] = a.a_edge[(size_t)(ebeg + e) * a.a_edge_stride + a.a_edge_offset + h];
    }
    if (IN > 0 && tid < n * IN) x0l[tid] = XF ? x0v : bf16r(x0v);
    if (IN == 0) {
        constexpr int Q8 = HC / EV;  // 16-byte pieces per row
        auto dst4 = [&](int v) -> trx_u4& {
            return *reinterpret_cast<trx_u4*>(xs + (v / Q8) * XS + (v - (v / Q8) * Q8) * EV);
        };
#pragma unroll
        for (int j = 0; j < kStageBatch; ++j) {
            const int v = tid + kInferThreads * j;
            if (v < nq) dst4(v) = stg[j];
        }
        for (int v = tid + kInferThreads * kStageBatch; v < nq; v += kInferThreads) dst4(v) = xsrc[v];
    }
    __syncthreads();
    for (int i = tid; i < n; i += kInferThreads)
        for (int p = rp[i]; p < rp[i + 1]; ++p) dlc[p] = i;
    TRX_ISTAMP(0);

    // 1. layer 0: xh = bf16(bf16(x0) @ w0^T); a thread owns 4 consecutive columns
    //    (weights in registers) and writes them packed
    if (IN > 0) {
        constexpr int INR = IN > 0 ? IN : 1;
        for (int q = tid; q < HC / 4; q += kInferThreads) {
            float w[4][INR];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < IN; ++j) w[r][j] = a.w0[(size_t)(4 * q + r) * IN + j];
            for (int i = 0; i < n; ++i) {
                float xv[INR];
#pragma unroll
                for (int j = 0; j < IN; ++j) xv[j] = x0l[i * IN + j];
                float acc[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc[r] = 0.0f;
#pragma unroll
                    for (int j = 0; j < IN; ++j) acc[r] += xv[j] * w[r][j];
                }
                xst4<XF>(xs + i * XS + 4 * q, acc[0], acc[1], acc[2], acc[3]);
            }
        }
        __syncthreads();
    }
    TRX_ISTAMP(1);

    // 2. attention dot products <xh[i,h,:], att[h,:]>: four (node, head) pairs per
    //    wave at a time, one per 16-lane row; a lane owns channels 4*sl + 64*m
    //    (conflict-free LDS reads) and the row sums by DPP (no readlane chain).
    //    Pairs t = h*n + i, groups of four dealt round-robin to the waves.
    //    When heads and waves nest (H | waves or waves | H) and C <= 256, a wave
    //    keeps one head: its lanes hold that head's att_src/att_dst slices in
    //    registers (loaded once) and loop over the nodes four at a time, so the
    //    loop reads only LDS (the per-pair global att loads were its latency).
    //    Same per-lane summation order either way.
    const bool head_waves = C <= 256 && C % 64 == 0 && (kInferWaves % H == 0 || H % kInferWaves == 0);
    if (head_waves) {
        const int sub = lane >> 4, sl = lane & 15;
        const int hstep = H >= kInferWaves ? kInferWaves : H;
        const int wph = H >= kInferWaves ? 1 : kInferWaves / H;  // waves sharing one head
        const int wi = H >= kInferWaves ? 0 : wave / H;
        const int CM = C / 64;
        for (int h = H >= kInferWaves ? wave : wave % H; h < H; h += hstep) {
            float4 sa[4], da[4];
#pragma unroll
            for (int m = 0; m < 4; ++m)
                if (m < CM) {
                    sa[m] = *reinterpret_cast<const float4*>(a.att_src + h * C + 4 * sl + 64 * m);
                    da[m] = *reinterpret_cast<const float4*>(a.att_dst + h * C + 4 * sl + 64 * m);
                }
            for (int i0 = 4 * wi; i0 < n; i0 += 4 * wph) {
                const int i = i0 + sub;
                const bool ok = i < n;
                float s1 = 0.0f, s2 = 0.0f;
                if (ok) {
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        if (m < CM) {
                            const float4 x4 = xld4<XF>(xs + i * XS + h * C + 4 * sl + 64 * m);
                            const float v0 = x4.x, v1 = x4.y, v2 = x4.z, v3 = x4.w;
                            s1 += (v0 * sa[m].x + v1 * sa[m].y) + (v2 * sa[m].z + v3 * sa[m].w);
                            s2 += (v0 * da[m].x + v1 * da[m].y) + (v2 * da[m].z + v3 * da[m].w);
                        }
                }
                s1 = row_sum16_f(s1);
                s2 = row_sum16_f(s2);
                if (ok && sl == 0) {
                    as_[i * H + h] = s1;
                    ad_[i * H + h] = s2;
                }
            }
        }
    } else {
        const int P = n * H, groups = (P + 3) / 4;
        const int sub = lane >> 4, sl = lane & 15;
        for (int gi = wave; gi < groups; gi += kInferWaves) {
            const int t = 4 * gi + sub;
            const bool ok = t < P;
            const int h = ok ? t / n : 0, i = ok ? t - h * n : 0;
            float s1 = 0.0f, s2 = 0.0f;
            if (ok) {
                for (int c = 4 * sl; c < C; c += 64) {
                    const float4 sa = *reinterpret_cast<const float4*>(a.att_src + h * C + c);
                    const float4 da = *reinterpret_cast<const float4*>(a.att_dst + h * C + c);
                    const float4 x4 = xld4<XF>(xs + i * XS + h * C + c);
                    const float v0 = x4.x, v1 = x4.y, v2 = x4.z, v3 = x4.w;
                    s1 += (v0 * sa.x + v1 * sa.y) + (v2 * sa.z + v3 * sa.w);
                    s2 += (v0 * da.x + v1 * da.y) + (v2 * da.z + v3 * da.w);
                }
            }
            s1 = row_sum16_f(s1);
            s2 = row_sum16_f(s2);
            if (ok && sl == 0) {
                as_[i * H + h] = s1;
                ad_[i * H + h] = s2;
            }
        }
    }
    __syncthreads();
    if (a.save_asd)
        for (int t = tid; t < n * H; t += kInferThreads) {
            const int i = t / H, h = t - (t / H) * H;
            a.save_asd[(size_t)(node0 + i) * 2 * H + h] = as_[t];
            a.save_asd[(size_t)(node0 + i) * 2 * H + H + h] = ad_[t];
        }
    TRX_ISTAMP(2);
    TRX_ISTAMP(3);

    // 3. softmax over in-edges, LDS only: (a) every (edge, head) logit
    //    leaky(a_src + a_dst + a_edge) in place, one thread each; (b) per (node,
    //    head) the max, the exp terms (kept in place) and their sum in edge
    //    order, the denominator into ad_ (a_dst is consumed); (c) every
    //    (edge, head) weight = exp / denominator.  Same values as one thread
    //    per (node, head) doing all three passes.
    for (int v = tid; v < ne * H; v += kInferThreads) {
        const int p = v / H, h = v - (v / H) * H;
        al[v] = leaky_f(as_[cl[p] * H + h] + ad_[dlc[p] * H + h] + al[v], a.negative_slope);
    }
    __syncthreads();
    for (int t = tid; t < n * H; t += kInferThreads) {
        const int i = t / H, h = t - (t / H) * H;
        const int p0 = rp[i], p1 = rp[i + 1];
        float m = -__builtin_huge_valf();
        for (int p = p0; p < p1; ++p) m = fmaxf(m, al[p * H + h]);
        float ssum = 0.0f;
        for (int p = p0; p < p1; ++p) {
            const float ex = __expf(al[p * H + h] - m);
            al[p * H + h] = ex;
            ssum += ex;
        }
        ad_[t] = ssum + 1e-16f;
    }
    __syncthreads();
    for (int v = tid; v < ne * H; v += kInferThreads) {
        const int p = v / H, h = v - (v / H) * H;
        al[v] = al[v] / ad_[dlc[p] * H + h];
    }
    __syncthreads();
    if (a.save_alpha)
        for (int v = tid; v < ne * H; v += kInferThreads) a.save_alpha[(size_t)ebeg * H + v] = al[v];
    TRX_ISTAMP(4);

    // 4. aggregation + epilogue, one wave per node; lane owns chunks q = lane + 64k.
    //    Per-column constants live in registers across the wave's nodes.  The
    //    weighted sums and the LayerNorm affine are fused multiply-adds (one
    //    rounding each; the backward reads the saved pre-LN rows, not a recompute).
    float bias_r[KC][4], lnw_r[KC][4], lnb_r[KC][4];
    float wp_r[KC][4][IN > 0 ? IN : 1], bp_r[KC][4];
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int f = 4 * (lane + kWave * k) + r;
            bias_r[k][r] = a.bias[f];
            lnw_r[k][r] = a.ln_weight[f];
            lnb_r[k][r] = a.ln_bias[f];
            if (IN > 0) {
#pragma unroll
                for (int j = 0; j < IN; ++j) wp_r[k][r][j] = a.wp[(size_t)f * IN + j];
                bp_r[k][r] = a.bp[f];
            }
        }
    // the residual rows (middle layers) are loaded one node ahead: node i's arrive
    // while the wave aggregates node i - kInferWaves (layer 0's residual is its
    // input projection, computed in registers)
    const bool res_in = IN == 0 && a.residual == 1;
    float4 res_next[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
        res_next[k] = res_in && wave < n
                          ? *reinterpret_cast<const float4*>(a.res + (size_t)(node0 + wave) * HC + 4 * (lane + kWave * k))
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = wave; i < n; i += kInferWaves) {
        const int node = node0 + i;
        float4 res4[KC];
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            res4[k] = res_next[k];
            res_next[k] = res_in && i + kInferWaves < n
                              ? *reinterpret_cast<const float4*>(a.res + (size_t)(node + kInferWaves) * HC +
                                                                 4 * (lane + kWave * k))
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float4 acc[KC];
#pragma unroll
        for (int k = 0; k < KC; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (KC == 4 && C == 256) {
            // chunk k is head k: the edge's four weights in one 16-byte LDS read
            // (al rows are 16-byte aligned: H == 4 floats per edge)
            for (int p = rp[i]; p < rp[i + 1]; ++p) {
                const XE* row = xs + cl[p] * XS;
                const float4 w4 = *reinterpret_cast<const float4*>(al + p * 4);
                const float wk[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (int k = 0; k < KC; ++k) {
                    const float w = wk[k & 3];
                    const float4 x4 = xld4<XF>(row + 4 * (lane + kWave * k));
                    acc[k].x = __builtin_fmaf(w, x4.x, acc[k].x);
                    acc[k].y = __builtin_fmaf(w, x4.y, acc[k].y);
                    acc[k].z = __builtin_fmaf(w, x4.z, acc[k].z);
                    acc[k].w = __builtin_fmaf(w, x4.w, acc[k].w);
                }
            }
        } else {
            for (int p = rp[i]; p < rp[i + 1]; ++p) {
                const XE* row = xs + cl[p] * XS;
                const float* alr = al + p * H;
#pragma unroll
                for (int k = 0; k < KC; ++k) {
                    const int q = lane + kWave * k;
                    const float w = alr[(4 * q) / C];
                    const float4 x4 = xld4<XF>(row + 4 * q);
                    acc[k].x = __builtin_fmaf(w, x4.x, acc[k].x);
                    acc[k].y = __builtin_fmaf(w, x4.y, acc[k].y);
                    acc[k].z = __builtin_fmaf(w, x4.z, acc[k].z);
                    acc[k].w = __builtin_fmaf(w, x4.w, acc[k].w);
                }
            }
        }
        float v[KC][4];
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            v[k][0] = acc[k].x + bias_r[k][0];
            v[k][1] = acc[k].y + bias_r[k][1];
            v[k][2] = acc[k].z + bias_r[k][2];
            v[k][3] = acc[k].w + bias_r[k][3];
            s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
        }
        const float mean = wave_sum_f(s) / (float)HC;
        float s2 = 0.0f;
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float d = v[k][r] - mean;
                s2 += d * d;
            }
        const float rstd = rsqrtf(wave_sum_f(s2) / (float)HC + a.ln_eps);
        if (a.save_v) {
#pragma unroll
            for (int k = 0; k < KC; ++k)
            {  // read back only by the backward, much later: non-temporal, past the caches
                typedef float trx_f4v __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store((trx_f4v){v[k][0], v[k][1], v[k][2], v[k][3]},
                                            reinterpret_cast<trx_f4v*>(a.save_v + (size_t)node * HC + 4 * (lane + kWave * k)));
            }
        }
        if (a.save_stats && lane == 0) {
            a.save_stats[2 * (size_t)node] = mean;
            a.save_stats[2 * (size_t)node + 1] = rstd;
        }
        float xr[IN > 0 ? IN : 1];  // the node's layer-0 inputs in registers (the LDS pool stores below
#pragma unroll                      // would otherwise force a reload per column)
        for (int j = 0; j < (IN > 0 ? IN : 1); ++j) xr[j] = IN > 0 ? x0l[i * IN + j] : 0.0f;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int f0 = 4 * (lane + kWave * k);
            const float resv[4] = {res4[k].x, res4[k].y, res4[k].z, res4[k].w};
            float y4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float y = __builtin_fmaf(lnw_r[k][r], rstd * (v[k][r] - mean), lnb_r[k][r]);
                if (IN > 0 && a.residual == 2) {
                    float t = 0.0f;
#pragma unroll
                    for (int j = 0; j < (IN > 0 ? IN : 1); ++j) t += xr[j] * wp_r[k][r][j];
                    y = y + (XF ? t + bp_r[k][r] : bf16r(t + bp_r[k][r]));
                } else if (IN == 0 && a.residual == 1) {
                    y = y + resv[r];
                }
                if (a.activation == 0)
                    y = y > 0.0f ? y : 0.0f;
                else
                    y = y <= 0.0f ? (expf(y) - 1.0f) : y;
                y4[r] = y;
            }
            // one 16-byte store per lane (four scalar stores at a 4-word lane stride hit
            // the same banks from lanes 16 apart)
            if (a.pool) *reinterpret_cast<float4*>(yt + i * HC + f0) = make_float4(y4[0], y4[1], y4[2], y4[3]);
            if (a.out_f32)
                *reinterpret_cast<float4*>(a.out_f32 + (size_t)node * HC + f0) = make_float4(y4[0], y4[1], y4[2], y4[3]);
            if (a.out_bf16) {
                uint2 u;
                u.x = pk_bf16(y4[0], y4[1]);
                u.y = pk_bf16(y4[2], y4[3]);
                *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.out_bf16) + (size_t)node * HC + f0) = u;
            }
        }
    }
    TRX_ISTAMP(5);
    if (a.pool) {
        __syncthreads();
        TRX_ISTAMP(6);
        for (int f = tid; f < HC; f += kInferThreads) {
            float s = 0.0f, mx = -__builtin_huge_valf();
            for (int i = 0; i < n; ++i) {
                const float y = yt[i * HC + f];
                s += y;
                mx = fmaxf(mx, y);
            }
            a.pool[(size_t)g * 2 * HC + f] = s / (float)n;
            a.pool[(size_t)g * 2 * HC + HC + f] = mx;
        }
        TRX_ISTAMP(7);
    }
}

// --------------------------------------------------------- edge scorer
// One workgroup per graph.  The graph's p rows (n x 2H bf16, contiguous in
// HBM), link endpoints, features and mask are staged in LDS by one batch of
// coalesced loads (no dependent index -> row loads per link); then one wave per
// link, lane owning 4 consecutive hidden units per 256-wide chunk (weights in
// registers), and a wave reduction of the 256->1 product.
constexpr int kEdgeED = 8;  // edge_dim <= 8

// DK: the link-feature count when fixed at compile time (the regular case, 6: no
// per-term edge_dim test and no padding terms in the link-feature product), 0 = any
// edge_dim <= kEdgeED.  The same terms in the same order either way.
template <int MQ, int DK, bool XF>  // hidden <= 256 * MQ, hidden % 4 == 0; XF: p float (exact mode)
__global__ void __launch_bounds__(kInferThreads) edge_head_infer_kernel(const NetList<trx_edge_head_args> nets) {
    const trx_edge_head_args& a = nets.a[blockIdx.y];
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename XElem<XF>::T XE;
    constexpr int EV = 16 / sizeof(XE);
    constexpr int ED = kEdgeED;
    const int g = blockIdx.x;
    const int E = a.edges_per_graph, Hd = a.hidden, D = a.edge_dim, n = a.nodes_per_graph;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
#ifdef TRX_PHASE_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif
    XE* pr = reinterpret_cast<XE*>(smem);                            // [n][2*Hd] bf16 (exact: float)
    float* eal = reinterpret_cast<float*>(pr + (size_t)n * 2 * Hd);  // [E][ED] link features (fp32)
    float* lg = eal + (size_t)E * ED;                                // [E] logits
    float* mk = lg + E;                                              // [E] mask
    int* sl = reinterpret_cast<int*>(mk + E);                        // [E] graph-local src
    int* dl = sl + E;                                                // [E] graph-local dst
    int* badl = dl + E;                                              // [1] link outside the node block
    if (tid == 0) *badl = 0;
    __syncthreads();

    // stage: the loads of a batch are all issued before its LDS stores
    const int64_t node0 = (int64_t)g * n;
    const trx_u4* src4 = reinterpret_cast<const trx_u4*>(static_cast<const XE*>(a.p) + node0 * 2 * Hd);
    trx_u4* dst4 = reinterpret_cast<trx_u4*>(pr);
    const int nq = n * 2 * Hd / EV;
#ifndef TRX_EH_ROWS
#define TRX_EH_ROWS 6
#endif
    constexpr int kRowRegs = TRX_EH_ROWS;
    trx_u4 rows[kRowRegs];
#pragma unroll
    for (int j = 0; j < kRowRegs; ++j) {
        const int v = tid + kInferThreads * j;
        if (v < nq) rows[j] = src4[v];
    }
    constexpr int kEaRegs = 4;
    float eav[kEaRegs];
#pragma unroll
    for (int j = 0; j < kEaRegs; ++j) {
        const int v = tid + kInferThreads * j, e = v / ED, jj = v - (v / ED) * ED;
        eav[j] = v < E * ED && jj < D ? a.ea[((int64_t)g * E + e) * D + jj] : 0.0f;
    }
    int badf = 0;
    for (int e = tid; e < E; e += kInferThreads) {
        const int64_t eg = (int64_t)g * E + e;
        const int64_t s = a.src[eg] - node0, d = a.dst[eg] - node0;
        const float mv = a.softmax ? a.mask[eg] : 1.0f;
        badf |= (s < 0) | (s >= n) | (d < 0) | (d >= n);
        sl[e] = (int)s;
        dl[e] = (int)d;
        mk[e] = mv;
    }
#pragma unroll
    for (int j = 0; j < kRowRegs; ++j) {
        const int v = tid + kInferThreads * j;
        if (v < nq) dst4[v] = rows[j];
    }
    for (int v = tid + kInferThreads * kRowRegs; v < nq; v += kInferThreads) dst4[v] = src4[v];
#pragma unroll
    for (int j = 0; j < kEaRegs; ++j) {
        const int v = tid + kInferThreads * j;
        if (v < E * ED) eal[v] = eav[j];
    }
    for (int v = tid + kInferThreads * kEaRegs; v < E * ED; v += kInferThreads) {
        const int e = v / ED, j = v - (v / ED) * ED;
        eal[v] = j < D ? a.ea[((int64_t)g * E + e) * D + j] : 0.0f;
    }
    constexpr int DC = DK > 0 ? DK : ED;
    // a lane's four hidden units as two pairs: the per-unit arithmetic below is written on
    // float32 pairs (for v_pk_mul_f32 / v_pk_add_f32); under -packed-fp32-ops (Makefile:
    // the gfx950 packed -> DPP hazard) each pair compiles to scalar ops, the
    // same IEEE operations in the same order per unit (bit-identical)
    trx_f2 we2[MQ][2][DC], c2[MQ][2];
    float w2_r[MQ][4];
#pragma unroll
    for (int m = 0; m < MQ; ++m) {
        const int k0 = 256 * m + 4 * lane;
        if (k0 < Hd) {  // hidden % 4 == 0: the lane's four units are all valid; 16-byte loads
            const float4 w2v = *reinterpret_cast<const float4*>(a.w2 + k0);
            const float4 cv = *reinterpret_cast<const float4*>(a.c + (int64_t)g * Hd + k0);
            w2_r[m][0] = w2v.x, w2_r[m][1] = w2v.y, w2_r[m][2] = w2v.z, w2_r[m][3] = w2v.w;
            c2[m][0] = (trx_f2){cv.x, cv.y};
            c2[m][1] = (trx_f2){cv.z, cv.w};
            if constexpr (DK == 6) {  // the four units' link-feature rows: 24 contiguous floats
                float wv[24];
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    const float4 t = *reinterpret_cast<const float4*>(a.we + (size_t)k0 * 6 + 4 * q);
                    wv[4 * q] = t.x, wv[4 * q + 1] = t.y, wv[4 * q + 2] = t.z, wv[4 * q + 3] = t.w;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int j = 0; j < 6; ++j) we2[m][r >> 1][j][r & 1] = wv[r * 6 + j];
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int j = 0; j < DC; ++j) we2[m][r >> 1][j][r & 1] = j < D ? a.we[(k0 + r) * D + j] : 0.0f;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w2_r[m][r] = 0.0f;
                c2[m][r >> 1][r & 1] = 0.0f;
#pragma unroll
                for (int j = 0; j < DC; ++j) we2[m][r >> 1][j][r & 1] = 0.0f;
            }
        }
    }
    const float b2 = a.b2[0];
    if (badf) *badl = 1;
    __syncthreads();
    if (*badl) {  // a link leaves the graph's node block: poison, never read outside LDS
        for (int e = tid; e < E; e += kInferThreads) {
            a.out[(int64_t)g * E + e] = __builtin_nanf("");
            if (a.softmax && a.logits) a.logits[(int64_t)g * E + e] = __builtin_nanf("");
        }
        return;
    }

    TRX_ESTAMP(0);
#ifndef TRX_EH_EU
#define TRX_EH_EU 2
#endif
    constexpr int EU = TRX_EH_EU;  // links per wave iteration
    for (int e0 = wave * EU; e0 < E; e0 += kInferWaves * EU) {
        float part[EU];
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const int e = e0 + u < E ? e0 + u : E - 1;
            const float4 ea0 = *reinterpret_cast<const float4*>(eal + e * ED);
            const float4 ea1 = *reinterpret_cast<const float4*>(eal + e * ED + 4);
            const float ear[ED] = {ea0.x, ea0.y, ea0.z, ea0.w, ea1.x, ea1.y, ea1.z, ea1.w};
            const XE* ps = pr + sl[e] * 2 * Hd;
            const XE* pd = pr + dl[e] * 2 * Hd + Hd;
            part[u] = 0.0f;
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                const int k0 = 256 * m + 4 * lane;
                if (k0 < Hd) {
                    const float4 s4 = xld4<XF>(ps + k0), d4 = xld4<XF>(pd + k0);
                    const trx_f2 psv[2] = {{s4.x, s4.y}, {s4.z, s4.w}};
                    const trx_f2 pdv[2] = {{d4.x, d4.y}, {d4.z, d4.w}};
#pragma unroll
                    for (int rp = 0; rp < 2; ++rp) {
                        // the link-feature term and the 256 -> 1 product as fused multiply-adds
                        // (one rounding per term; edge_head_bwd_kernel recomputes z the same way)
                        float ewx = 0.0f, ewy = 0.0f;
#pragma unroll
                        for (int j = 0; j < DC; ++j)
                            if (DK > 0 || j < D) {
                                ewx = __builtin_fmaf(ear[j], we2[m][rp][j].x, ewx);
                                ewy = __builtin_fmaf(ear[j], we2[m][rp][j].y, ewy);
                            }
                        // fp32 from the bf16 GEMM outputs on: the link's hidden units and
                        // their shares of the 256 -> 1 product (units in order)
                        const trx_f2 z = ((psv[rp] + pdv[rp]) + (trx_f2){ewx, ewy}) + c2[m][rp];
                        part[u] = __builtin_fmaf(fmaxf(z.x, 0.0f), w2_r[m][2 * rp], part[u]);
                        part[u] = __builtin_fmaf(fmaxf(z.y, 0.0f), w2_r[m][2 * rp + 1], part[u]);
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const float t = wave_sum_f(part[u]);
            if (lane == 0 && e0 + u < E) lg[e0 + u] = t + b2;
        }
    }
    __syncthreads();
    TRX_ESTAMP(1);
    if (!a.softmax) {
        for (int e = tid; e < E; e += kInferThreads) a.out[(int64_t)g * E + e] = lg[e];
        return;
    }
    if (wave != 0) return;
    for (int e = lane; e < E; e += kWave) lg[e] = mk[e] <= 0.0f ? -1e9f : lg[e];  // masked logits, in place
    if (a.logits)
        for (int e = lane; e < E; e += kWave) a.logits[(int64_t)g * E + e] = lg[e];
    float m = -__builtin_huge_valf();
    for (int e0 = 0; e0 < E; e0 += kWave) m = fmaxf(m, wave_max_f(e0 + lane < E ? lg[e0 + lane] : -__builtin_huge_valf()));
    float ssum = 0.0f;  // each exp term computed once, kept in mk[] (the mask is no longer needed)
    for (int e0 = 0; e0 < E; e0 += kWave) {
        const int e = e0 + lane;
        const float ex = e < E ? expf(lg[e] - m) : 0.0f;
        if (e < E) mk[e] = ex;
        ssum += wave_sum_f(ex);
    }
    const float denom = ssum + 1e-16f;
    for (int e = lane; e < E; e += kWave) a.out[(int64_t)g * E + e] = mk[e] / denom;
    TRX_ESTAMP(2);
    if (a.u) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // mk[] written by every lane, read by lane 0
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // one categorical draw per graph (inverse CDF over the same exp terms, summed in
        // link order): the terms come to the wave's registers 64 at a time and the
        // serial scan reads them with readlane (no dependent LDS reads)
        const float target = a.u[g] * ssum;
        float acc = 0.0f;
        int pick = -1, last = 0;
        for (int e0 = 0; e0 < E; e0 += kWave) {
            const float exl = e0 + lane < E ? mk[e0 + lane] : 0.0f;
            const int cnt = E - e0 < kWave ? E - e0 : kWave;
            for (int t = 0; t < cnt; ++t) {
                const float ex = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(exl), t));
                if (ex > 0.0f) last = e0 + t;
                acc += ex;
                if (pick < 0 && acc > target) pick = e0 + t;
            }
        }
        if (lane == 0) a.action[g] = pick >= 0 ? pick : last;  // u * total above the serial sum: last link with mass
    }
    TRX_ESTAMP(3);
}

// -------------------------------------------------------------- prologue
// M rows of every layer: one wave per (layer, head, feature), lanes over channels.
__global__ void __launch_bounds__(kWave) edge_att_weights_kernel(const NetList<trx_gat_prologue_args> nets) {
    const trx_gat_prologue_args& a = nets.a[blockIdx.y];
    const int lane = threadIdx.x, D = a.edge_dim;
    int l = 0, oo = blockIdx.x, row0 = 0;
    while (oo >= a.heads[l] * D) {
        oo -= a.heads[l] * D;
        row0 += a.heads[l];
        ++l;
    }
    const int h = oo / D, j = oo - (oo / D) * D, C = a.channels[l];
    float s = 0.0f;
    for (int c = lane; c < C; c += kWave) s += a.lin_edge_w[l][(size_t)(h * C + c) * D + j] * a.att_edge[l][h * C + c];
    s = wave_sum_f(s);
    if (lane == 0) a.m_work[(row0 + h) * D + j] = s;
}

constexpr int kProMD = 8;  // node_dim, edge_dim <= 8 (register rows)
constexpr int kProLS = 9;  // LDS row stride of the per-link / per-node rows: odd, so a wave's rows hit distinct banks

// x[0..d) -> LayerNorm (biased variance, like torch); compile-time bounded loops
__device__ __forceinline__ void layer_norm_row(float (&x)[kProMD], int d, const float* w, const float* b, float eps) {
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < kProMD; ++j)
        if (j < d) s += x[j];
    const float mu = s / (float)d;
    float v = 0.0f;
#pragma unroll
    for (int j = 0; j < kProMD; ++j)
        if (j < d) {
            const float t = x[j] - mu;
            v += t * t;
        }
    const float r = rsqrtf(v / (float)d + eps);
#pragma unroll
    for (int j = 0; j < kProMD; ++j)
        if (j < d) x[j] = (x[j] - mu) * r * w[j] + b[j];
}

// One workgroup per graph: input LayerNorms, self-loop means, a_edge of every
// layer in CSR order.  A node's self-loop attr is the mean over its kept
// in-links, summed in link order: its CSR-by-destination row lists them in
// that order (stable sort by destination), so each node walks only its own
// row.  NT threads per graph: 128 for the acting pass, 256 for the 256-graph
// update batches (one workgroup per CU either way has work for every SIMD).
template <int NT>
__global__ void __launch_bounds__(NT) gat_prologue_kernel(const NetList<trx_gat_prologue_args> nets, int A) {
    const trx_gat_prologue_args& a = nets.a[blockIdx.y];
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int MD = kProMD;
    const int g = blockIdx.x, tid = threadIdx.x;
    const int n = a.nodes_per_graph, E = a.edges_per_graph, ND = a.node_dim, D = a.edge_dim;
    constexpr int LS = kProLS;
    float* ean = reinterpret_cast<float*>(smem);  // [E][LS] normalised link features
    float* lp = ean + E * LS;                     // [n][LS] self-loop attrs
    float* Ml = lp + n * LS;                      // [A][8] bf16-rounded M rows (broadcast reads)
    const int64_t node0 = (int64_t)g * n, link0 = (int64_t)g * E;
    const int p0 = a.rowptr[node0], p1 = a.rowptr[node0 + n];
    for (int v = tid; v < A * D; v += NT) {
        const int k = v / D, j = v - (v / D) * D;
        Ml[k * MD + j] = a.exact ? a.m_work[v] : bf16r(a.m_work[v]);
    }
    for (int l = tid; l < E; l += NT) {
        float x[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) x[j] = j < D ? a.edge_x[(link0 + l) * D + j] : 0.0f;
        layer_norm_row(x, D, a.edge_ln_w, a.edge_ln_b, a.edge_ln_eps);
#pragma unroll
        for (int j = 0; j < MD; ++j)
            if (j < D) {
                ean[l * LS + j] = x[j];
                a.ea[(link0 + l) * D + j] = x[j];
            }
    }
    for (int i = tid; i < n; i += NT) {
        float x[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) x[j] = j < ND ? a.node_x[(node0 + i) * ND + j] : 0.0f;
        layer_norm_row(x, ND, a.node_ln_w, a.node_ln_b, a.node_ln_eps);
#pragma unroll
        for (int j = 0; j < MD; ++j)
            if (j < ND) a.x0[(node0 + i) * ND + j] = x[j];
    }
    __syncthreads();
    for (int i = tid; i < n; i += NT) {  // self-loop attr: mean over the kept in-links of i, in link order
        float s[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) s[j] = 0.0f;
        int cnt = 0;
        for (int p = a.rowptr[node0 + i]; p < a.rowptr[node0 + i + 1]; ++p) {
            const int code = a.pos_src[p];
            const int64_t li = (int64_t)code - link0;
            if (code < 0 || li < 0 || li >= E) continue;  // the appended self loop (or a foreign link)
            ++cnt;
#pragma unroll
            for (int j = 0; j < MD; ++j)
                if (j < D) s[j] += ean[li * LS + j];
        }
        const float deg = cnt > 0 ? (float)cnt : 1.0f;
#pragma unroll
        for (int j = 0; j < MD; ++j)
            if (j < D) lp[i * LS + j] = s[j] / deg;
    }
    __syncthreads();
    for (int p = p0 + tid; p < p1; p += NT) {
        const int code = a.pos_src[p];
        const int64_t li = (int64_t)code - link0, ni = -(int64_t)code - 1 - node0;
        const bool ok = code >= 0 ? (li >= 0 && li < E) : (ni >= 0 && ni < n);
        const float* fr = code >= 0 ? ean + (ok ? li : 0) * LS : lp + (ok ? ni : 0) * LS;
        float f[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) f[j] = j < D ? (a.exact ? fr[j] : bf16r(fr[j])) : 0.0f;
        for (int k = 0; k < A; ++k) {
            float acc = 0.0f;
#pragma unroll
            for (int j = 0; j < MD; ++j)
                if (j < D) acc += f[j] * Ml[k * MD + j];
            a.a_edge[(size_t)p * A + k] = ok ? (a.exact ? acc : bf16r(acc)) : __builtin_nanf("");
        }
    }
}

size_t gat_prologue_smem(const trx_gat_prologue_args& a) {
    int A = 0;
    for (int l = 0; l < a.num_layers; ++l) A += a.heads[l];
    return ((size_t)a.edges_per_graph * kProLS + (size_t)a.nodes_per_graph * kProLS + (size_t)A * kProMD +
            a.edges_per_graph) * 4;
}

// networks k < count (the same sizes and layer shapes: checked by the C ABI)
hipError_t launch_gat_prologue(const trx_gat_prologue_args* a, int count, hipStream_t stream) {
    const trx_gat_prologue_args& a0 = a[0];
    const NetList<trx_gat_prologue_args> l = net_list(a, count);
    int A = 0;
    for (int k = 0; k < a0.num_layers; ++k) A += a0.heads[k];
    hipLaunchKernelGGL(edge_att_weights_kernel, dim3(A * a0.edge_dim, count), dim3(kWave), 0, stream, l);
    if (a0.num_graphs * count < 2048)
        hipLaunchKernelGGL(gat_prologue_kernel<256>, dim3(a0.num_graphs, count), dim3(256), gat_prologue_smem(a0),
                           stream, l, A);
    else
        hipLaunchKernelGGL(gat_prologue_kernel<128>, dim3(a0.num_graphs, count), dim3(128), gat_prologue_smem(a0),
                           stream, l, A);
    return hipGetLastError();
}

size_t edge_head_infer_smem(const trx_edge_head_args& a) {
    return (size_t)a.nodes_per_graph * 2 * a.hidden * (a.exact ? 4 : 2) + (size_t)a.edges_per_graph * (kEdgeED * 4 + 4 * 4) + 4;
}

size_t gat_layer_infer_smem(const trx_gat_layer_args& a) {
    const int HC = a.heads * a.channels, n = a.nodes_per_graph, H = a.heads, me = a.max_graph_edges;
    const size_t alsz = (size_t)me * H;
    size_t b = (a.exact ? (size_t)n * (HC + 4) * 4 : (size_t)n * (HC + 8) * 2) + 2 * (size_t)n * H * 4 + alsz * 4 + (size_t)me * 4 * 2 + (size_t)(n + 1) * 4 +
               (size_t)n * a.in_dim * 4;
    if (a.pool) b += (size_t)n * HC * 4 + 12;  // + the 16-byte alignment of the pool rows
    return b;
}

template <int HC, int IN, int NT, bool XF = false>
static void set_lds_attr() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gat_layer_infer_kernel<HC, IN, NT, XF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

// One workgroup per graph.  The acting pass (4096 graphs) fills the CUs with
// 4-wave workgroups; the SAC update's passes (256 graphs: one workgroup per
// CU) take 8-wave workgroups, so each CU still has two waves per SIMD.
hipError_t launch_gat_layer_infer(const trx_gat_layer_args* al, int count, hipStream_t stream) {
    const trx_gat_layer_args& a = al[0];
    const NetList<trx_gat_layer_args> l = net_list(al, count);
    const int HC = a.heads * a.channels;
    const size_t smem = gat_layer_infer_smem(a);
    static bool attr_set = false;
    if (!attr_set) {  // allow > 64 KB of dynamic LDS (gfx950: 160 KB per CU)
        set_lds_attr<1024, 0, 256>();
        set_lds_attr<1024, 4, 256>();
        set_lds_attr<512, 0, 256>();
        set_lds_attr<512, 4, 256>();
        set_lds_attr<256, 0, 256>();
        set_lds_attr<256, 4, 256>();
        set_lds_attr<1024, 0, 512>();
        set_lds_attr<1024, 4, 512>();
        set_lds_attr<512, 0, 512>();
        set_lds_attr<512, 4, 512>();
        set_lds_attr<256, 0, 512>();
        set_lds_attr<256, 4, 512>();
        set_lds_attr<1024, 0, 512, true>();
        set_lds_attr<1024, 4, 512, true>();
        set_lds_attr<1024, 0, 256, true>();
        set_lds_attr<1024, 4, 256, true>();
        set_lds_attr<512, 0, 512, true>();
        set_lds_attr<512, 4, 512, true>();
        set_lds_attr<256, 0, 512, true>();
        set_lds_attr<256, 4, 512, true>();
        set_lds_attr<512, 0, 256, true>();
        set_lds_attr<512, 4, 256, true>();
        set_lds_attr<256, 0, 256, true>();
        set_lds_attr<256, 4, 256, true>();
        attr_set = true;
    }
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    const dim3 grid(a.num_graphs, count);
#ifndef TRX_WIDE_GRAPHS
#define TRX_WIDE_GRAPHS 2048
#endif
    const bool wide = a.num_graphs * count < TRX_WIDE_GRAPHS;
#define TRX_LAYER_CASE(HCV, INV, XFV)                                                                          \
    if (HC == HCV && a.in_dim == INV && (a.exact != 0) == XFV) {                                               \
        if (wide)                                                                                              \
            hipLaunchKernelGGL((gat_layer_infer_kernel<HCV, INV, 512, XFV>), grid, dim3(512), smem, stream, l); \
        else                                                                                                   \
            hipLaunchKernelGGL((gat_layer_infer_kernel<HCV, INV, 256, XFV>), grid, dim3(256), smem, stream, l); \
        return hipGetLastError();                                                                              \
    }
    TRX_LAYER_CASE(1024, 0, false)
    TRX_LAYER_CASE(1024, 4, false)
    TRX_LAYER_CASE(512, 0, false)
    TRX_LAYER_CASE(512, 4, false)
    TRX_LAYER_CASE(256, 0, false)
    TRX_LAYER_CASE(256, 4, false)
    TRX_LAYER_CASE(1024, 0, true)
    TRX_LAYER_CASE(1024, 4, true)
    TRX_LAYER_CASE(512, 0, true)
    TRX_LAYER_CASE(512, 4, true)
    TRX_LAYER_CASE(256, 0, true)
    TRX_LAYER_CASE(256, 4, true)
#undef TRX_LAYER_CASE
    return hipErrorInvalidValue;
}

// ------------------------------------------------ edge scorer, backward
// Training-path backward of the edge scorer (the logits of edge_head_infer
// with softmax = 0), one workgroup per graph, thread k = hidden unit k
// (hidden <= 256).  The forward is recomputed from the LDS-staged p rows.
// Everything after the bf16 p GEMM is fp32 (as in the forward): the incoming
// logit gradient g, dz = g * w2 behind the ReLU, the per-graph sums of dz
// (grad_c) and of g * relu(z) (grad_w2), and the p gradients as fp32 sums
// over the graph's links in a fixed link order, rounded to bf16 once (they
// feed the bf16 GEMM backward).  Two passes, no LDS read-modify-write chains,
// and four threads per hidden unit (1024 per graph: the update's 256 graphs
// are one workgroup per CU): (1) per link (links dealt to the four parts),
// thread k's gradient through unit k, kept fp32 in LDS, with per-part
// grad_c / grad_w2 sums added in part order; (2) per node (nodes dealt to the
// parts), the sums over its out-links (p[:, :H]) and in-links (p[:, H:]) in
// link order.
// Outputs: grad_p [N, 2H] bf16, grad_c [B, H], grad_w2_part [B, H] (per-graph
// sums of g * relu(z)), and the link-feature block in fp32 like its forward:
// grad_we_part [B, H, D] (per-graph sums of dz * ea, links in order) and
// grad_ea [E_total, D] (dz . we per link: (3), one wave per link, wave sums);
// grad_z [E_total, H] bf16 (dz) only when asked for.
constexpr int kEhbThreads = 1024, kEhbParts = kEhbThreads / 256;

template <bool XF>  // exact mode: p and grad_p float
__global__ void __launch_bounds__(kEhbThreads) edge_head_bwd_kernel(const NetList<EdgeHeadBwdItem> nets) {
    const trx_edge_head_args& a = nets.a[blockIdx.y].a;
    const trx_edge_head_bwd_io& io = nets.a[blockIdx.y].io;
    const float* const grad_logits = io.grad_logits;
    void* const grad_p_ = io.grad_p;
    float* const grad_c = io.grad_c;
    uint16_t* const grad_z = static_cast<uint16_t*>(io.grad_z);
    float* const grad_w2_part = io.grad_w2_part;
    float* const grad_we_part = io.grad_we_part;
    float* const grad_ea = io.grad_ea;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename XElem<XF>::T XE;
    constexpr int EV = 16 / sizeof(XE);
    XE* const grad_p = static_cast<XE*>(grad_p_);
    auto xv = [](XE t) -> float {
        if constexpr (XF) return t;
        else return bf2f(t);
    };
    constexpr int ED = kEdgeED, NT = kEhbThreads, P = kEhbParts;
    const int g = blockIdx.x, tid = threadIdx.x, k = tid & 255, part = tid >> 8;
    const int E = a.edges_per_graph, Hd = a.hidden, D = a.edge_dim, n = a.nodes_per_graph;
    // exact mode: the float p rows are read from global memory (L2) instead of
    // LDS, which then holds the [E][Hd] dz block and the sums within 160 KB
    XE* pr = reinterpret_cast<XE*>(smem);                               // [n][2*Hd] bf16 (exact: none)
    float* dzs = reinterpret_cast<float*>(pr + (XF ? 0 : (size_t)n * 2 * Hd));  // [E][Hd] dL/dz
    float* eal = dzs + (size_t)E * Hd;                                  // [E][ED] link features
    float* gl = eal + (size_t)E * ED;                                   // [E] grad logit
    float* red = gl + E;                                                // [P][2 + ED][256] per-part sums
    float* wes = red + P * (2 + ED) * 256;                              // [ED][256] link-feature weights
    int* sl = reinterpret_cast<int*>(wes + 256 * ED);                   // [E]
    int* dl = sl + E;                                                   // [E]
    int* lo = dl + E;                                                   // [E] links by source node, link order
    int* li = lo + E;                                                   // [E] links by destination node
    int* op = li + E;                                                   // [n+1] out-list offsets
    int* ip = op + n + 1;                                               // [n+1] in-list offsets
    const int64_t node0 = (int64_t)g * n;
    const XE* prow = XF ? static_cast<const XE*>(a.p) + node0 * 2 * Hd : pr;
    if (!XF) {
        const trx_u4* src4 = reinterpret_cast<const trx_u4*>(static_cast<const XE*>(a.p) + node0 * 2 * Hd);
        trx_u4* dst4 = reinterpret_cast<trx_u4*>(pr);
        for (int v = tid; v < n * 2 * Hd / EV; v += NT) dst4[v] = src4[v];
    }
    for (int e = tid; e < E; e += NT) {
        const int64_t eg = (int64_t)g * E + e;
        int s = (int)(a.src[eg] - node0), d = (int)(a.dst[eg] - node0);
        s = s < 0 ? 0 : (s >= n ? n - 1 : s);  // out-of-block links are refused on the host (topology check)
        d = d < 0 ? 0 : (d >= n ? n - 1 : d);
        sl[e] = s;
        dl[e] = d;
        gl[e] = grad_logits[eg];
    }
    for (int v = tid; v < E * ED; v += NT) {
        const int e = v / ED, j = v - (v / ED) * ED;
        eal[v] = j < D ? a.ea[((int64_t)g * E + e) * D + j] : 0.0f;
    }
    const bool on = k < Hd;
    float we[ED];
#pragma unroll
    for (int j = 0; j < ED; ++j) we[j] = (on && j < D) ? a.we[k * D + j] : 0.0f;
    if (part == 0)
#pragma unroll
        for (int j = 0; j < ED; ++j) wes[j * 256 + k] = we[j];   // unit-major per feature: (3) reads it conflict-free
    const float w2 = on ? a.w2[k] : 0.0f, ck = on ? a.c[(int64_t)g * Hd + k] : 0.0f;
    __syncthreads();
    if (tid < n) {  // per-node link lists (link order); counts first
        int co = 0, ci = 0;
        for (int e = 0; e < E; ++e) {
            co += sl[e] == tid;
            ci += dl[e] == tid;
        }
        op[tid + 1] = co;
        ip[tid + 1] = ci;
    }
    if (tid == 0) op[0] = ip[0] = 0;
    __syncthreads();
    if (tid == 0)
        for (int i = 0; i < n; ++i) {
            op[i + 1] += op[i];
            ip[i + 1] += ip[i];
        }
    __syncthreads();
    if (tid < n) {
        int wo = op[tid], wi = ip[tid];
        for (int e = 0; e < E; ++e) {
            if (sl[e] == tid) lo[wo++] = e;
            if (dl[e] == tid) li[wi++] = e;
        }
    }
    float gc = 0.0f, gw2 = 0.0f, gwe[ED];
#pragma unroll
    for (int j = 0; j < ED; ++j) gwe[j] = 0.0f;
    if (on) {  // (1) per link
        for (int e = part; e < E; e += P) {
            const int s = sl[e], d = dl[e];
            float ew = 0.0f;  // edge_head_infer_kernel's fused multiply-adds, same order
#pragma unroll
            for (int j = 0; j < ED; ++j)
                if (j < D) ew = __builtin_fmaf(eal[e * ED + j], we[j], ew);
            const float z = ((xv(prow[s * 2 * Hd + k]) + xv(prow[d * 2 * Hd + Hd + k])) + ew) + ck;
            const float gb = gl[e];
            gw2 += gb * fmaxf(z, 0.0f);
            const float dz = z > 0.0f ? gb * w2 : 0.0f;
            gc += dz;
#pragma unroll
            for (int j = 0; j < ED; ++j) gwe[j] += dz * eal[e * ED + j];
            if (grad_z) grad_z[((int64_t)g * E + e) * Hd + k] = f2bf(dz);
            dzs[e * Hd + k] = dz;
        }
    }
    constexpr int RS = 2 + ED;  // per-part rows: grad_c, grad_w2, grad_we[ED]
    red[(part * RS + 0) * 256 + k] = gc;
    red[(part * RS + 1) * 256 + k] = gw2;
#pragma unroll
    for (int j = 0; j < ED; ++j) red[(part * RS + 2 + j) * 256 + k] = gwe[j];
    __syncthreads();
    if (on && part == 0) {
        float t[RS];
#pragma unroll
        for (int r = 0; r < RS; ++r) t[r] = red[r * 256 + k];
#pragma unroll
        for (int q = 1; q < P; ++q)
#pragma unroll
            for (int r = 0; r < RS; ++r) t[r] += red[(q * RS + r) * 256 + k];
        grad_c[(int64_t)g * Hd + k] = t[0];
        grad_w2_part[(int64_t)g * Hd + k] = t[1];
        for (int j = 0; j < D; ++j) grad_we_part[((int64_t)g * Hd + k) * D + j] = t[2 + j];
    }
    // (3) per link: grad_ea[e, j] = sum_k dz[e, k] we[k, j], one wave per link
    {
        const int wv = tid >> 6, ln = tid & 63;
        for (int e = wv; e < E; e += NT / 64) {
            float s[ED];
#pragma unroll
            for (int j = 0; j < ED; ++j) s[j] = 0.0f;
            for (int kk = ln; kk < Hd; kk += 64) {
                const float dz = dzs[e * Hd + kk];
#pragma unroll
                for (int j = 0; j < ED; ++j) s[j] += dz * wes[j * 256 + kk];
            }
#pragma unroll
            for (int j = 0; j < ED; ++j) {
                const float t = wave_sum_f(s[j]);
                if (ln == 0 && j < D) grad_ea[((int64_t)g * E + e) * D + j] = t;
            }
        }
    }
    if (on)  // (2) per node: out-links feed p[:, :H], in-links p[:, H:]
        for (int i = part; i < n; i += P) {
            float so = 0.0f, si = 0.0f;
            for (int q = op[i]; q < op[i + 1]; ++q) so += dzs[lo[q] * Hd + k];
            for (int q = ip[i]; q < ip[i + 1]; ++q) si += dzs[li[q] * Hd + k];
            if constexpr (XF) {
                grad_p[(node0 + i) * 2 * Hd + k] = so;
                grad_p[(node0 + i) * 2 * Hd + Hd + k] = si;
            } else {
                grad_p[(node0 + i) * 2 * Hd + k] = f2bf(so);
                grad_p[(node0 + i) * 2 * Hd + Hd + k] = f2bf(si);
            }
        }
}

size_t edge_head_bwd_smem(const trx_edge_head_args& a) {
    const size_t n = a.nodes_per_graph, E = a.edges_per_graph, H = a.hidden;
    return (a.exact ? 0 : n * 2 * H * 2) + E * H * 4 + E * (kEdgeED * 4 + 4 + 16) + kEhbParts * (2 + kEdgeED) * 256 * 4 +
           256 * kEdgeED * 4 + 2 * (n + 1) * 4;
}

hipError_t launch_edge_head_bwd(const EdgeHeadBwdItem* items, int count, hipStream_t stream) {
    const trx_edge_head_args& a = items[0].a;
    const NetList<EdgeHeadBwdItem> l = net_list(items, count);
    const size_t smem = edge_head_bwd_smem(a);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    const void* fn = a.exact ? reinterpret_cast<const void*>(edge_head_bwd_kernel<true>)
                             : reinterpret_cast<const void*>(edge_head_bwd_kernel<false>);
    if (smem > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    if (a.exact)
        hipLaunchKernelGGL(edge_head_bwd_kernel<true>, dim3(a.num_graphs, count), dim3(kEhbThreads), smem, stream, l);
    else
        hipLaunchKernelGGL(edge_head_bwd_kernel<false>, dim3(a.num_graphs, count), dim3(kEhbThreads), smem, stream, l);
    return hipGetLastError();
}

template <int MQ, int DK, bool XF>
static hipError_t launch_edge_head_infer_t(const trx_edge_head_args* al, int count, size_t smem,
                                           hipStream_t stream) {
    if (smem > 64 * 1024) {  // opt in to more than 64 KB of dynamic LDS
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(edge_head_infer_kernel<MQ, DK, XF>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((edge_head_infer_kernel<MQ, DK, XF>), dim3(al[0].num_graphs, count), dim3(kInferThreads), smem,
                       stream, net_list(al, count));
    return hipGetLastError();
}

hipError_t launch_edge_head_infer(const trx_edge_head_args* al, int count, hipStream_t stream) {
    const trx_edge_head_args& a = al[0];
    const size_t smem = edge_head_infer_smem(a);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    const bool d6 = a.edge_dim == 6;  // the networks' link features (repair_env.py:800-808)
    if (a.exact) {
        if (a.hidden > 256) return hipErrorInvalidValue;
        return d6 ? launch_edge_head_infer_t<1, 6, true>(al, count, smem, stream)
                  : launch_edge_head_infer_t<1, 0, true>(al, count, smem, stream);
    }
    if (a.hidden <= 256)
        return d6 ? launch_edge_head_infer_t<1, 6, false>(al, count, smem, stream)
                  : launch_edge_head_infer_t<1, 0, false>(al, count, smem, stream);
    return d6 ? launch_edge_head_infer_t<2, 6, false>(al, count, smem, stream)
              : launch_edge_head_infer_t<2, 0, false>(al, count, smem, stream);
}

}  // namespace trx

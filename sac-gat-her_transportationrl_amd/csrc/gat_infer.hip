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

}  // namespace

// ------------------------------------------------------------- layer kernel
// IN: 0 = xh given (layers >= 1), else the layer-0 input width (4).
template <int HC, int IN>
__global__ void __launch_bounds__(kInferThreads) gat_layer_infer_kernel(trx_gat_layer_args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int KC = HC / 256;  // float4 chunks per lane in a row
    const int g = blockIdx.x;
    const int n = a.nodes_per_graph, H = a.heads, C = a.channels;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
    const int node0 = g * n;
    const int ebeg = a.rowptr[node0];
    const int ne = a.rowptr[node0 + n] - ebeg;
    if (ne > a.max_graph_edges || ne < 0) {  // LDS was sized for max_graph_edges: poison, do not overrun
        for (int idx = tid; idx < n * HC; idx += kInferThreads) {
            if (a.out_f32) a.out_f32[(size_t)node0 * HC + idx] = __builtin_nanf("");
            if (a.out_bf16) static_cast<uint16_t*>(a.out_bf16)[(size_t)node0 * HC + idx] = 0x7fc0;
        }
        if (a.pool)
            for (int f = tid; f < 2 * HC; f += kInferThreads) a.pool[(size_t)g * 2 * HC + f] = __builtin_nanf("");
        return;
    }

    const int SL = C < 64 ? C : 64, S = C / SL;          // attention dot-product segments
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem);   // [n][HC] bf16
    float* as_ = reinterpret_cast<float*>(xs + n * HC);  // [n*H]
    float* ad_ = as_ + n * H;                            // [n*H]
    const int alsz = a.max_graph_edges * H > 2 * n * H * S ? a.max_graph_edges * H : 2 * n * H * S;
    float* al = ad_ + n * H;        // [me*H] edge logits, then attention weights (in place)
    float* part = al;               // [2*n*H*S] partial dot products (step 2 only, aliases al)
    int* cl = reinterpret_cast<int*>(al + alsz);         // [me] source, graph-local
    int* rp = cl + a.max_graph_edges;                    // [n+1] graph-local row pointers
    float* x0l = reinterpret_cast<float*>(rp + n + 1);   // [n*IN]
    float* yt = x0l + n * IN;                            // [n][HC] (pool only)

    // 0. graph-local CSR slice, edge logits, layer-0 inputs
    for (int v = tid; v <= n; v += kInferThreads) rp[v] = a.rowptr[node0 + v] - ebeg;
    for (int v = tid; v < ne; v += kInferThreads) cl[v] = a.col[ebeg + v] - node0;
    if (IN > 0)
        for (int v = tid; v < n * IN; v += kInferThreads) x0l[v] = bf16r(a.x0[(size_t)node0 * IN + v]);
    if (IN == 0) {
        const uint4* src = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.xh) + (size_t)node0 * HC);
        uint4* dst4 = reinterpret_cast<uint4*>(xs);
        for (int v = tid; v < n * HC / 8; v += kInferThreads) dst4[v] = src[v];
    }
    __syncthreads();

    // 1. layer 0: xh = bf16(bf16(x0) @ w0^T), weights of a thread's columns in registers
    if (IN > 0) {
        constexpr int INR = IN > 0 ? IN : 1;
#pragma unroll
        for (int m = 0; m < KC; ++m) {
            const int f = tid + kInferThreads * m;
            float w[INR];
#pragma unroll
            for (int j = 0; j < IN; ++j) w[j] = a.w0[(size_t)f * IN + j];
            for (int i = 0; i < n; ++i) {
                float acc = 0.0f;
#pragma unroll
                for (int j = 0; j < IN; ++j) acc += x0l[i * IN + j] * w[j];
                xs[i * HC + f] = f2bf(acc);
            }
        }
        __syncthreads();
    }

    // 2. attention dot products <xh[i,h,:], att[h,:]>: every thread takes
    //    (node, head, 64-wide segment) units, partials are combined in order
    {
        for (int u = tid; u < n * H * S; u += kInferThreads) {
            const int sg = u % S, ih = u / S, i = ih / H, h = ih - (ih / H) * H;
            const uint16_t* xr = xs + i * HC + h * C + sg * SL;
            const float4* s_att = reinterpret_cast<const float4*>(a.att_src + h * C + sg * SL);
            const float4* d_att = reinterpret_cast<const float4*>(a.att_dst + h * C + sg * SL);
            float s1 = 0.0f, s2 = 0.0f;
            for (int c = 0; c < SL; c += 8) {
                const uint4 q = *reinterpret_cast<const uint4*>(xr + c);
                const float4 sa0 = s_att[c / 4], sa1 = s_att[c / 4 + 1];
                const float4 da0 = d_att[c / 4], da1 = d_att[c / 4 + 1];
                const float v[8] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                                    __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u),
                                    __uint_as_float(q.z << 16), __uint_as_float(q.z & 0xffff0000u),
                                    __uint_as_float(q.w << 16), __uint_as_float(q.w & 0xffff0000u)};
                const float sa[8] = {sa0.x, sa0.y, sa0.z, sa0.w, sa1.x, sa1.y, sa1.z, sa1.w};
                const float da[8] = {da0.x, da0.y, da0.z, da0.w, da1.x, da1.y, da1.z, da1.w};
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    s1 += v[r] * sa[r];
                    s2 += v[r] * da[r];
                }
            }
            part[2 * u] = s1;
            part[2 * u + 1] = s2;
        }
        __syncthreads();
        for (int t = tid; t < n * H; t += kInferThreads) {
            float s1 = 0.0f, s2 = 0.0f;
            for (int sg = 0; sg < S; ++sg) {
                s1 += part[2 * (t * S + sg)];
                s2 += part[2 * (t * S + sg) + 1];
            }
            as_[t] = s1;  // t = i*H + h
            ad_[t] = s2;
        }
        __syncthreads();
        for (int v = tid; v < ne * H; v += kInferThreads) {  // edge logits of this layer into al
            const int e = v / H, h = v - e * H;
            al[v] = a.a_edge[(size_t)(ebeg + e) * a.a_edge_stride + a.a_edge_offset + h];
        }
    }
    __syncthreads();

    // 3. softmax over in-edges: one thread per (node, head), LDS only
    for (int t = tid; t < n * H; t += kInferThreads) {
        const int i = t / H, h = t - (t / H) * H;
        const int p0 = rp[i], p1 = rp[i + 1];
        const float ad = ad_[t];
        float m = -__builtin_huge_valf();
        for (int p = p0; p < p1; ++p) m = fmaxf(m, leaky_f(as_[cl[p] * H + h] + ad + al[p * H + h], a.negative_slope));
        float ssum = 0.0f;
        for (int p = p0; p < p1; ++p)
            ssum += __expf(leaky_f(as_[cl[p] * H + h] + ad + al[p * H + h], a.negative_slope) - m);
        const float denom = ssum + 1e-16f;
        for (int p = p0; p < p1; ++p)  // in place: logit -> attention weight
            al[p * H + h] = __expf(leaky_f(as_[cl[p] * H + h] + ad + al[p * H + h], a.negative_slope) - m) / denom;
    }
    __syncthreads();

    // 4. aggregation + epilogue, one wave per node; lane owns chunks q = lane + 64k.
    //    Per-column constants live in registers across the wave's nodes.
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
    for (int i = wave; i < n; i += kInferWaves) {
        const int node = node0 + i;
        float4 res4[KC];  // issue the residual loads before the aggregation (latency overlap)
#pragma unroll
        for (int k = 0; k < KC; ++k)
            res4[k] = a.residual == 1 ? *reinterpret_cast<const float4*>(a.res + (size_t)node * HC + 4 * (lane + kWave * k))
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 acc[KC];
#pragma unroll
        for (int k = 0; k < KC; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int p = rp[i]; p < rp[i + 1]; ++p) {
            const uint16_t* row = xs + cl[p] * HC;
            const float* alr = al + p * H;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const int q = lane + kWave * k;
                const float w = alr[(4 * q) / C];
                const uint2 u = *reinterpret_cast<const uint2*>(row + 4 * q);
                acc[k].x += w * __uint_as_float(u.x << 16);
                acc[k].y += w * __uint_as_float(u.x & 0xffff0000u);
                acc[k].z += w * __uint_as_float(u.y << 16);
                acc[k].w += w * __uint_as_float(u.y & 0xffff0000u);
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
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int f0 = 4 * (lane + kWave * k);
            const float resv[4] = {res4[k].x, res4[k].y, res4[k].z, res4[k].w};
            float y4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float y = lnw_r[k][r] * (rstd * (v[k][r] - mean)) + lnb_r[k][r];
                if (IN > 0 && a.residual == 2) {
                    float t = 0.0f;
#pragma unroll
                    for (int j = 0; j < (IN > 0 ? IN : 1); ++j) t += x0l[i * IN + j] * wp_r[k][r][j];
                    y = y + bf16r(t + bp_r[k][r]);
                } else if (a.residual == 1) {
                    y = y + resv[r];
                }
                if (a.activation == 0)
                    y = y > 0.0f ? y : 0.0f;
                else
                    y = y <= 0.0f ? (expf(y) - 1.0f) : y;
                y4[r] = y;
                if (a.pool) yt[i * HC + f0 + r] = y;
            }
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
    if (a.pool) {
        __syncthreads();
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
    }
}

// --------------------------------------------------------- edge scorer
// One workgroup per graph, one wave per link; lane owns hidden units
// k = lane + 64m (hidden <= 512), whose weights stay in registers.
template <int MK>  // hidden <= 64 * MK
__global__ void __launch_bounds__(kInferThreads) edge_head_infer_kernel(trx_edge_head_args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* lg = reinterpret_cast<float*>(smem);  // [E]
    const int g = blockIdx.x;
    const int E = a.edges_per_graph, Hd = a.hidden, D = a.edge_dim;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
    const uint16_t* p = static_cast<const uint16_t*>(a.p);
    constexpr int ED = 8;  // edge_dim <= 8
    float we_r[MK][ED], w2_r[MK], c_r[MK];
#pragma unroll
    for (int m = 0; m < MK; ++m) {
        const int k = lane + kWave * m;
        const bool ok = k < Hd;
        w2_r[m] = ok ? a.w2[k] : 0.0f;
        c_r[m] = ok ? a.c[(size_t)g * Hd + k] : 0.0f;
#pragma unroll
        for (int j = 0; j < ED; ++j) we_r[m][j] = (ok && j < D) ? a.we[k * D + j] : 0.0f;
    }
    const float b2 = a.b2[0];
    constexpr int EU = 2;  // links per wave iteration: independent loads in flight together
    for (int e0 = wave * EU; e0 < E; e0 += kInferWaves * EU) {
        float ear[EU][ED];
        const uint16_t* ps[EU];
        const uint16_t* pd[EU];
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const int e = e0 + u < E ? e0 + u : E - 1;
            const int eg = g * E + e;
#pragma unroll
            for (int j = 0; j < ED; ++j) ear[u][j] = j < D ? bf16r(a.ea[(size_t)eg * D + j]) : 0.0f;
            ps[u] = p + (size_t)a.src[eg] * 2 * Hd;
            pd[u] = p + (size_t)a.dst[eg] * 2 * Hd + Hd;
        }
        float part[EU];
#pragma unroll
        for (int u = 0; u < EU; ++u) part[u] = 0.0f;
#pragma unroll
        for (int m = 0; m < MK; ++m) {
            const int k = lane + kWave * m;
            if (k < Hd) {
#pragma unroll
                for (int u = 0; u < EU; ++u) {
                    float ew = 0.0f;
#pragma unroll
                    for (int j = 0; j < ED; ++j)
                        if (j < D) ew += ear[u][j] * we_r[m][j];
                    const float z1 = bf16r(bf2f(ps[u][k]) + bf2f(pd[u][k]));
                    const float z2 = bf16r(z1 + bf16r(ew));
                    const float z3 = z2 + c_r[m];
                    part[u] += bf16r(fmaxf(z3, 0.0f)) * w2_r[m];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const float t = wave_sum_f(part[u]);
            if (lane == 0 && e0 + u < E) lg[e0 + u] = bf16r(t + b2);
        }
    }
    __syncthreads();
    if (!a.softmax) {
        for (int e = tid; e < E; e += kInferThreads) a.out[(size_t)g * E + e] = lg[e];
        return;
    }
    if (wave != 0) return;
    if (a.logits)
        for (int e = lane; e < E; e += kWave)
            a.logits[(size_t)g * E + e] = a.mask[(size_t)g * E + e] <= 0.0f ? -1e9f : lg[e];
    float m = -__builtin_huge_valf();
    for (int e0 = 0; e0 < E; e0 += kWave) {
        const int e = e0 + lane;
        float x = -__builtin_huge_valf();
        if (e < E) x = a.mask[(size_t)g * E + e] <= 0.0f ? -1e9f : lg[e];
        m = fmaxf(m, wave_max_f(x));
    }
    float ssum = 0.0f;
    for (int e0 = 0; e0 < E; e0 += kWave) {
        const int e = e0 + lane;
        float ex = 0.0f;
        if (e < E) ex = expf((a.mask[(size_t)g * E + e] <= 0.0f ? -1e9f : lg[e]) - m);
        ssum += wave_sum_f(ex);
    }
    const float denom = ssum + 1e-16f;
    for (int e0 = 0; e0 < E; e0 += kWave) {
        const int e = e0 + lane;
        if (e < E) a.out[(size_t)g * E + e] = expf((a.mask[(size_t)g * E + e] <= 0.0f ? -1e9f : lg[e]) - m) / denom;
    }
}

size_t gat_layer_infer_smem(const trx_gat_layer_args& a) {
    const int HC = a.heads * a.channels, n = a.nodes_per_graph, H = a.heads, me = a.max_graph_edges;
    const int SL = a.channels < 64 ? a.channels : 64, S = a.channels / SL;
    const size_t alsz = (size_t)me * H > 2 * (size_t)n * H * S ? (size_t)me * H : 2 * (size_t)n * H * S;
    size_t b = (size_t)n * HC * 2 + 2 * (size_t)n * H * 4 + alsz * 4 + (size_t)me * 4 + (size_t)(n + 1) * 4 +
               (size_t)n * a.in_dim * 4;
    if (a.pool) b += (size_t)n * HC * 4;
    return b;
}

template <int HC, int IN>
static void set_lds_attr() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gat_layer_infer_kernel<HC, IN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

hipError_t launch_gat_layer_infer(const trx_gat_layer_args& a, hipStream_t stream) {
    const int HC = a.heads * a.channels;
    const size_t smem = gat_layer_infer_smem(a);
    static bool attr_set = false;
    if (!attr_set) {  // allow > 64 KB of dynamic LDS (gfx950: 160 KB per CU)
        set_lds_attr<1024, 0>();
        set_lds_attr<1024, 4>();
        set_lds_attr<512, 0>();
        set_lds_attr<512, 4>();
        set_lds_attr<256, 0>();
        set_lds_attr<256, 4>();
        attr_set = true;
    }
    const dim3 grid(a.num_graphs), block(kInferThreads);
#define TRX_LAYER_CASE(HCV, INV)                                                                         \
    if (HC == HCV && a.in_dim == INV) {                                                                  \
        hipLaunchKernelGGL((gat_layer_infer_kernel<HCV, INV>), grid, block, smem, stream, a);            \
        return hipGetLastError();                                                                        \
    }
    TRX_LAYER_CASE(1024, 0)
    TRX_LAYER_CASE(1024, 4)
    TRX_LAYER_CASE(512, 0)
    TRX_LAYER_CASE(512, 4)
    TRX_LAYER_CASE(256, 0)
    TRX_LAYER_CASE(256, 4)
#undef TRX_LAYER_CASE
    return hipErrorInvalidValue;
}

hipError_t launch_edge_head_infer(const trx_edge_head_args& a, hipStream_t stream) {
    const size_t smem = (size_t)a.edges_per_graph * sizeof(float);
    if (a.hidden <= 256)
        hipLaunchKernelGGL(edge_head_infer_kernel<4>, dim3(a.num_graphs), dim3(kInferThreads), smem, stream, a);
    else
        hipLaunchKernelGGL(edge_head_infer_kernel<8>, dim3(a.num_graphs), dim3(kInferThreads), smem, stream, a);
    return hipGetLastError();
}

}  // namespace trx

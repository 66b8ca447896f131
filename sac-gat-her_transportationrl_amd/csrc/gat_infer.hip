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

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ float leaky_f(float x, float slope) { return x > 0.0f ? x : x * slope; }

// fp32 -> bf16 bits, round to nearest even (torch's conversion)
__device__ __forceinline__ uint16_t f2bf(float x) {
    uint32_t u = __float_as_uint(x);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
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

    uint16_t* xs = reinterpret_cast<uint16_t*>(smem);   // [n][HC] bf16
    float* as_ = reinterpret_cast<float*>(xs + n * HC);  // [n*H]
    float* ad_ = as_ + n * H;                            // [n*H]
    float* al = ad_ + n * H;                             // [ne*H] attention weights
    float* ae = al + a.max_graph_edges * H;              // [ne*H] edge logits of this layer
    int* cl = reinterpret_cast<int*>(ae + a.max_graph_edges * H);  // [ne] source, graph-local
    int* rp = cl + a.max_graph_edges;                    // [n+1] graph-local row pointers
    float* x0l = reinterpret_cast<float*>(rp + 33);      // [n*IN]
    float* yt = x0l + 32 * (IN > 0 ? IN : 1);            // [n][HC] (pool only)

    // 0. graph-local CSR slice, edge logits, layer-0 inputs
    for (int v = tid; v <= n; v += kInferThreads) rp[v] = a.rowptr[node0 + v] - ebeg;
    for (int v = tid; v < ne; v += kInferThreads) cl[v] = a.col[ebeg + v] - node0;
    for (int v = tid; v < ne * H; v += kInferThreads) {
        const int e = v / H, h = v - e * H;
        ae[v] = a.a_edge[(size_t)(ebeg + e) * a.a_edge_stride + a.a_edge_offset + h];
    }
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

    // 2. attention dot products: unit u = (h, i), h-major so a wave keeps att in registers
    {
        int hcur = -1;
        float ats[4], atd[4];  // C <= 256: c = lane + 64m
        for (int u = wave; u < n * H; u += kInferWaves) {
            const int h = u / n, i = u - h * n;
            if (h != hcur) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int c = lane + kWave * m;
                    ats[m] = c < C ? a.att_src[h * C + c] : 0.0f;
                    atd[m] = c < C ? a.att_dst[h * C + c] : 0.0f;
                }
                hcur = h;
            }
            float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int c = lane + kWave * m;
                if (c < C) {
                    const float v = bf2f(xs[i * HC + h * C + c]);
                    s1 += v * ats[m];
                    s2 += v * atd[m];
                }
            }
            s1 = wave_sum_f(s1);
            s2 = wave_sum_f(s2);
            if (lane == 0) {
                as_[i * H + h] = s1;
                ad_[i * H + h] = s2;
            }
        }
    }
    __syncthreads();

    // 3. softmax over in-edges: one thread per (node, head), LDS only
    for (int t = tid; t < n * H; t += kInferThreads) {
        const int i = t / H, h = t - (t / H) * H;
        const int p0 = rp[i], p1 = rp[i + 1];
        const float ad = ad_[t];
        float m = -__builtin_huge_valf();
        for (int p = p0; p < p1; ++p) m = fmaxf(m, leaky_f(as_[cl[p] * H + h] + ad + ae[p * H + h], a.negative_slope));
        float ssum = 0.0f;
        for (int p = p0; p < p1; ++p)
            ssum += __expf(leaky_f(as_[cl[p] * H + h] + ad + ae[p * H + h], a.negative_slope) - m);
        const float denom = ssum + 1e-16f;
        for (int p = p0; p < p1; ++p)
            al[p * H + h] = __expf(leaky_f(as_[cl[p] * H + h] + ad + ae[p * H + h], a.negative_slope) - m) / denom;
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
            float4 res4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.residual == 1) res4 = *reinterpret_cast<const float4*>(a.res + (size_t)node * HC + f0);
            const float resv[4] = {res4.x, res4.y, res4.z, res4.w};
            float y4[4];
            uint16_t ob[4];
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
                ob[r] = f2bf(y);
                if (a.pool) yt[i * HC + f0 + r] = y;
            }
            if (a.out_f32)
                *reinterpret_cast<float4*>(a.out_f32 + (size_t)node * HC + f0) = make_float4(y4[0], y4[1], y4[2], y4[3]);
            if (a.out_bf16) {
                uint2 u;
                u.x = (uint32_t)ob[0] | ((uint32_t)ob[1] << 16);
                u.y = (uint32_t)ob[2] | ((uint32_t)ob[3] << 16);
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
    for (int e = wave; e < E; e += kInferWaves) {
        const int eg = g * E + e;
        const int s = a.src[eg], d = a.dst[eg];
        float ear[ED];
#pragma unroll
        for (int j = 0; j < ED; ++j) ear[j] = j < D ? bf16r(a.ea[(size_t)eg * D + j]) : 0.0f;
        const uint16_t* ps = p + (size_t)s * 2 * Hd;
        const uint16_t* pd = p + (size_t)d * 2 * Hd + Hd;
        float part = 0.0f;
#pragma unroll
        for (int m = 0; m < MK; ++m) {
            const int k = lane + kWave * m;
            if (k < Hd) {
                float ew = 0.0f;
#pragma unroll
                for (int j = 0; j < ED; ++j)
                    if (j < D) ew += ear[j] * we_r[m][j];
                const float z1 = bf16r(bf2f(ps[k]) + bf2f(pd[k]));
                const float z2 = bf16r(z1 + bf16r(ew));
                const float z3 = z2 + c_r[m];
                part += bf16r(fmaxf(z3, 0.0f)) * w2_r[m];
            }
        }
        const float t = wave_sum_f(part);
        if (lane == 0) lg[e] = bf16r(t + b2);
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
    size_t b = (size_t)n * HC * 2 + 2 * (size_t)n * H * 4 + 2 * (size_t)me * H * 4 + (size_t)me * 4 + 33 * 4 +
               32 * 4 * (a.in_dim > 0 ? a.in_dim : 1);
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

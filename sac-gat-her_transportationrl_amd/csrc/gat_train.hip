// gat_train.hip -- fused backward of the GAT-SAC networks for the SAC update
// (src/rl/sac.py:157-243 through src/models/gat_encoder.py:32-53), gfx950.
//
// The update's training forwards run the fused inference kernels
// (gat_infer.hip) with their save_* outputs; the backward of one network is
// then a handful of launches instead of hundreds of autograd ops:
//   * trx_gat_layer_backward: one workgroup per graph for a whole GATConv
//     layer + its tail -- activation (ReLU / ELU), residual, LayerNorm,
//     bias, neighbour aggregation, edge softmax, leaky ReLU and the attention
//     dot products (and, on layer 0, the in-kernel 4 -> H*C projection and the
//     input_proj residual; on the last layer the mean|max pooling).  Outputs:
//     the bf16 gradient of the layer's `lin` output (its weight / input
//     gradients are GEMMs on the host side), the residual's gradient, the edge
//     logits' gradient, and per-graph partial sums of every per-column
//     parameter gradient (reduced in a fixed order by trx_partial_sum: no
//     float atomics, deterministic);
//   * trx_gat_prologue_backward: the input LayerNorms, the self-loop mean
//     edge attributes and every layer's edge-logit projection, one wave per graph;
//   * trx_sac_loss: the three SAC losses of sac.py:184-219 with their
//     gradients w.r.t. the critics' Q values, the actor's logits and log_alpha
//     written directly (the losses are closed-form in those tensors).
// All arithmetic is float32 on bf16-rounded operands exactly where the forward
// rounded; gradients of bf16 tensors are rounded to bf16 once (autocast's
// dtype rules), parameter gradients stay float32.
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kW = 64;
constexpr int kT = 256;  // threads per workgroup

#define TRX_TDPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, false))
__device__ __forceinline__ float wsum(float v) {
    v = v + TRX_TDPP(v, 0xB1);
    v = v + TRX_TDPP(v, 0x4E);
    v = v + TRX_TDPP(v, 0x141);
    v = v + TRX_TDPP(v, 0x140);
    return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
           (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}
__device__ __forceinline__ float rsum16(float v) {
    v = v + TRX_TDPP(v, 0xB1);
    v = v + TRX_TDPP(v, 0x4E);
    v = v + TRX_TDPP(v, 0x141);
    v = v + TRX_TDPP(v, 0x140);
    return v;
}
#undef TRX_TDPP

typedef float tf2 __attribute__((ext_vector_type(2)));
typedef __bf16 tb2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pkbf(float lo, float hi) {
    const tf2 v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, tb2));
}
__device__ __forceinline__ uint16_t tobf(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ __forceinline__ float frbf(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ float rbf(float x) { return frbf(tobf(x)); }
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// xh / g_xh row elements: bf16 bits, or float32 in the exact mode
template <bool XF> struct XE_ { typedef uint16_t T; };
template <> struct XE_<true> { typedef float T; };
template <bool XF>
__device__ __forceinline__ float4 ld4x(const typename XE_<XF>::T* p) {
    if constexpr (XF) {
        return *reinterpret_cast<const float4*>(p);
    } else {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        return make_float4(lo_bf(u.x), hi_bf(u.x), lo_bf(u.y), hi_bf(u.y));
    }
}
// store four values (bf16: rounded); returns the values as stored
template <bool XF>
__device__ __forceinline__ float4 st4x(typename XE_<XF>::T* p, float a, float b, float c, float d) {
    if constexpr (XF) {
        *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
        return make_float4(a, b, c, d);
    } else {
        uint2 u;
        u.x = pkbf(a, b);
        u.y = pkbf(c, d);
        *reinterpret_cast<uint2*>(p) = u;
        return make_float4(lo_bf(u.x), hi_bf(u.x), lo_bf(u.y), hi_bf(u.y));
    }
}

}  // namespace

// ------------------------------------------------------------ layer backward
// Partial-sum layout per graph (floats): [0,F) bias, [F,2F) ln weight, [2F,3F) ln
// bias, [3F,4F) att_src, [4F,5F) att_dst; layer 0 adds [5F,9F) lin.weight (F x 4,
// row-major), [9F,13F) input_proj.weight, [13F,14F) input_proj.bias.  F = heads*channels.
template <int HC, int IN, int NT, bool XF>
__global__ void __launch_bounds__(NT) gat_layer_bwd_kernel(const NetList<trx_gat_layer_bwd_args> nets) {
    const trx_gat_layer_bwd_args& a = nets.a[blockIdx.y];  // network blockIdx.y (*_multi launches)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename XE_<XF>::T XE;
    constexpr int EV = 16 / sizeof(XE);
    // exact mode at HC 1024: float xh rows and float gv rows do not both fit in
    // LDS; xh is then read from global memory (layers >= 1) or recomputed from
    // the 4 inputs (layer 0, the same arithmetic as the staged rows)
    constexpr bool XG = XF && HC > 512;
    constexpr int KC = HC / 256;  // float4 chunks per lane in a row
    constexpr int kT = NT, kNW = NT / kW;  // threads / waves per workgroup
    constexpr int INR = IN > 0 ? IN : 1;
    const int g = blockIdx.x;
    const int n = a.nodes_per_graph, H = a.heads, C = a.channels;
    const int tid = threadIdx.x, lane = tid & (kW - 1), wave = tid / kW;
    const int node0 = g * n;
    const int ebeg = a.rowptr[node0];
    const int ne = a.rowptr[node0 + n] - ebeg;
    const int sbeg = a.sptr[node0];
    if (ne > a.max_graph_edges || ne < 0 || a.sptr[node0 + n] - sbeg != ne) return;  // host checks the topology

    // rows padded by 16 B: phase C1 reads four pairs' rows per wave instruction,
    // which unpadded 2 KB / 4 KB strides put on the same LDS banks
    constexpr int XS = HC + EV, GS = HC + 4;
    XE* xs = reinterpret_cast<XE*>(smem);                      // [n][XS] bf16 lin output (exact: float; XG: none)
    float* w0s = reinterpret_cast<float*>(smem);               // XG, layer 0: [HC][IN] lin.weight (for the xh recompute)
    float* gv = XG ? w0s + (IN > 0 ? HC * IN : 0)
                   : reinterpret_cast<float*>(xs + n * XS);    // [n][GS] dL/d(aggregate + bias)
    float* al = gv + n * GS;                                   // [me*H] attention weights
    float* ge = al + a.max_graph_edges * H;                    // [me*H] dL/dalpha, then dL/de
    float* asd = ge + a.max_graph_edges * H;                   // [n][2H] a_src | a_dst
    float* gas = asd + 2 * n * H;                              // [n][H] dL/da_src
    float* gad = gas + n * H;                                  // [n][H] dL/da_dst
    float* st = gad + n * H;                                   // [n][2] mean, rstd
    float* x0l = st + 2 * n;                                   // [n][4] bf16-rounded layer-0 input
    float* gx0 = x0l + 4 * n;                                  // [n][4] dL/dx0 (residual part)
    float* pmx = gx0 + 4 * n;                                  // [HC] pool: column max
    float* pti = pmx + (a.g_pool ? HC : 0);                    // [HC] pool: ties
    int* cl = reinterpret_cast<int*>(pti + (a.g_pool ? HC : 0));  // [me] source (local) per CSR position
    int* dl = cl + a.max_graph_edges;                          // [me] destination (local)
    int* rp = dl + a.max_graph_edges;                          // [n+1]
    int* sp = rp + n + 1;                                      // [n+1] source CSR
    int* spp = sp + n + 1;                                     // [me] local dst-CSR position per source entry

    // ---- setup: CSR slices, saved small tensors, xh rows (layer 0: recomputed)
    for (int t = tid; t <= n; t += kT) {
        rp[t] = a.rowptr[node0 + t] - ebeg;
        sp[t] = a.sptr[node0 + t] - sbeg;
    }
    for (int p = tid; p < ne; p += kT) {
        cl[p] = a.col[ebeg + p] - node0;
        spp[p] = a.spos[sbeg + p] - ebeg;
    }
    for (int v = tid; v < ne * H; v += kT) al[v] = a.alpha[(size_t)ebeg * H + v];
    for (int v = tid; v < 2 * n * H; v += kT) asd[v] = a.asd[(size_t)node0 * 2 * H + v];
    for (int v = tid; v < 2 * n; v += kT) st[v] = a.stats[(size_t)node0 * 2 + v];
    if (IN > 0)
        for (int v = tid; v < n * IN; v += kT) {
            x0l[v] = XF ? a.x0[(size_t)node0 * IN + v] : rbf(a.x0[(size_t)node0 * IN + v]);
            gx0[v] = 0.0f;
        }
    if (XG && IN > 0)  // every xh recompute below reads the weights from LDS, not per term from global memory
        for (int v = tid; v < HC * IN; v += kT) w0s[v] = a.w0[v];
    if (IN == 0 && !XG) {
        const uint4* src = reinterpret_cast<const uint4*>(static_cast<const XE*>(a.xh) + (size_t)node0 * HC);
        constexpr int Q8 = HC / EV;
        for (int v = tid; v < n * Q8; v += kT)
            *reinterpret_cast<uint4*>(xs + (v / Q8) * XS + (v - (v / Q8) * Q8) * EV) = src[v];
    }
    __syncthreads();
    for (int i = tid; i < n; i += kT)
        for (int p = rp[i]; p < rp[i + 1]; ++p) dl[p] = i;
    if (IN > 0 && !XG) {  // xh = bf16(x0l @ w0^T), the forward's arithmetic (gat_infer.hip phase 1)
        for (int q = tid; q < HC / 4; q += kT) {
            float w[4][INR];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < INR; ++j) w[r][j] = a.w0[(size_t)(4 * q + r) * IN + j];
            for (int i = 0; i < n; ++i) {
                float acc[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc[r] = 0.0f;
#pragma unroll
                    for (int j = 0; j < INR; ++j) acc[r] += x0l[i * IN + j] * w[r][j];
                }
                st4x<XF>(xs + i * XS + 4 * q, acc[0], acc[1], acc[2], acc[3]);
            }
        }
    }
    // xh[i, col..col+3] as floats (staged rows, or the XG sources above)
    auto xget4 = [&](int i, int col) -> float4 {
        if constexpr (!XG) {
            return ld4x<XF>(xs + i * XS + col);
        } else if constexpr (IN == 0) {
            return *reinterpret_cast<const float4*>(static_cast<const float*>(a.xh) + (size_t)(node0 + i) * HC + col);
        } else {
            float acc[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc[r] = 0.0f;
#pragma unroll
                for (int j = 0; j < INR; ++j) acc[r] += x0l[i * IN + j] * w0s[(col + r) * IN + j];
            }
            return make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
    };
    if (a.g_pool) {  // column max and its multiplicity over the graph's rows (torch amax backward)
        for (int c = tid; c < HC; c += kT) {
            float mx = -__builtin_huge_valf(), cnt = 0.0f;
            for (int i = 0; i < n; ++i) {
                const float y = a.y[(size_t)(node0 + i) * HC + c];
                if (y > mx) {
                    mx = y;
                    cnt = 1.0f;
                } else if (y == mx) {
                    cnt += 1.0f;
                }
            }
            pmx[c] = mx;
            pti[c] = cnt;
        }
    }
    __syncthreads();

    // ---- A: wave per node -- activation, residual, LayerNorm backward -> gv
    float wp_r[KC][4][INR];
    if (IN > 0 && a.residual == 2) {
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < INR; ++j) wp_r[k][r][j] = a.wp[(size_t)(4 * (lane + kW * k) + r) * IN + j];
    }
    for (int i = wave; i < n; i += kNW) {
        const size_t row = (size_t)(node0 + i) * HC;
        const float mean = st[2 * i], rstd = st[2 * i + 1];
        float gx[KC][4], xh_[KC][4];
        float s1 = 0.0f, s2 = 0.0f;
        float rx[INR];
#pragma unroll
        for (int j = 0; j < INR; ++j) rx[j] = 0.0f;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int f0 = 4 * (lane + kW * k);
            float4 gy = a.gy ? *reinterpret_cast<const float4*>(a.gy + row + f0) : make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.gy_bf16) {
                const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(a.gy_bf16) + row + f0);
                gy.x += lo_bf(u.x);
                gy.y += hi_bf(u.x);
                gy.z += lo_bf(u.y);
                gy.w += hi_bf(u.y);
            }
            const float4 y4 = *reinterpret_cast<const float4*>(a.y + row + f0);
            const float4 v4 = *reinterpret_cast<const float4*>(a.v + row + f0);
            const float gyv[4] = {gy.x, gy.y, gy.z, gy.w}, yv[4] = {y4.x, y4.y, y4.z, y4.w},
                        vv[4] = {v4.x, v4.y, v4.z, v4.w};
            float gt[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float gyr = gyv[r];
                if (a.g_pool) {
                    const float* gp = a.g_pool + (size_t)g * 2 * HC;
                    gyr += gp[f0 + r] / (float)n;
                    if (yv[r] == pmx[f0 + r]) gyr += gp[HC + f0 + r] / pti[f0 + r];
                }
                // relu'(t) = [y > 0]; elu'(t) = 1 (t > 0) or exp(t) = y + 1
                gt[r] = a.activation == 0 ? (yv[r] > 0.0f ? gyr : 0.0f) : (yv[r] > 0.0f ? gyr : gyr * (yv[r] + 1.0f));
                xh_[k][r] = (vv[r] - mean) * rstd;
                gx[k][r] = gt[r] * a.ln_weight[f0 + r];
                s1 += gx[k][r];
                s2 += gx[k][r] * xh_[k][r];
                if (IN > 0 && a.residual == 2) {
#pragma unroll
                    for (int j = 0; j < INR; ++j) rx[j] += gt[r] * wp_r[k][r][j];
                }
            }
            if (a.g_res) *reinterpret_cast<float4*>(a.g_res + row + f0) = make_float4(gt[0], gt[1], gt[2], gt[3]);
        }
        const float m1 = wsum(s1) / (float)HC, m2 = wsum(s2) / (float)HC;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int f0 = 4 * (lane + kW * k);
            float4 o;
            o.x = rstd * (gx[k][0] - m1 - xh_[k][0] * m2);
            o.y = rstd * (gx[k][1] - m1 - xh_[k][1] * m2);
            o.z = rstd * (gx[k][2] - m1 - xh_[k][2] * m2);
            o.w = rstd * (gx[k][3] - m1 - xh_[k][3] * m2);
            *reinterpret_cast<float4*>(gv + i * GS + f0) = o;
        }
        if (IN > 0 && a.residual == 2) {
#pragma unroll
            for (int j = 0; j < INR; ++j) {
                const float t = wsum(rx[j]);
                if (lane == 0) gx0[i * IN + j] = t;
            }
        }
    }
    __syncthreads();

    // ---- B: thread per 4 columns -- bias / LayerNorm (/ input_proj) partials.
    //      Nodes four at a time: their global rows are loaded before the first
    //      is used (one memory round trip per four nodes, same summation order).
    const int PW = IN > 0 ? 14 * HC : 5 * HC;
    float* part = a.part + (size_t)g * PW;
    for (int q = tid; q < HC / 4; q += kT) {
        float pb[4] = {0, 0, 0, 0}, pw[4] = {0, 0, 0, 0}, pl[4] = {0, 0, 0, 0}, ppb[4] = {0, 0, 0, 0};
        float pwp[4][INR];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < INR; ++j) pwp[r][j] = 0.0f;
        auto node_terms = [&](int i, const float4 t4, const float4 v4) {
            const float4 g4 = *reinterpret_cast<const float4*>(gv + i * GS + 4 * q);
            const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, tt[4] = {t4.x, t4.y, t4.z, t4.w},
                        vv[4] = {v4.x, v4.y, v4.z, v4.w};
            const float mean = st[2 * i], rstd = st[2 * i + 1];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pb[r] += gg[r];
                pw[r] += tt[r] * ((vv[r] - mean) * rstd);
                pl[r] += tt[r];
                if (IN > 0 && a.residual == 2) {
                    ppb[r] += tt[r];
#pragma unroll
                    for (int j = 0; j < INR; ++j) pwp[r][j] += tt[r] * x0l[i * IN + j];
                }
            }
        };
        int i = 0;
        for (; i + 4 <= n; i += 4) {
            float4 t4[4], v4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const size_t row = (size_t)(node0 + i + u) * HC;
                t4[u] = *reinterpret_cast<const float4*>(a.g_res + row + 4 * q);
                v4[u] = *reinterpret_cast<const float4*>(a.v + row + 4 * q);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) node_terms(i + u, t4[u], v4[u]);
        }
        for (; i < n; ++i) {
            const size_t row = (size_t)(node0 + i) * HC;
            node_terms(i, *reinterpret_cast<const float4*>(a.g_res + row + 4 * q),
                       *reinterpret_cast<const float4*>(a.v + row + 4 * q));
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = 4 * q + r;
            part[c] = pb[r];
            part[HC + c] = pw[r];
            part[2 * HC + c] = pl[r];
            if (IN > 0) {
#pragma unroll
                for (int j = 0; j < INR; ++j) part[9 * HC + c * IN + j] = a.residual == 2 ? pwp[r][j] : 0.0f;
                part[13 * HC + c] = a.residual == 2 ? ppb[r] : 0.0f;
            }
        }
    }

    // ---- C1: dL/dalpha[p,h] = <gv[dst_p, h], xh[src_p, h]>, four pairs per wave (16-lane rows)
    {
        const int sub = lane >> 4, sl = lane & 15;
        const int P = ne * H, groups = (P + 3) / 4;
        for (int gi = wave; gi < groups; gi += kNW) {
            const int t = 4 * gi + sub;
            const bool ok = t < P;
            const int p = ok ? t / H : 0, h = ok ? t - (t / H) * H : 0;
            float s = 0.0f;
            if (ok) {
                const float* gr = gv + dl[p] * GS + h * C;
                for (int c = 4 * sl; c < C; c += 64) {
                    const float4 g4 = *reinterpret_cast<const float4*>(gr + c);
                    const float4 x4 = xget4(cl[p], h * C + c);
                    s += (g4.x * x4.x + g4.y * x4.y) + (g4.z * x4.z + g4.w * x4.w);
                }
            }
            s = rsum16(s);
            if (ok && sl == 0) ge[t] = s;
        }
    }
    __syncthreads();

    // ---- C2: softmax + leaky ReLU backward per (node, head); edge-logit gradient
    for (int t = tid; t < n * H; t += kT) {
        const int i = t / H, h = t - (t / H) * H;
        const int p0 = rp[i], p1 = rp[i + 1];
        float s = 0.0f;
        for (int p = p0; p < p1; ++p) s += al[p * H + h] * ge[p * H + h];
        float sd = 0.0f;
        const float ad = asd[i * 2 * H + H + h];
        for (int p = p0; p < p1; ++p) {
            const float gl = al[p * H + h] * (ge[p * H + h] - s);
            const float e = asd[cl[p] * 2 * H + h] + ad +
                            a.a_edge[(size_t)(ebeg + p) * a.a_edge_stride + a.a_edge_offset + h];
            const float gev = e > 0.0f ? gl : gl * a.negative_slope;
            ge[p * H + h] = gev;
            a.g_a_edge[(size_t)(ebeg + p) * a.a_edge_stride + a.a_edge_offset + h] = gev;
            sd += gev;
        }
        gad[t] = sd;
    }
    __syncthreads();
    // ---- C3: dL/da_src[j,h] over j's out-positions (fixed source-CSR order)
    for (int t = tid; t < n * H; t += kT) {
        const int j = t / H, h = t - (t / H) * H;
        float s = 0.0f;
        for (int k = sp[j]; k < sp[j + 1]; ++k) s += ge[spp[k] * H + h];
        gas[t] = s;
    }
    __syncthreads();

    // ---- D: wave per node j -- dL/dxh[j] = sum_{p: src=j} alpha_p gv[dst_p] + attention-dot terms
    for (int j = wave; j < n; j += kNW) {
        float acc[KC][4];
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[k][r] = 0.0f;
        for (int k2 = sp[j]; k2 < sp[j + 1]; ++k2) {
            const int p = spp[k2];
            const float* gr = gv + dl[p] * GS;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const int f0 = 4 * (lane + kW * k);
                const float w = al[p * H + f0 / C];
                const float4 g4 = *reinterpret_cast<const float4*>(gr + f0);
                acc[k][0] += w * g4.x;
                acc[k][1] += w * g4.y;
                acc[k][2] += w * g4.z;
                acc[k][3] += w * g4.w;
            }
        }
        float rx[INR];
#pragma unroll
        for (int jj = 0; jj < INR; ++jj) rx[jj] = 0.0f;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int f0 = 4 * (lane + kW * k), h = f0 / C;
            const float4 s4 = *reinterpret_cast<const float4*>(a.att_src + f0);
            const float4 d4 = *reinterpret_cast<const float4*>(a.att_dst + f0);
            const float gs = gas[j * H + h], gd = gad[j * H + h];
            float o[4];
            o[0] = acc[k][0] + (gs * s4.x + gd * d4.x);
            o[1] = acc[k][1] + (gs * s4.y + gd * d4.y);
            o[2] = acc[k][2] + (gs * s4.z + gd * d4.z);
            o[3] = acc[k][3] + (gs * s4.w + gd * d4.w);
            const float4 ov = st4x<XF>(static_cast<XE*>(a.g_xh) + (size_t)(node0 + j) * HC + f0, o[0], o[1], o[2], o[3]);
            if (IN > 0) {  // dL/dx0 through xh = bf16(x0l @ w0^T): the (bf16) gradient times w0
                const float ob[4] = {ov.x, ov.y, ov.z, ov.w};
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int jj = 0; jj < INR; ++jj)
                        rx[jj] += ob[r] * (XG ? w0s[(f0 + r) * IN + jj] : a.w0[(size_t)(f0 + r) * IN + jj]);
            }
        }
        if (IN > 0) {
#pragma unroll
            for (int jj = 0; jj < INR; ++jj) {
                const float t = wsum(rx[jj]);
                if (lane == 0) a.g_x0[(size_t)(node0 + j) * IN + jj] = gx0[j * IN + jj] + t;
            }
        }
    }
    __syncthreads();

    // ---- E: thread per 4 columns -- att_src / att_dst (/ layer-0 lin.weight) partials
    //      (layer 0: the g_xh rows four nodes at a time, as in B)
    for (int q = tid; q < HC / 4; q += kT) {
        const int h = (4 * q) / C;
        float ps[4] = {0, 0, 0, 0}, pd[4] = {0, 0, 0, 0};
        float pw0[4][INR];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < INR; ++j) pw0[r][j] = 0.0f;
        auto node_terms = [&](int j, const float4 w) {
            const float4 x4 = xget4(j, 4 * q);
            const float xv[4] = {x4.x, x4.y, x4.z, x4.w};
            const float gs = gas[j * H + h], gd = gad[j * H + h];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                ps[r] += gs * xv[r];
                pd[r] += gd * xv[r];
            }
            if (IN > 0) {
                const float gb[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int jj = 0; jj < INR; ++jj) pw0[r][jj] += gb[r] * x0l[j * IN + jj];
            }
        };
        auto gxh = [&](int j) {
            return IN > 0 ? ld4x<XF>(static_cast<const XE*>(a.g_xh) + (size_t)(node0 + j) * HC + 4 * q)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        };
        int j = 0;
        for (; j + 4 <= n; j += 4) {
            float4 w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) w[u] = gxh(j + u);
#pragma unroll
            for (int u = 0; u < 4; ++u) node_terms(j + u, w[u]);
        }
        for (; j < n; ++j) node_terms(j, gxh(j));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = 4 * q + r;
            part[3 * HC + c] = ps[r];
            part[4 * HC + c] = pd[r];
            if (IN > 0) {
#pragma unroll
                for (int jj = 0; jj < INR; ++jj) part[5 * HC + c * IN + jj] = pw0[r][jj];
            }
        }
    }
}

size_t gat_layer_bwd_smem(const trx_gat_layer_bwd_args& a) {
    const size_t HC = (size_t)a.heads * a.channels, n = a.nodes_per_graph, H = a.heads, me = a.max_graph_edges;
    return (a.exact ? (HC > 512 ? (a.in_dim > 0 ? HC * a.in_dim * 4 : 0) : n * (HC + 4) * 4) : n * (HC + 8) * 2) + n * (HC + 4) * 4 + 2 * me * H * 4 + 2 * n * H * 4 + 2 * n * H * 4 + 2 * n * 4 + 8 * n * 4 +
           (a.g_pool ? 2 * HC * 4 : 0) + (2 * me + 2 * (n + 1) + me) * 4;
}

template <int HC, int IN, int NT, bool XF = false>
static void set_bwd_lds_attr() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gat_layer_bwd_kernel<HC, IN, NT, XF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

// One workgroup per graph and ~144 KB of LDS for HC 1024: one workgroup per
// CU, so the waves per workgroup are the occupancy -- 8 (two per SIMD) where
// the registers allow it (HC 1024: up to 218 VGPRs), 16 for the narrower layers.
hipError_t launch_gat_layer_bwd(const trx_gat_layer_bwd_args* al, int count, hipStream_t stream) {
    const trx_gat_layer_bwd_args& a = al[0];
    const NetList<trx_gat_layer_bwd_args> l = net_list(al, count);
    static bool attr_set = false;
    if (!attr_set) {
        set_bwd_lds_attr<1024, 0, 512>();
        set_bwd_lds_attr<1024, 4, 512>();
        set_bwd_lds_attr<512, 0, 1024>();
        set_bwd_lds_attr<512, 4, 1024>();
        set_bwd_lds_attr<256, 0, 1024>();
        set_bwd_lds_attr<256, 4, 1024>();
        set_bwd_lds_attr<1024, 0, 512, true>();
        set_bwd_lds_attr<1024, 4, 512, true>();
        set_bwd_lds_attr<512, 0, 1024, true>();
        set_bwd_lds_attr<512, 4, 1024, true>();
        set_bwd_lds_attr<256, 0, 1024, true>();
        set_bwd_lds_attr<256, 4, 1024, true>();
        attr_set = true;
    }
    const int HC = a.heads * a.channels;
    const size_t smem = gat_layer_bwd_smem(a);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    const dim3 grid(a.num_graphs, count);
#define TRX_BWD_CASE(HCV, INV, NTV, XFV)                                                                 \
    if (HC == HCV && a.in_dim == INV && (a.exact != 0) == XFV) {                                         \
        hipLaunchKernelGGL((gat_layer_bwd_kernel<HCV, INV, NTV, XFV>), grid, dim3(NTV), smem, stream, l); \
        return hipGetLastError();                                                                        \
    }
    TRX_BWD_CASE(1024, 0, 512, false)
    TRX_BWD_CASE(1024, 4, 512, false)
    TRX_BWD_CASE(512, 0, 1024, false)
    TRX_BWD_CASE(512, 4, 1024, false)
    TRX_BWD_CASE(256, 0, 1024, false)
    TRX_BWD_CASE(256, 4, 1024, false)
    TRX_BWD_CASE(1024, 0, 512, true)
    TRX_BWD_CASE(1024, 4, 512, true)
    TRX_BWD_CASE(512, 0, 1024, true)
    TRX_BWD_CASE(512, 4, 1024, true)
    TRX_BWD_CASE(256, 0, 1024, true)
    TRX_BWD_CASE(256, 4, 1024, true)
#undef TRX_BWD_CASE
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------ partial sums
// out[k] = sum_r part[r * stride + k] for r < rows, k < width, r ascending.
// Column sums of a [rows][width] partial block in a fixed order (deterministic):
// 16 waves per 64 columns, wave w sums rows w, w+16, ... (loads four rows
// ahead), then wave 0 adds the 16 wave sums in wave order.
constexpr int kPsWaves = 16;
// out index k -> out + (k / out_cols) * out_ld + k % out_cols (out_cols 0: out + k)
__device__ __forceinline__ void partial_sum_block(const float* __restrict__ part, int rows, int width, int64_t stride,
                                                  float* __restrict__ out, int out_cols, int64_t out_ld) {
    __shared__ float red[kPsWaves][kW];
    const int lane = threadIdx.x & (kW - 1), w = threadIdx.x / kW;
    const int k = blockIdx.x * kW + lane;
    float s = 0.0f;
    if (k < width) {
        int r = w;
        for (; r + 3 * kPsWaves < rows; r += 4 * kPsWaves) {
            const float a0 = part[(size_t)r * stride + k];
            const float a1 = part[(size_t)(r + kPsWaves) * stride + k];
            const float a2 = part[(size_t)(r + 2 * kPsWaves) * stride + k];
            const float a3 = part[(size_t)(r + 3 * kPsWaves) * stride + k];
            s += a0;
            s += a1;
            s += a2;
            s += a3;
        }
        for (; r < rows; r += kPsWaves) s += part[(size_t)r * stride + k];
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && k < width) {
        float t = red[0][lane];
#pragma unroll
        for (int j = 1; j < kPsWaves; ++j) t += red[j][lane];
        out[out_cols > 0 ? (int64_t)(k / out_cols) * out_ld + k % out_cols : (int64_t)k] = t;
    }
}

__global__ void __launch_bounds__(kW * kPsWaves) partial_sum_kernel(const float* __restrict__ part, int rows, int width,
                                                                    int64_t stride, float* __restrict__ out) {
    partial_sum_block(part, rows, width, stride, out, 0, 0);
}

// several column-sum problems in one launch (blockIdx.y = problem): the fused update's
// per-network parameter partials, same summation order as partial_sum_kernel
__global__ void __launch_bounds__(kW * kPsWaves) partial_sum_multi_kernel(trx_psum_list l) {
    const int e = blockIdx.y;
    if (e >= l.count || (int)blockIdx.x * kW >= l.width[e]) return;  // block-uniform
    partial_sum_block(l.part[e], l.rows, l.width[e], l.stride[e], l.out[e], l.out_cols[e], l.out_ld[e]);
}

hipError_t launch_partial_sum(const float* part, int rows, int width, int64_t stride, float* out,
                              hipStream_t stream) {
    hipLaunchKernelGGL(partial_sum_kernel, dim3((width + kW - 1) / kW), dim3(kW * kPsWaves), 0, stream, part, rows,
                       width, stride, out);
    return hipGetLastError();
}

hipError_t launch_partial_sum_multi(const trx_psum_list& l, hipStream_t stream) {
    int mx = 1;
    for (int e = 0; e < l.count; ++e) mx = l.width[e] > mx ? l.width[e] : mx;
    hipLaunchKernelGGL(partial_sum_multi_kernel, dim3((mx + kW - 1) / kW, l.count), dim3(kW * kPsWaves), 0, stream, l);
    return hipGetLastError();
}

// ------------------------------------------- edge-attention weight backward
// Backward of every layer's M rows (edge_att_weights_kernel, gat_infer.hip:
// M[h, j] = sum_c lin_edge.weight[h*C + c, j] * att_edge[h, c]) from gM [A, stride]:
//   g_lin_edge[h*C + c, j] = gM[h, j] * att_edge[h, c]
//   g_att_edge[h, c]       = sum_j lin_edge.weight[h*C + c, j] * gM[h, j]   (j ascending)
// One thread per (layer, h, c); out holds per layer [g_lin_edge (H*C*D) | g_att_edge (H*C)].
__global__ void __launch_bounds__(256) edge_att_weights_bwd_kernel(trx_gat_prologue_args a, const float* __restrict__ gm,
                                                                   int gm_stride, float* __restrict__ out) {
    int t = blockIdx.x * 256 + threadIdx.x;
    const int D = a.edge_dim;
    int l = 0, row0 = 0;
    size_t o = 0;
    while (l < a.num_layers && t >= a.heads[l] * a.channels[l]) {
        const int hc = a.heads[l] * a.channels[l];
        t -= hc;
        o += (size_t)hc * (D + 1);
        row0 += a.heads[l];
        ++l;
    }
    if (l >= a.num_layers) return;
    const int C = a.channels[l], HC = a.heads[l] * C;
    const int h = t / C;
    const float att = a.att_edge[l][t];
    const float* w = a.lin_edge_w[l] + (size_t)t * D;
    const float* g = gm + (size_t)(row0 + h) * gm_stride;
    float s = 0.0f;
    for (int j = 0; j < D; ++j) {
        out[o + (size_t)t * D + j] = g[j] * att;
        s += w[j] * g[j];
    }
    out[o + (size_t)HC * D + t] = s;
}

hipError_t launch_edge_att_weights_bwd(const trx_gat_prologue_args& a, const float* gm, int gm_stride, float* out,
                                       hipStream_t stream) {
    int n = 0;
    for (int l = 0; l < a.num_layers; ++l) n += a.heads[l] * a.channels[l];
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(edge_att_weights_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a, gm, gm_stride, out);
    return hipGetLastError();
}

// --------------------------------------------------------- prologue backward
// One 4-wave workgroup per graph.  Forward (gat_infer.hip gat_prologue_kernel): ea = LN(edge_x),
// x0 = LN(node_x), loop[i] = mean of ea over i's kept in-links, a_edge[p, k] =
// bf16(bf16(full[p]) . Ml[k]) with Ml = bf16(M).  Per-graph partials (floats,
// width 8A + 32): [0, 8A) dL/dMl (rows of 8), then edge LN weight / bias,
// node LN weight / bias (8 each).
constexpr int kPD = 8;
constexpr int kPLS = 9;  // LDS row stride of the per-link / per-node rows

__device__ __forceinline__ void ln_fwd_row(float (&x)[kPD], int d, const float* w, const float* b, float eps,
                                           float (&xhat)[kPD]) {
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < kPD; ++j)
        if (j < d) s += x[j];
    const float mu = s / (float)d;
    float v = 0.0f;
#pragma unroll
    for (int j = 0; j < kPD; ++j)
        if (j < d) {
            const float t = x[j] - mu;
            v += t * t;
        }
    const float r = rsqrtf(v / (float)d + eps);
#pragma unroll
    for (int j = 0; j < kPD; ++j) {
        xhat[j] = j < d ? (x[j] - mu) * r : 0.0f;
        x[j] = j < d ? (x[j] - mu) * r * w[j] + b[j] : 0.0f;
    }
}

constexpr int kPBT = 256;  // prologue backward: threads per graph

__global__ void __launch_bounds__(kPBT) gat_prologue_bwd_kernel(const NetList<trx_gat_prologue_bwd_args> nets) {
    const trx_gat_prologue_bwd_args& a = nets.a[blockIdx.y];
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int MD = kPD, NW = kPBT / kW;
    const int g = blockIdx.x, tid = threadIdx.x, lane = tid & (kW - 1), wave = tid / kW;
    const int n = a.nodes_per_graph, E = a.edges_per_graph, ND = a.node_dim, D = a.edge_dim, A = a.A;
    constexpr int LS = kPLS;                      // odd LDS row stride: a wave's rows on distinct banks
    float* ean = reinterpret_cast<float*>(smem);  // [E][LS] normalised link features
    float* exh = ean + E * LS;                    // [E][LS] their xhat
    float* gea = exh + E * LS;                    // [E][LS] dL/dea
    float* lp = gea + E * LS;                     // [n][LS] loop attrs
    float* glp = lp + n * LS;                     // [n][LS] dL/dloop
    float* Ml = glp + n * LS;                     // [A][8] (broadcast reads)
    float* dg = Ml + A * MD;                      // [n] kept in-degree
    int* ld = reinterpret_cast<int*>(dg + n);     // [E] local dst of kept links, else -1
    const int64_t node0 = (int64_t)g * n, link0 = (int64_t)g * E;
    const int p0 = a.rowptr[node0], p1 = a.rowptr[node0 + n];
    float* part = a.part + (size_t)g * (8 * A + 32);
    for (int v = tid; v < A * MD; v += kPBT) {
        const int k = v / MD, j = v - (v / MD) * MD;
        Ml[v] = j < D ? (a.exact ? a.m_work[k * D + j] : rbf(a.m_work[k * D + j])) : 0.0f;
    }
    for (int l = tid; l < E; l += kPBT) {
        float x[MD], xh[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) x[j] = j < D ? a.edge_x[(link0 + l) * D + j] : 0.0f;
        ln_fwd_row(x, D, a.edge_ln_w, a.edge_ln_b, a.edge_ln_eps, xh);
        const int64_t s = a.src[link0 + l] - node0, d = a.dst[link0 + l] - node0;
#pragma unroll
        for (int j = 0; j < MD; ++j) {
            ean[l * LS + j] = x[j];
            exh[l * LS + j] = xh[j];
            gea[l * LS + j] = (a.g_ea_head && j < D) ? a.g_ea_head[(link0 + l) * D + j] : 0.0f;
        }
        ld[l] = (s == d || d < 0 || d >= n) ? -1 : (int)d;
    }
    __syncthreads();
    // loop attrs, the forward's order: a node's CSR row lists its kept in-links in link order
    for (int i = tid; i < n; i += kPBT) {
        float s[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) s[j] = 0.0f;
        int cnt = 0;
        for (int p = a.rowptr[node0 + i]; p < a.rowptr[node0 + i + 1]; ++p) {
            const int code = a.pos_src[p];
            const int64_t li = (int64_t)code - link0;
            if (code < 0 || li < 0 || li >= E) continue;
            ++cnt;
#pragma unroll
            for (int j = 0; j < MD; ++j) s[j] += ean[li * LS + j];
        }
        const float deg = cnt > 0 ? (float)cnt : 1.0f;
        dg[i] = deg;
#pragma unroll
        for (int j = 0; j < MD; ++j) {
            lp[i * LS + j] = j < D ? s[j] / deg : 0.0f;
            glp[i * LS + j] = 0.0f;
        }
    }
    __syncthreads();
    // positions: dL/dfull into the link / loop rows (each position is its link's or
    // node's only one)
    for (int p = p0 + tid; p < p1; p += kPBT) {
        const int code = a.pos_src[p];
        const int64_t li = (int64_t)code - link0, ni = -(int64_t)code - 1 - node0;
        float gf[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) gf[j] = 0.0f;
        for (int k = 0; k < A; ++k) {
            const float gk = a.g_a_edge[(size_t)p * A + k];
#pragma unroll
            for (int j = 0; j < MD; ++j) gf[j] += gk * Ml[k * MD + j];
        }
        float* dstg = code >= 0 ? gea + li * LS : glp + ni * LS;
#pragma unroll
        for (int j = 0; j < MD; ++j) dstg[j] += gf[j];
    }
    // dL/dMl row by row, rows dealt to the waves (lane partials over positions + wave sums)
    for (int k = wave; k < A; k += NW) {
        float gm[MD];
#pragma unroll
        for (int j = 0; j < MD; ++j) gm[j] = 0.0f;
        for (int p = p0 + lane; p < p1; p += kW) {
            const int code = a.pos_src[p];
            const float* fr = code >= 0 ? ean + ((int64_t)code - link0) * LS : lp + (-(int64_t)code - 1 - node0) * LS;
            const float gk = a.g_a_edge[(size_t)p * A + k];
#pragma unroll
            for (int j = 0; j < MD; ++j) gm[j] += gk * (j < D ? (a.exact ? fr[j] : rbf(fr[j])) : 0.0f);
        }
#pragma unroll
        for (int j = 0; j < MD; ++j) {
            const float t = wsum(gm[j]);
            if (lane == 0) part[k * MD + j] = t;
        }
    }
    __syncthreads();
    float pw[MD], pb[MD];
#pragma unroll
    for (int j = 0; j < MD; ++j) pw[j] = pb[j] = 0.0f;
    if (wave == 0) {  // loop-mean backward into the kept links, then edge LayerNorm weight / bias
        for (int l = lane; l < E; l += kW) {
            const int d = ld[l];
#pragma unroll
            for (int j = 0; j < MD; ++j) {
                float gj = gea[l * LS + j];
                if (d >= 0) gj += glp[d * LS + j] / dg[d];
                pw[j] += gj * exh[l * LS + j];
                pb[j] += gj;
            }
        }
#pragma unroll
        for (int j = 0; j < MD; ++j) {
            const float w = wsum(pw[j]), b = wsum(pb[j]);
            if (lane == 0) {
                part[8 * A + j] = w;
                part[8 * A + 8 + j] = b;
            }
        }
    } else if (wave == 1) {  // node LayerNorm weight / bias from dL/dx0
        for (int i = lane; i < n; i += kW) {
            float x[MD], xh[MD];
#pragma unroll
            for (int j = 0; j < MD; ++j) x[j] = j < ND ? a.node_x[(node0 + i) * ND + j] : 0.0f;
            ln_fwd_row(x, ND, a.node_ln_w, a.node_ln_b, a.node_ln_eps, xh);
#pragma unroll
            for (int j = 0; j < MD; ++j)
                if (j < ND) {
                    const float gj = a.g_x0[(node0 + i) * ND + j];
                    pw[j] += gj * xh[j];
                    pb[j] += gj;
                }
        }
#pragma unroll
        for (int j = 0; j < MD; ++j) {
            const float w = wsum(pw[j]), b = wsum(pb[j]);
            if (lane == 0) {
                part[8 * A + 16 + j] = w;
                part[8 * A + 24 + j] = b;
            }
        }
    }
}

size_t gat_prologue_bwd_smem(const trx_gat_prologue_bwd_args& a) {
    return ((size_t)a.edges_per_graph * kPLS * 3 + (size_t)a.nodes_per_graph * kPLS * 2 + (size_t)a.A * kPD +
            a.nodes_per_graph + a.edges_per_graph) * 4;
}

hipError_t launch_gat_prologue_bwd(const trx_gat_prologue_bwd_args* a, int count, hipStream_t stream) {
    hipLaunchKernelGGL(gat_prologue_bwd_kernel, dim3(a[0].num_graphs, count), dim3(kPBT), gat_prologue_bwd_smem(a[0]),
                       stream, net_list(a, count));
    return hipGetLastError();
}

// ------------------------------------------------------------------ SAC loss
// One workgroup (256 threads) per graph b, edges e < E (E <= 256: one thread each).
// Per-graph partials (part[b*8 + k]): critic loss term, actor loss term, sum p log p,
// sum p, log(valid + 1e-8), q_taken, sum q_all, sum p log p (logp metric) -- the
// finish kernel forms the means, the alpha loss and dL/dlog_alpha.
constexpr int kLossParts = 8;

__global__ void __launch_bounds__(kT) sac_loss_kernel(trx_sac_loss_args a) {
    __shared__ float red[kT / kW][4];
    const int b = blockIdx.x, e = threadIdx.x, lane = e & (kW - 1), wave = e / kW;
    const int E = a.edges_per_graph, B = a.num_graphs;
    const bool on = e < E;
    const size_t ix = (size_t)b * E + e;
    const float alpha = expf(*a.log_alpha);
    // soft state value of the next state and the TD target (sac.py:184-191)
    float vn = 0.0f;
    if (on) {
        const float np = a.next_probs[ix];
        const float qn = fminf(a.qt1[ix], a.qt2[ix]);
        vn = np * (qn - alpha * logf(np + 1e-8f));
    }
    // actor softmax over the masked logits (sac.py:45-46 + 207-210)
    const float lg = on ? (a.mask[ix] <= 0.0f ? -1e9f : a.logits[ix]) : -__builtin_huge_valf();
    float mx = lg;
    {
        float m = mx;
        for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        if (lane == 0) red[wave][0] = m;
        __syncthreads();
        mx = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]));
        __syncthreads();
    }
    const float ex = on ? expf(lg - mx) : 0.0f;
    float vsum, exsum, validc;
    {
        float t0 = wsum(vn), t1 = wsum(ex), t2 = wsum(on && a.mask[ix] > 0.0f ? 1.0f : 0.0f);
        if (lane == 0) {
            red[wave][0] = t0;
            red[wave][1] = t1;
            red[wave][2] = t2;
        }
        __syncthreads();
        vsum = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
        exsum = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
        validc = (red[0][2] + red[1][2]) + (red[2][2] + red[3][2]);
        __syncthreads();
    }
    const float target = a.reward[b] + (1.0f - a.done[b]) * a.gamma * vsum;
    const float p = ex / (exsum + 1e-16f);
    const float lp = logf(p + 1e-8f);
    const float q1a = on ? a.q1[ix] : 0.0f, q2a = on ? a.q2[ix] : 0.0f;
    const float qall = fminf(q1a, q2a);
    // actor: L_b = sum_e p (alpha lp - q); dL/dp = alpha lp - q + alpha p / (p + 1e-8)
    const float term = on ? p * (alpha * lp - qall) : 0.0f;
    const float dLdp = on ? (alpha * lp - qall + alpha * p / (p + 1e-8f)) / (float)B : 0.0f;
    float sterm, spd, splp, sp, sq;
    {
        float t0 = wsum(term), t1 = wsum(p * dLdp), t2 = wsum(on ? p * lp : 0.0f), t3 = wsum(on ? qall : 0.0f);
        float t4 = wsum(on ? p : 0.0f);
        if (lane == 0) {
            red[wave][0] = t0;
            red[wave][1] = t1;
            red[wave][2] = t2;
            red[wave][3] = t3;
        }
        __syncthreads();
        sterm = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
        spd = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
        splp = (red[0][2] + red[1][2]) + (red[2][2] + red[3][2]);
        sq = (red[0][3] + red[1][3]) + (red[2][3] + red[3][3]);
        __syncthreads();
        if (lane == 0) red[wave][0] = t4;
        __syncthreads();
        sp = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
    }
    if (on) {
        // masked_fill blocks the gradient of masked logits
        a.g_logits[ix] = a.mask[ix] <= 0.0f ? 0.0f : p * (dLdp - spd);
        const bool act = e == a.action[b];
        const float w = a.weights[b];
        a.g_q1[ix] = act ? w * 2.0f * (q1a - target) / (float)B : 0.0f;
        a.g_q2[ix] = act ? w * 2.0f * (q2a - target) / (float)B : 0.0f;
        if (act) {
            a.td_error[b] = fabsf(target - q1a);
            float* pt = a.part + (size_t)b * kLossParts;
            const float d1 = q1a - target, d2 = q2a - target;
            pt[0] = w * (d1 * d1 + d2 * d2);
            pt[1] = sterm;
            pt[2] = splp;
            pt[3] = sp;
            pt[4] = logf(validc + 1e-8f);
            pt[5] = fminf(q1a, q2a);
            pt[6] = sq;
            pt[7] = 0.0f;
        }
    }
}

// One workgroup: the batch means (fixed order), target entropy, alpha loss and
// dL/dlog_alpha.  out: [0] critic_loss, [1] actor_loss, [2] alpha_loss,
// [3] entropy, [4] q_taken, [5] q_mean, [6] logp_mean, [7] alpha; g_log_alpha[0].
__global__ void __launch_bounds__(kW) sac_loss_finish_kernel(trx_sac_loss_args a) {
    const int lane = threadIdx.x, B = a.num_graphs;
    float s[kLossParts];
#pragma unroll
    for (int k = 0; k < kLossParts; ++k) s[k] = 0.0f;
    for (int b = lane; b < B; b += kW)
#pragma unroll
        for (int k = 0; k < kLossParts; ++k) s[k] += a.part[(size_t)b * kLossParts + k];
#pragma unroll
    for (int k = 0; k < kLossParts; ++k) s[k] = wsum(s[k]);
    const float te = a.target_entropy_given ? a.target_entropy : a.target_entropy_ratio * (s[4] / (float)B);
    float at = 0.0f;  // mean_b sum_e p (log p + te) = (sum p log p + te sum p) / B
    for (int b = lane; b < B; b += kW) {
        const float* pt = a.part + (size_t)b * kLossParts;
        at += pt[2] + te * pt[3];
    }
    at = wsum(at) / (float)B;
    if (lane == 0) {
        const float la = *a.log_alpha;
        a.out[0] = s[0] / (float)B;
        a.out[1] = s[1] / (float)B;
        a.out[2] = -(la * at);
        a.out[3] = -s[2] / (float)B;
        a.out[4] = s[5] / (float)B;
        a.out[5] = s[6] / ((float)B * (float)a.edges_per_graph);
        a.out[6] = s[2] / (float)B;
        a.out[7] = expf(la);
        a.g_log_alpha[0] = -at;
    }
}

hipError_t launch_sac_loss(const trx_sac_loss_args& a, hipStream_t stream) {
    hipLaunchKernelGGL(sac_loss_kernel, dim3(a.num_graphs), dim3(kT), 0, stream, a);
    hipLaunchKernelGGL(sac_loss_finish_kernel, dim3(1), dim3(kW), 0, stream, a);
    return hipGetLastError();
}

}  // namespace trx

// gat_layer0.hip -- the GAT encoder's first layer for inference, in its linear
// form (gfx950).
//
// Layer 0 of GATEncoder (src/models/gat_encoder.py:36-47: GATConv(4 -> H*C)
// + LayerNorm + relu(x + input_proj(x_in))) sees 4 raw features per node.
// Its projection xh[j] = W0 x[j] is linear in those 4 numbers, so
//   * the attention logits are 4-dots: <xh[j]_h, att_h> = x[j] . (W0_h^T att_h);
//   * the aggregate is W0_h (sum_j alpha_jh x[j]): a 4-vector per (node, head)
//     ("xbar") instead of C channels;
//   * the LayerNorm statistics over the H*C outputs v = W0 xbar + b are a linear
//     and a quadratic form of xbar per head (sum_c W0[c], sum_c b_c W0[c],
//     sum_c W0[c] W0[c]^T), evaluated in float64;
// so a graph's whole layer needs ~30 numbers per node before its output rows
// are written.  The kernel is then a streaming writer: one workgroup per
// graph, thread t owns output channels 4t..4t+3 (its weights, bias, norm and
// input-projection constants in registers), and every node's row is written
// as float32 (the next layer's residual) and bf16 (the next layer's GEMM
// input) with 16- and 8-byte stores.  fp32 arithmetic throughout (the
// reference's precision): no bf16 rounding of x, W0 or the projection.
//
// The per-head constants come from trx_gat_layer0_prepare (one small launch
// whenever the weights change).  Training keeps gat_layer_infer_kernel with
// its saved intermediates (gat_train.hip's backward reads them).
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

__device__ __forceinline__ float leaky0(float x, float slope) { return x > 0.0f ? x : x * slope; }

typedef float l0_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 l0_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16_l0(float lo, float hi) {
    const l0_f2 v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, l0_b2));
}

// wave-wide sum on DPP + readlane: quad butterflies, row mirrors, then the four
// 16-lane row totals (every lane gets the total)
#define L0_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, false))
__device__ __forceinline__ float wave_sum_l0(float v) {
    v = v + L0_DPP(v, 0xB1);
    v = v + L0_DPP(v, 0x4E);
    v = v + L0_DPP(v, 0x141);
    v = v + L0_DPP(v, 0x140);
    return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
           (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}
#undef L0_DPP

// 4-term dot product in a fixed order (no contraction: -ffp-contract=off)
__device__ __forceinline__ float dot4(const float (&x)[4], float a0, float a1, float a2, float a3) {
    return (x[0] * a0 + x[1] * a1) + (x[2] * a2 + x[3] * a3);
}

template <int HC>
__global__ void __launch_bounds__(HC / 4) gat_layer0_lin_kernel(trx_gat_layer0_args a) {
    constexpr int NT = HC / 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int g = blockIdx.x, tid = threadIdx.x;
    const int n = a.nodes_per_graph, H = a.heads, C = HC / a.heads;
    const int node0 = g * n;
    const int ebeg = a.rowptr[node0];
    const int ne = a.rowptr[node0 + n] - ebeg;
    const int me = a.max_graph_edges;

    // this thread's channels f0..f0+3 (one head: C % 4 == 0): constants in registers,
    // their loads issued before the graph's staging
    const int f0 = 4 * tid;
    const int hh = f0 / C;
    float w[4][4], wp[4][4], bias[4], lnw[4], lnb[4], bp[4];
    {
        const float4* w4 = reinterpret_cast<const float4*>(a.w0 + (size_t)f0 * 4);
        const float4* p4 = reinterpret_cast<const float4*>(a.wp + (size_t)f0 * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 x = w4[r], y = p4[r];
            w[r][0] = x.x;
            w[r][1] = x.y;
            w[r][2] = x.z;
            w[r][3] = x.w;
            wp[r][0] = y.x;
            wp[r][1] = y.y;
            wp[r][2] = y.z;
            wp[r][3] = y.w;
        }
        const float4 b4 = *reinterpret_cast<const float4*>(a.bias + f0);
        const float4 g4 = *reinterpret_cast<const float4*>(a.ln_weight + f0);
        const float4 l4 = *reinterpret_cast<const float4*>(a.ln_bias + f0);
        const float4 q4 = *reinterpret_cast<const float4*>(a.bp + f0);
        bias[0] = b4.x, bias[1] = b4.y, bias[2] = b4.z, bias[3] = b4.w;
        lnw[0] = g4.x, lnw[1] = g4.y, lnw[2] = g4.z, lnw[3] = g4.w;
        lnb[0] = l4.x, lnb[1] = l4.y, lnb[2] = l4.z, lnb[3] = l4.w;
        bp[0] = q4.x, bp[1] = q4.y, bp[2] = q4.z, bp[3] = q4.w;
    }

    if (ne > me || ne < 0) {  // LDS was sized for max_graph_edges: poison, do not overrun
        for (int i = 0; i < n; ++i) {
            const size_t o = (size_t)(node0 + i) * HC + f0;
            if (a.out_f32)
                *reinterpret_cast<float4*>(a.out_f32 + o) =
                    make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
            if (a.out_bf16) *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.out_bf16) + o) = make_uint2(0x7fc07fc0u, 0x7fc07fc0u);
        }
        return;
    }

    float* xb = reinterpret_cast<float*>(smem);  // [n][H][4] aggregated raw features (16-B rows)
    float* xs = xb + n * H * 4;                  // [n][4] raw features (16-B rows)
    float* as_ = xs + n * 4;                     // [n*H] a_src
    float* ad_ = as_ + n * H;                    // [n*H] a_dst, then softmax denominators
    float* st = ad_ + n * H;                     // [n][2] LayerNorm mean, rstd
    float* al = st + 2 * n;                      // [me*H] edge logits -> attention weights
    int* cl = reinterpret_cast<int*>(al + me * H);  // [me] graph-local source per CSR position
    int* dlc = cl + me;                          // [me] graph-local destination
    int* rp = dlc + me;                          // [n+1] graph-local row pointers

    // stage the graph: row pointers, sources, this layer's edge logits, raw features
    if (tid <= n) rp[tid] = a.rowptr[node0 + tid] - ebeg;
    for (int p = tid; p < ne; p += NT) cl[p] = a.col[ebeg + p] - node0;
    for (int v = tid; v < ne * H; v += NT) {
        const int p = v / H, h = v - p * H;
        al[v] = a.a_edge[(size_t)(ebeg + p) * a.a_edge_stride + a.a_edge_offset + h];
    }
    for (int v = tid; v < n * 4; v += NT) xs[v] = a.x0[(size_t)node0 * 4 + v];
    __syncthreads();
    for (int i = tid; i < n; i += NT)
        for (int p = rp[i]; p < rp[i + 1]; ++p) dlc[p] = i;
    // a_src / a_dst = x . u (u = W0_h^T att_h, from the prepare kernel)
    for (int t = tid; t < n * H; t += NT) {
        const int i = t / H, h = t - i * H;
        const float x[4] = {xs[4 * i], xs[4 * i + 1], xs[4 * i + 2], xs[4 * i + 3]};
        const float* us = a.u + 4 * h;
        const float* ud = a.u + 4 * (H + h);
        as_[t] = dot4(x, us[0], us[1], us[2], us[3]);
        ad_[t] = dot4(x, ud[0], ud[1], ud[2], ud[3]);
    }
    __syncthreads();
    // edge softmax over each node's in-edges (gat_layer_infer_kernel's arithmetic)
    for (int v = tid; v < ne * H; v += NT) {
        const int p = v / H, h = v - p * H;
        al[v] = leaky0(as_[cl[p] * H + h] + ad_[dlc[p] * H + h] + al[v], a.negative_slope);
    }
    __syncthreads();
    for (int t = tid; t < n * H; t += NT) {
        const int i = t / H, h = t - i * H;
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
    // xbar[i][h] = sum_p alpha[p,h] x[src p]  (CSR order), one thread per (node, head, feature)
    for (int t = tid; t < n * H * 4; t += NT) {
        const int k = t & 3, ih = t >> 2, i = ih / H, h = ih - i * H;
        const float den = ad_[ih];
        float s = 0.0f;
        for (int p = rp[i]; p < rp[i + 1]; ++p) s += (al[p * H + h] / den) * xs[4 * cl[p] + k];
        xb[t] = s;
    }
    __syncthreads();
    // LayerNorm statistics of v = W0 xbar + b over the HC channels, float64 forms
    for (int i = tid; i < n; i += NT) {
        double sv = a.stats[H * 24], sq = a.stats[H * 24 + 1];  // sum b, sum b^2
        for (int h = 0; h < H; ++h) {
            const double* k = a.stats + 24 * h;
            double x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x[q] = (double)xb[(i * H + h) * 4 + q];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                sv += k[q] * x[q];
                sq += 2.0 * k[4 + q] * x[q];
                double row = 0.0;
#pragma unroll
                for (int r = 0; r < 4; ++r) row += k[8 + 4 * q + r] * x[r];
                sq += x[q] * row;
            }
        }
        const double mean = sv / (double)HC;
        double var = sq / (double)HC - mean * mean;
        var = var > 0.0 ? var : 0.0;
        st[2 * i] = (float)mean;
        st[2 * i + 1] = (float)(1.0 / sqrt(var + (double)a.ln_eps));
    }
    __syncthreads();
    if (a.desc) {  // per-node descriptor: xbar [H][4], x [4], mean, rstd (trx_gat_mid_infer regenerates the row)
        const int DS = 4 * H + 8;
        for (int v = tid; v < n * DS; v += NT) {
            const int i = v / DS, q = v - i * DS;
            float val = 0.0f;
            if (q < 4 * H)
                val = xb[i * H * 4 + q];
            else if (q < 4 * H + 4)
                val = xs[4 * i + q - 4 * H];
            else if (q < 4 * H + 6)
                val = st[2 * i + q - 4 * H - 4];
            a.desc[(size_t)(node0 + i) * DS + q] = val;
        }
    }

    // output rows: v = W0 xbar + b, y = relu(LN(v) + (Wp x + bp)), float32 + bf16
    for (int i = 0; i < n; ++i) {
        const float4 xbv = *reinterpret_cast<const float4*>(xb + (i * H + hh) * 4);
        const float4 xv = *reinterpret_cast<const float4*>(xs + 4 * i);
        const float xbr[4] = {xbv.x, xbv.y, xbv.z, xbv.w};
        const float xr[4] = {xv.x, xv.y, xv.z, xv.w};
        const float mean = st[2 * i], rstd = st[2 * i + 1];
        float y[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float v = dot4(xbr, w[r][0], w[r][1], w[r][2], w[r][3]) + bias[r];
            const float res = dot4(xr, wp[r][0], wp[r][1], wp[r][2], wp[r][3]) + bp[r];
            const float yy = (lnw[r] * (rstd * (v - mean)) + lnb[r]) + res;
            y[r] = yy > 0.0f ? yy : 0.0f;
        }
        const size_t o = (size_t)(node0 + i) * HC + f0;
        // the float32 rows (the next layer's residual, 4 KB per node) stream past the
        // caches as non-temporal stores, so the bf16 rows the lin GEMM reads next stay
        // cached: this kernel 131 -> 104 us, the GEMM 175 -> 159 us per 4096-graph act
        typedef float trx_f4v __attribute__((ext_vector_type(4)));
        if (a.out_f32)
            __builtin_nontemporal_store((trx_f4v){y[0], y[1], y[2], y[3]}, reinterpret_cast<trx_f4v*>(a.out_f32 + o));
        if (a.out_bf16)
            *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.out_bf16) + o) =
                make_uint2(pk_bf16_l0(y[0], y[1]), pk_bf16_l0(y[2], y[3]));
    }
}

// ------------------------------------------------------------------ layer 1
// The middle GAT layer (gat_encoder.py:41-47 for 0 < i < L-1, residual x_in =
// layer 0's output) with the residual regenerated from layer 0's per-node
// descriptor (xbar, x, mean, rstd) and layer 0's parameters, with the very
// expression trx_gat_layer0_infer evaluates (bit-identical rows), instead of
// reading a float32 [N, H*C] residual from HBM.  Layout: thread t owns
// channels 4t..4t+3 of every row (channels == 256: wave w = head w), the
// graph's xh rows (bf16) staged in LDS; attention dots are wave sums; the
// LayerNorm moments of NB nodes at a time are combined across the waves
// through LDS (two barriers per batch).  Output bf16 (the last layer's GEMM
// input) and optionally float32.
template <int HC, int NB>
__global__ void __launch_bounds__(HC / 4) gat_mid_gen_kernel(trx_gat_mid_args a) {
    constexpr int NT = HC / 4, NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = a.nodes_per_graph, H = a.heads;  // H == NW (channels 256)
    const int H0 = a.l0_heads, C0 = HC / H0, DS = 4 * H0 + 8;
    const int node0 = g * n;
    const int ebeg = a.rowptr[node0];
    const int ne = a.rowptr[node0 + n] - ebeg;
    const int me = a.max_graph_edges;
    const int f0 = 4 * tid, h0 = f0 / C0;

    // xh rows of the graph (n * HC bf16, contiguous in HBM and in LDS): LDS-DMA,
    // 1 KB per wave instruction, no VGPRs; all in flight before the constants load
    const int nq = n * HC / 8;
    {
        const uint4* xsrc = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.xh) + (size_t)node0 * HC);
        for (int base = wave * 64; base < nq; base += NT) {
            const int v = base + lane;
            if (v < nq)
                __builtin_amdgcn_global_load_lds(xsrc + v, (__attribute__((address_space(3))) void*)(smem + (size_t)base * 16),
                                                 16, 0, 0);
        }
    }
    // constants of this thread's four channels: layer 1 (attention, bias, norm) and layer 0
    float as_r[4], ad_r[4], b1[4], g1[4], e1[4], w0[4][4], wp[4][4], b0[4], g0[4], e0[4], bp[4];
    {
        const float4 x = *reinterpret_cast<const float4*>(a.att_src + f0), y = *reinterpret_cast<const float4*>(a.att_dst + f0);
        const float4 p = *reinterpret_cast<const float4*>(a.bias + f0), q = *reinterpret_cast<const float4*>(a.ln_weight + f0);
        const float4 r = *reinterpret_cast<const float4*>(a.ln_bias + f0);
        as_r[0] = x.x, as_r[1] = x.y, as_r[2] = x.z, as_r[3] = x.w;
        ad_r[0] = y.x, ad_r[1] = y.y, ad_r[2] = y.z, ad_r[3] = y.w;
        b1[0] = p.x, b1[1] = p.y, b1[2] = p.z, b1[3] = p.w;
        g1[0] = q.x, g1[1] = q.y, g1[2] = q.z, g1[3] = q.w;
        e1[0] = r.x, e1[1] = r.y, e1[2] = r.z, e1[3] = r.w;
        const float4* w4 = reinterpret_cast<const float4*>(a.l0_w0 + (size_t)f0 * 4);
        const float4* p4 = reinterpret_cast<const float4*>(a.l0_wp + (size_t)f0 * 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 u = w4[k], v = p4[k];
            w0[k][0] = u.x, w0[k][1] = u.y, w0[k][2] = u.z, w0[k][3] = u.w;
            wp[k][0] = v.x, wp[k][1] = v.y, wp[k][2] = v.z, wp[k][3] = v.w;
        }
        const float4 c = *reinterpret_cast<const float4*>(a.l0_bias + f0), d = *reinterpret_cast<const float4*>(a.l0_ln_weight + f0);
        const float4 e = *reinterpret_cast<const float4*>(a.l0_ln_bias + f0), f = *reinterpret_cast<const float4*>(a.l0_bp + f0);
        b0[0] = c.x, b0[1] = c.y, b0[2] = c.z, b0[3] = c.w;
        g0[0] = d.x, g0[1] = d.y, g0[2] = d.z, g0[3] = d.w;
        e0[0] = e.x, e0[1] = e.y, e0[2] = e.z, e0[3] = e.w;
        bp[0] = f.x, bp[1] = f.y, bp[2] = f.z, bp[3] = f.w;
    }
    if (ne > me || ne < 0) {  // LDS was sized for max_graph_edges: poison, do not overrun
        for (int i = 0; i < n; ++i) {
            const size_t o = (size_t)(node0 + i) * HC + f0;
            if (a.out_f32)
                *reinterpret_cast<float4*>(a.out_f32 + o) =
                    make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
            if (a.out_bf16) *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.out_bf16) + o) = make_uint2(0x7fc07fc0u, 0x7fc07fc0u);
        }
        return;
    }
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem);                 // [n][HC] bf16
    float* dsc = reinterpret_cast<float*>(xs + (size_t)n * HC);       // [n][DS] layer-0 descriptors
    float* as_ = dsc + n * DS;                                        // [n*H]
    float* ad_ = as_ + n * H;                                         // [n*H] then softmax denominators
    float* red = ad_ + n * H;                                         // [2][NW][NB] LayerNorm partials
    float* al = red + 2 * NW * NB;                                    // [me*H]
    int* cl = reinterpret_cast<int*>(al + me * H);                    // [me]
    int* dlc = cl + me;                                               // [me]
    int* rp = dlc + me;                                               // [n+1]
    if (tid <= n) rp[tid] = a.rowptr[node0 + tid] - ebeg;
    for (int p = tid; p < ne; p += NT) cl[p] = a.col[ebeg + p] - node0;
    for (int v = tid; v < ne * H; v += NT) {
        const int p = v / H, h = v - p * H;
        al[v] = a.a_edge[(size_t)(ebeg + p) * a.a_edge_stride + a.a_edge_offset + h];
    }
    for (int v = tid; v < n * DS; v += NT) dsc[v] = a.desc[(size_t)node0 * DS + v];
    __syncthreads();   // (waits for the LDS-DMA: vmcnt(0) before the barrier)
    for (int i = tid; i < n; i += NT)
        for (int p = rp[i]; p < rp[i + 1]; ++p) dlc[p] = i;
    // attention dots: wave w = head w, each node's 256-channel dot as a wave sum
    for (int i = 0; i < n; ++i) {
        const uint2 u = *reinterpret_cast<const uint2*>(xs + (size_t)i * HC + f0);
        const float x0v = __uint_as_float(u.x << 16), x1v = __uint_as_float(u.x & 0xffff0000u);
        const float x2v = __uint_as_float(u.y << 16), x3v = __uint_as_float(u.y & 0xffff0000u);
        float s1 = (x0v * as_r[0] + x1v * as_r[1]) + (x2v * as_r[2] + x3v * as_r[3]);
        float s2 = (x0v * ad_r[0] + x1v * ad_r[1]) + (x2v * ad_r[2] + x3v * ad_r[3]);
        s1 = wave_sum_l0(s1);
        s2 = wave_sum_l0(s2);
        if (lane == 0) {
            as_[i * H + wave] = s1;
            ad_[i * H + wave] = s2;
        }
    }
    __syncthreads();
    for (int v = tid; v < ne * H; v += NT) {
        const int p = v / H, h = v - p * H;
        al[v] = leaky0(as_[cl[p] * H + h] + ad_[dlc[p] * H + h] + al[v], a.negative_slope);
    }
    __syncthreads();
    for (int t = tid; t < n * H; t += NT) {
        const int i = t / H, h = t - i * H;
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
    for (int v = tid; v < ne * H; v += NT) {
        const int p = v / H, h = v - p * H;
        al[v] = al[v] / ad_[dlc[p] * H + h];
    }
    __syncthreads();
    // aggregation + bias + LayerNorm + regenerated residual + ReLU, NB nodes per round.
    // The four channels as two float pairs (written for v_pk_mul_f32 / v_pk_add_f32; the
    // library is built with -packed-fp32-ops, so each pair compiles to two scalar ops:
    // the same IEEE operations, and the regenerated residual keeps layer 0's values)
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 w0p[4][2], wpp[4][2], b0p[2], g0p[2], e0p[2], bpp[2], b1p[2], g1p[2], e1p[2];
#pragma unroll
    for (int P = 0; P < 2; ++P) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            w0p[k][P] = f2{w0[2 * P][k], w0[2 * P + 1][k]};
            wpp[k][P] = f2{wp[2 * P][k], wp[2 * P + 1][k]};
        }
        b0p[P] = f2{b0[2 * P], b0[2 * P + 1]};
        g0p[P] = f2{g0[2 * P], g0[2 * P + 1]};
        e0p[P] = f2{e0[2 * P], e0[2 * P + 1]};
        bpp[P] = f2{bp[2 * P], bp[2 * P + 1]};
        b1p[P] = f2{b1[2 * P], b1[2 * P + 1]};
        g1p[P] = f2{g1[2 * P], g1[2 * P + 1]};
        e1p[P] = f2{e1[2 * P], e1[2 * P + 1]};
    }
    for (int i0 = 0; i0 < n; i0 += NB) {
        f2 v[NB][2];
        float s[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int i = i0 + b;
            f2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
            if (i < n)
                for (int p = rp[i]; p < rp[i + 1]; ++p) {
                    const float w = al[p * H + wave];
                    const uint2 u = *reinterpret_cast<const uint2*>(xs + (size_t)cl[p] * HC + f0);
                    const f2 x01 = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u)};
                    const f2 x23 = {__uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
                    acc0 += w * x01;
                    acc1 += w * x23;
                }
            v[b][0] = acc0 + b1p[0];
            v[b][1] = acc1 + b1p[1];
            const f2 t = v[b][0] + v[b][1];
            s[b] = wave_sum_l0(t.x + t.y);
        }
        if (lane == 0)
#pragma unroll
            for (int b = 0; b < NB; ++b) red[wave * NB + b] = s[b];
        __syncthreads();
        float mean[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            float t = 0.0f;
            for (int w = 0; w < NW; ++w) t += red[w * NB + b];
            mean[b] = t / (float)HC;
            const f2 d0 = v[b][0] - mean[b], d1 = v[b][1] - mean[b];
            const f2 q = d0 * d0 + d1 * d1;
            s[b] = wave_sum_l0(q.x + q.y);
        }
        if (lane == 0)
#pragma unroll
            for (int b = 0; b < NB; ++b) red[(NW + wave) * NB + b] = s[b];
        __syncthreads();
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int i = i0 + b;
            if (i >= n) break;
            float t = 0.0f;
            for (int w = 0; w < NW; ++w) t += red[(NW + w) * NB + b];
            const float rstd = rsqrtf(t / (float)HC + a.ln_eps);
            // layer 0's row i, channels f0..f0+3 (trx_gat_layer0_infer's expression)
            const float* d = dsc + i * DS;
            const float4 xb4 = *reinterpret_cast<const float4*>(d + 4 * h0);
            const float4 x4 = *reinterpret_cast<const float4*>(d + 4 * H0);
            const float mean0 = d[4 * H0 + 4], rstd0 = d[4 * H0 + 5];
            f2 y[2];
#pragma unroll
            for (int P = 0; P < 2; ++P) {
                const f2 v0 = ((xb4.x * w0p[0][P] + xb4.y * w0p[1][P]) + (xb4.z * w0p[2][P] + xb4.w * w0p[3][P])) + b0p[P];
                const f2 res = ((x4.x * wpp[0][P] + x4.y * wpp[1][P]) + (x4.z * wpp[2][P] + x4.w * wpp[3][P])) + bpp[P];
                f2 y0 = (g0p[P] * (rstd0 * (v0 - mean0)) + e0p[P]) + res;
                y0.x = y0.x > 0.0f ? y0.x : 0.0f;
                y0.y = y0.y > 0.0f ? y0.y : 0.0f;
                f2 yy = (g1p[P] * (rstd * (v[b][P] - mean[b])) + e1p[P]) + y0;
                yy.x = yy.x > 0.0f ? yy.x : 0.0f;
                yy.y = yy.y > 0.0f ? yy.y : 0.0f;
                y[P] = yy;
            }
            const size_t o = (size_t)(node0 + i) * HC + f0;
            if (a.out_f32) *reinterpret_cast<float4*>(a.out_f32 + o) = make_float4(y[0].x, y[0].y, y[1].x, y[1].y);
            if (a.out_bf16)
                *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.out_bf16) + o) =
                    make_uint2(pk_bf16_l0(y[0].x, y[0].y), pk_bf16_l0(y[1].x, y[1].y));
        }
    }
}

// Per-weight-set constants: u = [W0_h^T att_src_h ; W0_h^T att_dst_h] (float32
// [2, H, 4], from float64 sums) and the LayerNorm forms (float64, layout above).
// One workgroup per head (+ one for the bias sums): each thread forms its
// channels' 32 products (4 u_src, 4 u_dst, 4 s, 4 t, 16 G) in float64, then
// a fixed-order tree reduction over the workgroup (deterministic).
__global__ void __launch_bounds__(256) gat_layer0_prepare_kernel(int H, int C, const float* __restrict__ w0,
                                                                  const float* __restrict__ att_src,
                                                                  const float* __restrict__ att_dst,
                                                                  const float* __restrict__ bias, float* __restrict__ u,
                                                                  double* __restrict__ stats) {
    __shared__ double red[256];
    const int tid = threadIdx.x, h = blockIdx.x;
    if (h == H) {  // sum b, sum b^2 over all channels
        for (int q = 0; q < 2; ++q) {
            double acc = 0.0;
            for (int c = tid; c < H * C; c += 256) {
                const double b = bias[c];
                acc += q == 0 ? b : b * b;
            }
            red[tid] = acc;
            __syncthreads();
            for (int w = 128; w > 0; w >>= 1) {
                if (tid < w) red[tid] += red[tid + w];
                __syncthreads();
            }
            if (tid == 0) stats[H * 24 + q] = red[0];
            __syncthreads();
        }
        return;
    }
    double acc[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) acc[q] = 0.0;
    for (int c = h * C + tid; c < (h + 1) * C; c += 256) {
        const float4 wv = *reinterpret_cast<const float4*>(w0 + (size_t)c * 4);
        const double w[4] = {wv.x, wv.y, wv.z, wv.w};
        const double as = att_src[c], ad = att_dst[c], b = bias[c];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            acc[k] += w[k] * as;
            acc[4 + k] += w[k] * ad;
            acc[8 + k] += w[k];
            acc[12 + k] += b * w[k];
#pragma unroll
            for (int l = 0; l < 4; ++l) acc[16 + 4 * k + l] += w[k] * w[l];
        }
    }
    for (int q = 0; q < 32; ++q) {
        red[tid] = acc[q];
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (tid < w) red[tid] += red[tid + w];
            __syncthreads();
        }
        if (tid == 0) {
            const double v = red[0];
            if (q < 4)
                u[4 * h + q] = (float)v;
            else if (q < 8)
                u[4 * (H + h) + q - 4] = (float)v;
            else
                stats[24 * h + (q - 8)] = v;
        }
        __syncthreads();
    }
}

}  // namespace

size_t gat_layer0_smem(const trx_gat_layer0_args& a) {
    const size_t n = a.nodes_per_graph, H = a.heads, me = a.max_graph_edges;
    return (n * 4 + 2 * n * H + n * H * 4 + 2 * n + me * H) * 4 + (2 * me + n + 1) * 4;
}

hipError_t launch_gat_layer0(const trx_gat_layer0_args& a, hipStream_t stream) {
    const int HC = a.heads * a.channels;
    const size_t smem = gat_layer0_smem(a);
    const dim3 grid(a.num_graphs);
    switch (HC) {
        case 256:
            hipLaunchKernelGGL((gat_layer0_lin_kernel<256>), grid, dim3(64), smem, stream, a);
            break;
        case 512:
            hipLaunchKernelGGL((gat_layer0_lin_kernel<512>), grid, dim3(128), smem, stream, a);
            break;
        default:
            hipLaunchKernelGGL((gat_layer0_lin_kernel<1024>), grid, dim3(256), smem, stream, a);
            break;
    }
    return hipGetLastError();
}

constexpr int kMidNB = 8;

size_t gat_mid_smem(const trx_gat_mid_args& a) {
    const size_t n = a.nodes_per_graph, H = a.heads, me = a.max_graph_edges, HC = (size_t)a.heads * a.channels;
    const size_t DS = 4 * (size_t)a.l0_heads + 8;
    return n * HC * 2 + (n * DS + 2 * n * H + 2 * (HC / 256) * kMidNB + me * H) * 4 + (2 * me + n + 1) * 4;
}

hipError_t launch_gat_mid(const trx_gat_mid_args& a, hipStream_t stream) {
    const int HC = a.heads * a.channels;
    const size_t smem = gat_mid_smem(a);
    static bool attr_set = false;
    if (!attr_set) {  // > 64 KB of dynamic LDS at n = 32
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gat_mid_gen_kernel<1024, kMidNB>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    const dim3 grid(a.num_graphs);
    switch (HC) {
        case 256:
            hipLaunchKernelGGL((gat_mid_gen_kernel<256, kMidNB>), grid, dim3(64), smem, stream, a);
            break;
        case 512:
            hipLaunchKernelGGL((gat_mid_gen_kernel<512, kMidNB>), grid, dim3(128), smem, stream, a);
            break;
        default:
            hipLaunchKernelGGL((gat_mid_gen_kernel<1024, kMidNB>), grid, dim3(256), smem, stream, a);
            break;
    }
    return hipGetLastError();
}

hipError_t launch_gat_layer0_prepare(int H, int C, const float* w0, const float* att_src, const float* att_dst,
                                     const float* bias, float* u, double* stats, hipStream_t stream) {
    hipLaunchKernelGGL(gat_layer0_prepare_kernel, dim3(H + 1), dim3(256), 0, stream, H, C, w0, att_src, att_dst, bias,
                       u, stats);
    return hipGetLastError();
}

}  // namespace trx

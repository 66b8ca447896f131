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
        if (a.out_f32) *reinterpret_cast<float4*>(a.out_f32 + o) = make_float4(y[0], y[1], y[2], y[3]);
        if (a.out_bf16)
            *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.out_bf16) + o) =
                make_uint2(pk_bf16_l0(y[0], y[1]), pk_bf16_l0(y[2], y[3]));
    }
}

// Per-weight-set constants: u = [W0_h^T att_src_h ; W0_h^T att_dst_h] (float32
// [2, H, 4], from float64 sums) and the LayerNorm forms (float64, layout above).
// One workgroup of 256 threads; thread (h, q) sums one quantity over the head's
// C channels in channel order.
__global__ void __launch_bounds__(256) gat_layer0_prepare_kernel(int H, int C, const float* __restrict__ w0,
                                                                  const float* __restrict__ att_src,
                                                                  const float* __restrict__ att_dst,
                                                                  const float* __restrict__ bias, float* __restrict__ u,
                                                                  double* __restrict__ stats) {
    // quantities per head: 4 u_src + 4 u_dst + 4 s + 4 t + 16 G = 32
    for (int t = threadIdx.x; t < H * 32 + 2; t += blockDim.x) {
        double acc = 0.0;
        if (t >= H * 32) {
            for (int c = 0; c < H * C; ++c) {
                const double b = bias[c];
                acc += t == H * 32 ? b : b * b;
            }
            stats[H * 24 + (t - H * 32)] = acc;
            continue;
        }
        const int h = t / 32, q = t - h * 32;
        for (int c = h * C; c < (h + 1) * C; ++c) {
            const float* wr = w0 + (size_t)c * 4;
            if (q < 4)
                acc += (double)wr[q] * (double)att_src[c];
            else if (q < 8)
                acc += (double)wr[q - 4] * (double)att_dst[c];
            else if (q < 12)
                acc += (double)wr[q - 8];
            else if (q < 16)
                acc += (double)bias[c] * (double)wr[q - 12];
            else
                acc += (double)wr[(q - 16) >> 2] * (double)wr[(q - 16) & 3];
        }
        if (q < 4)
            u[4 * h + q] = (float)acc;
        else if (q < 8)
            u[4 * (H + h) + q - 4] = (float)acc;
        else
            stats[24 * h + (q - 8)] = acc;
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

hipError_t launch_gat_layer0_prepare(int H, int C, const float* w0, const float* att_src, const float* att_dst,
                                     const float* bias, float* u, double* stats, hipStream_t stream) {
    hipLaunchKernelGGL(gat_layer0_prepare_kernel, dim3(1), dim3(256), 0, stream, H, C, w0, att_src, att_dst, bias, u,
                       stats);
    return hipGetLastError();
}

}  // namespace trx

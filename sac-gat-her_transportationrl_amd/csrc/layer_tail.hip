// layer_tail.hip -- the post-aggregation tail of a GATEncoder layer in the
// training (autograd) path, forward and backward as single kernels.
//
// GATEncoder (src/models/gat_encoder.py:40-49) after each GATConv:
//     z = out + bias;  h = LayerNorm(z; w, b)
//     middle layers: y = relu(h + res)     last layer: y = elu(h)
// Through torch ops that is 4 kernels forward (bias add, LayerNorm, residual
// add, ReLU) and ~7 backward (ReLU backward, LayerNorm input / gamma / beta
// gradients, bias reduction, residual add), each a pass over an [N, F] fp32
// tensor.  Here: forward = one wave per row (lane owns float4 chunks
// q = lane + 64k), z / h / y in registers, mean and rstd saved per row;
// backward = one wave per row for dz and dres, with the column sums of
// dz (bias), dh*xhat (LayerNorm weight) and dh (LayerNorm bias) accumulated
// per workgroup over kTailRows rows and written as partials, then one
// reduction launch sums the partials over a fixed tree (deterministic).
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kWave = 64;
constexpr int kTailWaves = 4;
constexpr int kTailRows = 16;      // rows per workgroup in the backward (4 per wave): >= 384 workgroups at N = 6144
constexpr int kTailChunks = 4;     // F <= 64 * 4 * 4 = 1024

#define TRX_DPPS(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, false))
#define TRX_RL(v, l) __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l))
__device__ __forceinline__ float wave_sum(float v) {
    v = v + TRX_DPPS(v, 0xB1);
    v = v + TRX_DPPS(v, 0x4E);
    v = v + TRX_DPPS(v, 0x141);
    v = v + TRX_DPPS(v, 0x140);
    return (TRX_RL(v, 0) + TRX_RL(v, 16)) + (TRX_RL(v, 32) + TRX_RL(v, 48));
}
#undef TRX_DPPS
#undef TRX_RL

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }

template <typename TR>
__device__ __forceinline__ float4 ld_res(const TR* p);
template <>
__device__ __forceinline__ float4 ld_res<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <>
__device__ __forceinline__ float4 ld_res<uint16_t>(const uint16_t* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
}
template <typename TR>
__device__ __forceinline__ void st_res(TR* p, float4 v);
template <>
__device__ __forceinline__ void st_res<float>(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
template <>
__device__ __forceinline__ void st_res<uint16_t>(uint16_t* p, float4 v) {
    uint2 u;
    u.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
    u.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
    *reinterpret_cast<uint2*>(p) = u;
}

// ACT: 0 relu(h + res), 1 elu(h).  TR: residual dtype (float / bf16 bits).
template <int ACT, typename TR>
__global__ void __launch_bounds__(kWave * kTailWaves)
    layer_tail_fwd_kernel(int N, int F, const float* __restrict__ out, const float* __restrict__ bias,
                          const float* __restrict__ w, const float* __restrict__ b, float eps,
                          const TR* __restrict__ res, float* __restrict__ y, float* __restrict__ stats) {
    const int lane = threadIdx.x & (kWave - 1);
    const int i = blockIdx.x * kTailWaves + threadIdx.x / kWave;
    if (i >= N) return;
    const int nq = F / 4;
    float4 z[kTailChunks];
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < kTailChunks; ++k) {
        const int q = lane + kWave * k;
        z[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q < nq) {
            const float4 o = *reinterpret_cast<const float4*>(out + (size_t)i * F + 4 * q);
            const float4 bb = *reinterpret_cast<const float4*>(bias + 4 * q);
            z[k] = make_float4(o.x + bb.x, o.y + bb.y, o.z + bb.z, o.w + bb.w);
            s += (z[k].x + z[k].y) + (z[k].z + z[k].w);
        }
    }
    const float mean = wave_sum(s) / (float)F;
    float s2 = 0.0f;
#pragma unroll
    for (int k = 0; k < kTailChunks; ++k) {
        const int q = lane + kWave * k;
        if (q < nq) {
            const float dx = z[k].x - mean, dy = z[k].y - mean, dz = z[k].z - mean, dw = z[k].w - mean;
            s2 += (dx * dx + dy * dy) + (dz * dz + dw * dw);
        }
    }
    const float rstd = rsqrtf(wave_sum(s2) / (float)F + eps);
#pragma unroll
    for (int k = 0; k < kTailChunks; ++k) {
        const int q = lane + kWave * k;
        if (q < nq) {
            const float4 ww = *reinterpret_cast<const float4*>(w + 4 * q);
            const float4 bb = *reinterpret_cast<const float4*>(b + 4 * q);
            float4 h = make_float4((z[k].x - mean) * rstd * ww.x + bb.x, (z[k].y - mean) * rstd * ww.y + bb.y,
                                   (z[k].z - mean) * rstd * ww.z + bb.z, (z[k].w - mean) * rstd * ww.w + bb.w);
            if (ACT == 0) {
                const float4 r = ld_res<TR>(res + (size_t)i * F + 4 * q);
                h = make_float4(fmaxf(h.x + r.x, 0.0f), fmaxf(h.y + r.y, 0.0f), fmaxf(h.z + r.z, 0.0f),
                                fmaxf(h.w + r.w, 0.0f));
            } else {
                h = make_float4(h.x > 0.0f ? h.x : expm1f(h.x), h.y > 0.0f ? h.y : expm1f(h.y),
                                h.z > 0.0f ? h.z : expm1f(h.z), h.w > 0.0f ? h.w : expm1f(h.w));
            }
            *reinterpret_cast<float4*>(y + (size_t)i * F + 4 * q) = h;
        }
    }
    if (lane == 0) {
        stats[2 * i] = mean;
        stats[2 * i + 1] = rstd;
    }
}

// Backward: dz (= d out = d bias rows), dres; column partials [blk][3][F].
template <int ACT, typename TR>
__global__ void __launch_bounds__(kWave * kTailWaves)
    layer_tail_bwd_kernel(int N, int F, const float* __restrict__ gy, const float* __restrict__ out,
                          const float* __restrict__ bias, const float* __restrict__ w, const float* __restrict__ y,
                          const float* __restrict__ stats, float* __restrict__ gout, TR* __restrict__ gres,
                          float* __restrict__ part) {
    __shared__ float red[kTailWaves][kTailChunks * kWave * 4];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int nq = F / 4;
    float4 cb[kTailChunks], cw[kTailChunks], cbb[kTailChunks];  // column partials: dz, dh*xhat, dh
#pragma unroll
    for (int k = 0; k < kTailChunks; ++k) cb[k] = cw[k] = cbb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int row0 = blockIdx.x * kTailRows;
    for (int i = row0 + wv; i < row0 + kTailRows && i < N; i += kTailWaves) {
        const float mean = stats[2 * i], rstd = stats[2 * i + 1];
        float4 dh[kTailChunks], xh[kTailChunks], wl[kTailChunks];
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
        for (int k = 0; k < kTailChunks; ++k) {
            const int q = lane + kWave * k;
            dh[k] = xh[k] = wl[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < nq) {
                const size_t o = (size_t)i * F + 4 * q;
                const float4 g = *reinterpret_cast<const float4*>(gy + o);
                const float4 yy = *reinterpret_cast<const float4*>(y + o);
                const float4 ot = *reinterpret_cast<const float4*>(out + o);
                const float4 bb = *reinterpret_cast<const float4*>(bias + 4 * q);
                wl[k] = *reinterpret_cast<const float4*>(w + 4 * q);
                float4 d;
                if (ACT == 0) {
                    d = make_float4(yy.x > 0.0f ? g.x : 0.0f, yy.y > 0.0f ? g.y : 0.0f, yy.z > 0.0f ? g.z : 0.0f,
                                    yy.w > 0.0f ? g.w : 0.0f);
                    st_res<TR>(gres + o, d);
                } else {
                    d = make_float4(yy.x > 0.0f ? g.x : g.x * (yy.x + 1.0f), yy.y > 0.0f ? g.y : g.y * (yy.y + 1.0f),
                                    yy.z > 0.0f ? g.z : g.z * (yy.z + 1.0f), yy.w > 0.0f ? g.w : g.w * (yy.w + 1.0f));
                }
                dh[k] = d;
                xh[k] = make_float4(((ot.x + bb.x) - mean) * rstd, ((ot.y + bb.y) - mean) * rstd,
                                    ((ot.z + bb.z) - mean) * rstd, ((ot.w + bb.w) - mean) * rstd);
                const float4 dw = make_float4(d.x * wl[k].x, d.y * wl[k].y, d.z * wl[k].z, d.w * wl[k].w);
                s1 += (dw.x + dw.y) + (dw.z + dw.w);
                s2 += (dw.x * xh[k].x + dw.y * xh[k].y) + (dw.z * xh[k].z + dw.w * xh[k].w);
                cw[k] = make_float4(cw[k].x + d.x * xh[k].x, cw[k].y + d.y * xh[k].y, cw[k].z + d.z * xh[k].z,
                                    cw[k].w + d.w * xh[k].w);
                cbb[k] = make_float4(cbb[k].x + d.x, cbb[k].y + d.y, cbb[k].z + d.z, cbb[k].w + d.w);
            }
        }
        const float m1 = wave_sum(s1) / (float)F, m2 = wave_sum(s2) / (float)F;
#pragma unroll
        for (int k = 0; k < kTailChunks; ++k) {
            const int q = lane + kWave * k;
            if (q < nq) {
                const float4 d = dh[k];
                const float4 dz = make_float4(rstd * (d.x * wl[k].x - m1 - xh[k].x * m2),
                                              rstd * (d.y * wl[k].y - m1 - xh[k].y * m2),
                                              rstd * (d.z * wl[k].z - m1 - xh[k].z * m2),
                                              rstd * (d.w * wl[k].w - m1 - xh[k].w * m2));
                *reinterpret_cast<float4*>(gout + (size_t)i * F + 4 * q) = dz;
                cb[k] = make_float4(cb[k].x + dz.x, cb[k].y + dz.y, cb[k].z + dz.z, cb[k].w + dz.w);
            }
        }
    }
    // combine the waves' column partials in wave order, write this workgroup's partial
#pragma unroll
    for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int k = 0; k < kTailChunks; ++k) {
            const float4 v = t == 0 ? cb[k] : t == 1 ? cw[k] : cbb[k];
            const int c = 4 * (lane + kWave * k);
            red[wv][c] = v.x;
            red[wv][c + 1] = v.y;
            red[wv][c + 2] = v.z;
            red[wv][c + 3] = v.w;
        }
        __syncthreads();
        for (int c = threadIdx.x; c < F; c += kWave * kTailWaves) {
            float v = 0.0f;
#pragma unroll
            for (int ww = 0; ww < kTailWaves; ++ww) v += red[ww][c];
            part[((size_t)blockIdx.x * 3 + t) * F + c] = v;
        }
        __syncthreads();
    }
}

// grads[idx] = sum over workgroups of part[blk][idx]: one wave per output,
// lanes over workgroups, fixed DPP tree (deterministic)
__global__ void __launch_bounds__(256) layer_tail_reduce_kernel(int nblk, int F, const float* __restrict__ part,
                                                                float* __restrict__ grads) {
    const int lane = threadIdx.x & (kWave - 1), idx = blockIdx.x * 4 + threadIdx.x / kWave;
    if (idx >= 3 * F) return;
    float v = 0.0f;
    for (int blk = lane; blk < nblk; blk += kWave) v += part[(size_t)blk * 3 * F + idx];
    v = wave_sum(v);
    if (lane == 0) grads[idx] = v;
}

}  // namespace

int layer_tail_blocks(int N) { return (N + kTailRows - 1) / kTailRows; }

hipError_t launch_layer_tail_fwd(int N, int F, int act, int res_bf16, const float* out, const float* bias,
                                 const float* w, const float* b, float eps, const void* res, float* y, float* stats,
                                 hipStream_t stream) {
    const dim3 grid((N + kTailWaves - 1) / kTailWaves), block(kWave * kTailWaves);
    if (act == 1)
        hipLaunchKernelGGL((layer_tail_fwd_kernel<1, float>), grid, block, 0, stream, N, F, out, bias, w, b, eps,
                           static_cast<const float*>(nullptr), y, stats);
    else if (res_bf16)
        hipLaunchKernelGGL((layer_tail_fwd_kernel<0, uint16_t>), grid, block, 0, stream, N, F, out, bias, w, b, eps,
                           static_cast<const uint16_t*>(res), y, stats);
    else
        hipLaunchKernelGGL((layer_tail_fwd_kernel<0, float>), grid, block, 0, stream, N, F, out, bias, w, b, eps,
                           static_cast<const float*>(res), y, stats);
    return hipGetLastError();
}

hipError_t launch_layer_tail_bwd(int N, int F, int act, int res_bf16, const float* gy, const float* out,
                                 const float* bias, const float* w, const float* y, const float* stats, float* gout,
                                 void* gres, float* part, float* grads, hipStream_t stream) {
    const int nblk = layer_tail_blocks(N);
    const dim3 grid(nblk), block(kWave * kTailWaves);
    if (act == 1)
        hipLaunchKernelGGL((layer_tail_bwd_kernel<1, float>), grid, block, 0, stream, N, F, gy, out, bias, w, y, stats,
                           gout, static_cast<float*>(nullptr), part);
    else if (res_bf16)
        hipLaunchKernelGGL((layer_tail_bwd_kernel<0, uint16_t>), grid, block, 0, stream, N, F, gy, out, bias, w, y,
                           stats, gout, static_cast<uint16_t*>(gres), part);
    else
        hipLaunchKernelGGL((layer_tail_bwd_kernel<0, float>), grid, block, 0, stream, N, F, gy, out, bias, w, y, stats,
                           gout, static_cast<float*>(gres), part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(layer_tail_reduce_kernel, dim3((3 * F + 3) / 4), dim3(256), 0, stream, nblk, F, part, grads);
    return hipGetLastError();
}

}  // namespace trx

// att_dots.hip -- GATConv's per-head attention dot products in the training
// (autograd) path: a_src[i,h] = <xh[i,h,:], att_src[h,:]>, a_dst likewise
// (PyG GATConv, src/models/gat_encoder.py:22-25).  Through torch this was a
// float32 cast of xh, a block-diagonal [H*C, 2H] matrix built from the
// attention vectors, a GEMM, and on the way back a GEMM, a cast, a split-K
// weight product and the block-matrix backward -- ~20 launches per layer.
// Here: forward = one wave per node (lane owns float4 chunks q = lane + 64k,
// each inside one head since C % 4 == 0), per-head masked DPP wave sums;
// backward = one wave per node for dxh = g_src[h] att_src + g_dst[h] att_dst
// (written in xh's dtype) with the column sums for d att accumulated per
// workgroup, then one fixed-order reduction launch.
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kWave = 64;
constexpr int kAdWaves = 4;
constexpr int kAdRows = 16;    // rows per workgroup in the backward (>= 384 workgroups at N = 6144)
constexpr int kAdChunks = 4;   // H*C <= 1024
constexpr int kAdHeads = 8;

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

template <typename T>
__device__ __forceinline__ float4 ld4(const T* p);
template <>
__device__ __forceinline__ float4 ld4<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <>
__device__ __forceinline__ float4 ld4<uint16_t>(const uint16_t* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
}
template <typename T>
__device__ __forceinline__ void st4(T* p, float4 v);
template <>
__device__ __forceinline__ void st4<float>(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
template <>
__device__ __forceinline__ void st4<uint16_t>(uint16_t* p, float4 v) {
    uint2 u;
    u.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.x) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.y) << 16);
    u.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.z) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.w) << 16);
    *reinterpret_cast<uint2*>(p) = u;
}
__device__ __forceinline__ float dot4(float4 a, float4 b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w); }

template <typename T>
__global__ void __launch_bounds__(kWave * kAdWaves)
    att_dots_fwd_kernel(int N, int H, int C, const T* __restrict__ xh, const float* __restrict__ att_src,
                        const float* __restrict__ att_dst, float* __restrict__ a_src, float* __restrict__ a_dst) {
    const int lane = threadIdx.x & (kWave - 1);
    const int i = blockIdx.x * kAdWaves + threadIdx.x / kWave;
    if (i >= N) return;
    const int HC = H * C, nq = HC / 4;
    float ps[kAdHeads], pd[kAdHeads];
#pragma unroll
    for (int h = 0; h < kAdHeads; ++h) ps[h] = pd[h] = 0.0f;
#pragma unroll
    for (int k = 0; k < kAdChunks; ++k) {
        const int q = lane + kWave * k;
        if (q < nq) {
            const float4 x = ld4<T>(xh + (size_t)i * HC + 4 * q);
            const float s = dot4(x, *reinterpret_cast<const float4*>(att_src + 4 * q));
            const float d = dot4(x, *reinterpret_cast<const float4*>(att_dst + 4 * q));
            const int hq = (4 * q) / C;
#pragma unroll
            for (int h = 0; h < kAdHeads; ++h)
                if (h == hq) {
                    ps[h] += s;
                    pd[h] += d;
                }
        }
    }
#pragma unroll
    for (int h = 0; h < kAdHeads; ++h)
        if (h < H) {
            const float s = wave_sum(ps[h]), d = wave_sum(pd[h]);
            if (lane == 0) {
                a_src[(size_t)i * H + h] = s;
                a_dst[(size_t)i * H + h] = d;
            }
        }
}

template <typename T>
__global__ void __launch_bounds__(kWave * kAdWaves)
    att_dots_bwd_kernel(int N, int H, int C, const T* __restrict__ xh, const float* __restrict__ att_src,
                        const float* __restrict__ att_dst, const float* __restrict__ g_src,
                        const float* __restrict__ g_dst, T* __restrict__ g_xh, float* __restrict__ part) {
    __shared__ float red[kAdWaves][kAdChunks * kWave * 4];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int HC = H * C, nq = HC / 4;
    float4 as[kAdChunks], ad[kAdChunks], cs[kAdChunks], cd[kAdChunks];
    int hq[kAdChunks];
#pragma unroll
    for (int k = 0; k < kAdChunks; ++k) {
        const int q = lane + kWave * k;
        hq[k] = (4 * q) / C;
        cs[k] = cd[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        as[k] = q < nq ? *reinterpret_cast<const float4*>(att_src + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        ad[k] = q < nq ? *reinterpret_cast<const float4*>(att_dst + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int row0 = blockIdx.x * kAdRows;
    for (int i = row0 + wv; i < row0 + kAdRows && i < N; i += kAdWaves) {
#pragma unroll
        for (int k = 0; k < kAdChunks; ++k) {
            const int q = lane + kWave * k;
            if (q < nq) {
                const float gs = g_src[(size_t)i * H + hq[k]], gd = g_dst[(size_t)i * H + hq[k]];
                const float4 x = ld4<T>(xh + (size_t)i * HC + 4 * q);
                st4<T>(g_xh + (size_t)i * HC + 4 * q,
                       make_float4(gs * as[k].x + gd * ad[k].x, gs * as[k].y + gd * ad[k].y,
                                   gs * as[k].z + gd * ad[k].z, gs * as[k].w + gd * ad[k].w));
                cs[k] = make_float4(cs[k].x + gs * x.x, cs[k].y + gs * x.y, cs[k].z + gs * x.z, cs[k].w + gs * x.w);
                cd[k] = make_float4(cd[k].x + gd * x.x, cd[k].y + gd * x.y, cd[k].z + gd * x.z, cd[k].w + gd * x.w);
            }
        }
    }
    // combine the waves' column partials in wave order: part[blk][t][HC]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int k = 0; k < kAdChunks; ++k) {
            const float4 v = t == 0 ? cs[k] : cd[k];
            const int c = 4 * (lane + kWave * k);
            red[wv][c] = v.x;
            red[wv][c + 1] = v.y;
            red[wv][c + 2] = v.z;
            red[wv][c + 3] = v.w;
        }
        __syncthreads();
        for (int c = threadIdx.x; c < HC; c += kWave * kAdWaves) {
            float v = 0.0f;
#pragma unroll
            for (int ww = 0; ww < kAdWaves; ++ww) v += red[ww][c];
            part[((size_t)blockIdx.x * 2 + t) * HC + c] = v;
        }
        __syncthreads();
    }
}

// out[idx] = sum over workgroups of part[blk][idx], idx < 2*HC: one wave per
// output, lanes over workgroups, fixed DPP tree (deterministic)
__global__ void __launch_bounds__(256) att_dots_reduce_kernel(int nblk, int n_out, const float* __restrict__ part,
                                                              float* __restrict__ out) {
    const int lane = threadIdx.x & (kWave - 1), idx = blockIdx.x * 4 + threadIdx.x / kWave;
    if (idx >= n_out) return;
    float v = 0.0f;
    for (int blk = lane; blk < nblk; blk += kWave) v += part[(size_t)blk * n_out + idx];
    v = wave_sum(v);
    if (lane == 0) out[idx] = v;
}

}  // namespace

int att_dots_blocks(int N) { return (N + kAdRows - 1) / kAdRows; }

hipError_t launch_att_dots_fwd(int N, int H, int C, const void* xh, int bf16, const float* att_src,
                               const float* att_dst, float* a_src, float* a_dst, hipStream_t stream) {
    const dim3 grid((N + kAdWaves - 1) / kAdWaves), block(kWave * kAdWaves);
    if (bf16)
        hipLaunchKernelGGL(att_dots_fwd_kernel<uint16_t>, grid, block, 0, stream, N, H, C,
                           static_cast<const uint16_t*>(xh), att_src, att_dst, a_src, a_dst);
    else
        hipLaunchKernelGGL(att_dots_fwd_kernel<float>, grid, block, 0, stream, N, H, C, static_cast<const float*>(xh),
                           att_src, att_dst, a_src, a_dst);
    return hipGetLastError();
}

hipError_t launch_att_dots_bwd(int N, int H, int C, const void* xh, int bf16, const float* att_src,
                               const float* att_dst, const float* g_src, const float* g_dst, void* g_xh,
                               float* g_att, float* part, hipStream_t stream) {
    const int nblk = att_dots_blocks(N);
    const dim3 grid(nblk), block(kWave * kAdWaves);
    if (bf16)
        hipLaunchKernelGGL(att_dots_bwd_kernel<uint16_t>, grid, block, 0, stream, N, H, C,
                           static_cast<const uint16_t*>(xh), att_src, att_dst, g_src, g_dst,
                           static_cast<uint16_t*>(g_xh), part);
    else
        hipLaunchKernelGGL(att_dots_bwd_kernel<float>, grid, block, 0, stream, N, H, C, static_cast<const float*>(xh),
                           att_src, att_dst, g_src, g_dst, static_cast<float*>(g_xh), part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int n_out = 2 * H * C;
    hipLaunchKernelGGL(att_dots_reduce_kernel, dim3((n_out + 3) / 4), dim3(256), 0, stream, nblk, n_out, part, g_att);
    return hipGetLastError();
}

}  // namespace trx

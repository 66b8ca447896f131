// gat_kernel.hip -- GATConv edge softmax + neighbour aggregation on gfx950.
//
// Replaces the message-passing core of torch_geometric GATConv as used by
// src/models/gat_encoder.py:22-25,36-42 (heads=4, negative_slope=0.2,
// self loops with mean edge_attr, softmax over each destination's in-edges
// with the PyG +1e-16 denominator):
//     logit_e,h = leaky_relu(a_src[j,h] + a_dst[i,h] + a_edge[e,h], slope)
//     alpha_e,h = exp(logit - max_dst) / (sum_dst exp(logit - max_dst) + 1e-16)
//     out[i,h,:] = sum_{e=(j->i)} alpha_e,h * xh[j,h,:]
// The dense projections (lin, att dot products) stay in MFMA GEMMs on the
// torch side; this file owns the gather/scatter-bound part.
//
// Layout: graph in CSR by destination (rowptr, src) -- the order PyG's
// scatter uses is irrelevant for the max/sum but our sums run in CSR order,
// deterministic.  xh row-major [Nt, H*C] float32 or bfloat16 (C % 4 == 0).
// One wave64 per node; each lane owns float4 column chunks q = lane + 64k.
//
// Backward is two deterministic kernels (no float atomics):
//   per destination: dalpha = <gout_i, xh_j> -> softmax/leaky_relu backward
//                    -> ga_edge, ga_dst
//   per source:      gxh_j = sum alpha * gout_i, ga_src_j = sum dlogit
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kWave = 64;
constexpr int kGatWaves = 4;         // waves (nodes) per workgroup
constexpr int kMaxChunks = 8;        // float4 chunks per lane: H*C <= 64*4*8 = 2048
constexpr int kMaxDegCache = 64;     // in-edges whose alphas are cached in LDS

// Wave reductions on DPP row ops + readlane (no LDS round trips, unlike
// ds_bpermute shuffles): every lane gets the (uniform) result.
#define TRX_DPPS(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, false))
#define TRX_DPPM(v, ctrl) \
    __int_as_float(__builtin_amdgcn_update_dpp((int)0xff800000, __float_as_int(v), ctrl, 0xf, 0xf, false))
#define TRX_RL(v, l) __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l))
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, TRX_DPPM(v, 0xB1));   // quad_perm [1,0,3,2]
    v = fmaxf(v, TRX_DPPM(v, 0x4E));   // quad_perm [2,3,0,1]
    v = fmaxf(v, TRX_DPPM(v, 0x141));  // row_half_mirror
    v = fmaxf(v, TRX_DPPM(v, 0x140));  // row_mirror
    return fmaxf(fmaxf(TRX_RL(v, 0), TRX_RL(v, 16)), fmaxf(TRX_RL(v, 32), TRX_RL(v, 48)));
}
__device__ __forceinline__ float wave_sum(float v) {
    v = v + TRX_DPPS(v, 0xB1);
    v = v + TRX_DPPS(v, 0x4E);
    v = v + TRX_DPPS(v, 0x141);
    v = v + TRX_DPPS(v, 0x140);
    return (TRX_RL(v, 0) + TRX_RL(v, 16)) + (TRX_RL(v, 32) + TRX_RL(v, 48));
}
#undef TRX_DPPS
#undef TRX_DPPM
#undef TRX_RL
// sum over aligned groups of `group` lanes (power of two <= 64)
__device__ __forceinline__ float group_sum(float v, int group) {
    if (group == kWave) return wave_sum(v);
    for (int o = group >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

template <typename T>
__device__ __forceinline__ float4 load4(const T* p);
template <>
__device__ __forceinline__ float4 load4<float>(const float* p) {
    return *reinterpret_cast<const float4*>(p);
}
template <>
__device__ __forceinline__ float4 load4<__hip_bfloat16>(const __hip_bfloat16* p) {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    float4 f;
    f.x = __uint_as_float(u.x << 16);
    f.y = __uint_as_float(u.x & 0xffff0000u);
    f.z = __uint_as_float(u.y << 16);
    f.w = __uint_as_float(u.y & 0xffff0000u);
    return f;
}

template <typename T>
__device__ __forceinline__ void store4(T* p, float4 v);
template <>
__device__ __forceinline__ void store4<float>(float* p, float4 v) {
    *reinterpret_cast<float4*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<__hip_bfloat16>(__hip_bfloat16* p, float4 v) {
    uint2 u;
    u.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.x) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.y) << 16);
    u.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.z) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v.w) << 16);
    *reinterpret_cast<uint2*>(p) = u;
}

__device__ __forceinline__ float leaky(float x, float slope) { return x > 0.0f ? x : x * slope; }

}  // namespace

// ---------------------------------------------------------------- forward
template <typename T>
__global__ void __launch_bounds__(kWave * kGatWaves)
    gat_fwd_kernel(int Nt, int H, int C, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ src,
                   const T* __restrict__ xh, const float* __restrict__ a_src, const float* __restrict__ a_dst,
                   const float* __restrict__ a_edge, float slope, const float* __restrict__ bias,
                   float* __restrict__ out, float* __restrict__ alpha) {
    __shared__ float s_alpha[kGatWaves][kMaxDegCache * 8];
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    const int i = blockIdx.x * kGatWaves + w;
    if (i >= Nt) return;
    const int HC = H * C;
    const int beg = rowptr[i], deg = rowptr[i + 1] - beg;
    float* sa = s_alpha[w];

    // -------- per-head softmax over the in-edges of i
    if (deg * H <= kWave && H <= 8) {
        // lanes = (edge, head) pairs: one round of gathers, per-head masked wave reductions
        const int e = lane / H, h = lane - (lane / H) * H;
        const bool on = lane < deg * H;
        const float lg = on ? leaky(a_src[(size_t)src[beg + e] * H + h] + a_dst[(size_t)i * H + h] +
                                        a_edge[(size_t)(beg + e) * H + h], slope)
                            : -__builtin_huge_valf();
        float m = -__builtin_huge_valf();
#pragma unroll
        for (int hh = 0; hh < 8; ++hh)
            if (hh < H) {
                const float mh = wave_max(on && h == hh ? lg : -__builtin_huge_valf());
                if (h == hh) m = mh;
            }
        const float ex = on ? __expf(lg - m) : 0.0f;
        float denom = 1.0f;
#pragma unroll
        for (int hh = 0; hh < 8; ++hh)
            if (hh < H) {
                const float sh = wave_sum(h == hh ? ex : 0.0f);
                if (h == hh) denom = sh + 1e-16f;
            }
        if (on) {
            const float al = ex / denom;
            alpha[(size_t)(beg + e) * H + h] = al;
            sa[lane] = al;  // = sa[e * H + h]
        }
    } else
    for (int h = 0; h < H; ++h) {
        const float ad = a_dst[(size_t)i * H + h];
        float m = -__builtin_huge_valf();
        for (int e0 = 0; e0 < deg; e0 += kWave) {
            int e = e0 + lane;
            float v = -__builtin_huge_valf();
            if (e < deg) v = leaky(a_src[(size_t)src[beg + e] * H + h] + ad + a_edge[(size_t)(beg + e) * H + h], slope);
            m = fmaxf(m, wave_max(v));
        }
        float ssum = 0.0f;
        for (int e0 = 0; e0 < deg; e0 += kWave) {
            int e = e0 + lane;
            float ex = 0.0f;
            if (e < deg)
                ex = __expf(leaky(a_src[(size_t)src[beg + e] * H + h] + ad + a_edge[(size_t)(beg + e) * H + h], slope) - m);
            ssum += wave_sum(ex);
        }
        const float denom = ssum + 1e-16f;
        for (int e0 = 0; e0 < deg; e0 += kWave) {
            int e = e0 + lane;
            if (e < deg) {
                float lg = leaky(a_src[(size_t)src[beg + e] * H + h] + ad + a_edge[(size_t)(beg + e) * H + h], slope);
                float al = __expf(lg - m) / denom;
                alpha[(size_t)(beg + e) * H + h] = al;
                if (e < kMaxDegCache && H <= 8) sa[e * H + h] = al;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

    // -------- aggregation: lane owns float4 chunks q = lane + 64k
    const int nq = HC / 4;
    float4 acc[kMaxChunks];
#pragma unroll
    for (int k = 0; k < kMaxChunks; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = 0; e < deg; ++e) {
        const int j = src[beg + e];
        const T* row = xh + (size_t)j * HC;
#pragma unroll
        for (int k = 0; k < kMaxChunks; ++k) {
            const int q = lane + kWave * k;
            if (q < nq) {
                const int h = (4 * q) / C;
                const float al = (e < kMaxDegCache && H <= 8) ? sa[e * H + h] : alpha[(size_t)(beg + e) * H + h];
                float4 x = load4<T>(row + 4 * q);
                acc[k].x += al * x.x;
                acc[k].y += al * x.y;
                acc[k].z += al * x.z;
                acc[k].w += al * x.w;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxChunks; ++k) {
        const int q = lane + kWave * k;
        if (q < nq) {
            float4 r = acc[k];
            if (bias) {
                float4 b = *reinterpret_cast<const float4*>(bias + 4 * q);
                r.x += b.x; r.y += b.y; r.z += b.z; r.w += b.w;
            }
            *reinterpret_cast<float4*>(out + (size_t)i * HC + 4 * q) = r;
        }
    }
}

// ------------------------------------------------------- backward (dst)
template <typename T>
__global__ void __launch_bounds__(kWave * kGatWaves)
    gat_bwd_dst_kernel(int Nt, int H, int C, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ src,
                       const T* __restrict__ xh, const float* __restrict__ a_src, const float* __restrict__ a_dst,
                       const float* __restrict__ a_edge, float slope, const float* __restrict__ alpha,
                       const float* __restrict__ gout, float* __restrict__ dlogit, float* __restrict__ ga_dst) {
    __shared__ float s_da[kGatWaves][kMaxDegCache * 8];
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    const int i = blockIdx.x * kGatWaves + w;
    if (i >= Nt) return;
    const int HC = H * C;
    const int nq = HC / 4;
    const int beg = rowptr[i], deg = rowptr[i + 1] - beg;
    // lanes sharing a head inside one chunk slot k: group of min(64, C/4) lanes
    const int group = (C / 4) < kWave ? (C / 4) : kWave;
    float* sda = s_da[w];
    // gout row of i in registers
    float4 go[kMaxChunks];
#pragma unroll
    for (int k = 0; k < kMaxChunks; ++k) {
        const int q = lane + kWave * k;
        go[k] = q < nq ? *reinterpret_cast<const float4*>(gout + (size_t)i * HC + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // dalpha[e][h] = <gout_i[h], xh_j[h]>
    for (int e = 0; e < deg; ++e) {
        const int j = src[beg + e];
        const T* row = xh + (size_t)j * HC;
        float hs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < kMaxChunks; ++k) {
            const int q = lane + kWave * k;
            float part = 0.0f;
            int h = 0;
            if (q < nq) {
                float4 x = load4<T>(row + 4 * q);
                part = go[k].x * x.x + go[k].y * x.y + go[k].z * x.z + go[k].w * x.w;
                h = (4 * q) / C;
            }
            if (k * kWave < nq) {
                float gsum = group_sum(part, group);
                if (group == kWave) {  // C >= 256: a chunk lies in one head, the sum is wave-uniform
                    const int hk = (4 * kWave * k) / C;
#pragma unroll
                    for (int hh = 0; hh < 8; ++hh) hs[hh] += (hh == hk) ? gsum : 0.0f;
                } else {
                    // every lane of the group now holds the group sum; lane leader adds it
                    const bool leader = (lane & (group - 1)) == 0;
                    if (leader && q < nq) {
#pragma unroll
                        for (int hh = 0; hh < 8; ++hh) hs[hh] += (hh == h) ? gsum : 0.0f;
                    }
                }
            }
        }
        // combine leaders (distinct heads / chunks) through the wave
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            if (h < H) {
                float v = group == kWave ? hs[h] : wave_sum(hs[h]);
                if (lane == 0 && e < kMaxDegCache) sda[e * H + h] = v;
                if (e >= kMaxDegCache && lane == 0) dlogit[(size_t)(beg + e) * H + h] = v;  // temp: dalpha
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // softmax + leaky_relu backward
    if (deg * H <= kWave && deg <= kMaxDegCache && H <= 8) {
        // lanes = (edge, head) pairs, per-head masked wave reductions
        const int e = lane / H, h = lane - (lane / H) * H;
        const bool on = lane < deg * H;
        float da = 0.0f, al = 0.0f, raw = 0.0f;
        if (on) {
            da = sda[lane];  // = sda[e * H + h]
            al = alpha[(size_t)(beg + e) * H + h];
            raw = a_src[(size_t)src[beg + e] * H + h] + a_dst[(size_t)i * H + h] + a_edge[(size_t)(beg + e) * H + h];
        }
        float t = 0.0f;
#pragma unroll
        for (int hh = 0; hh < 8; ++hh)
            if (hh < H) {
                const float th = wave_sum(h == hh ? al * da : 0.0f);
                if (h == hh) t = th;
            }
        const float dl = on ? al * (da - t) * (raw > 0.0f ? 1.0f : slope) : 0.0f;
        if (on) dlogit[(size_t)(beg + e) * H + h] = dl;
#pragma unroll
        for (int hh = 0; hh < 8; ++hh)
            if (hh < H) {
                const float gd = wave_sum(h == hh ? dl : 0.0f);
                if (lane == hh) ga_dst[(size_t)i * H + hh] = gd;
            }
        return;
    }
    for (int h = 0; h < H; ++h) {
        const float ad = a_dst[(size_t)i * H + h];
        float t = 0.0f;
        for (int e0 = 0; e0 < deg; e0 += kWave) {
            int e = e0 + lane;
            float v = 0.0f;
            if (e < deg) {
                float da = e < kMaxDegCache ? sda[e * H + h] : dlogit[(size_t)(beg + e) * H + h];
                v = alpha[(size_t)(beg + e) * H + h] * da;
            }
            t += wave_sum(v);
        }
        float gd = 0.0f;
        for (int e0 = 0; e0 < deg; e0 += kWave) {
            int e = e0 + lane;
            float dl = 0.0f;
            if (e < deg) {
                float da = e < kMaxDegCache ? sda[e * H + h] : dlogit[(size_t)(beg + e) * H + h];
                float raw = a_src[(size_t)src[beg + e] * H + h] + ad + a_edge[(size_t)(beg + e) * H + h];
                dl = alpha[(size_t)(beg + e) * H + h] * (da - t) * (raw > 0.0f ? 1.0f : slope);
                dlogit[(size_t)(beg + e) * H + h] = dl;
            }
            gd += wave_sum(dl);
        }
        if (lane == 0) ga_dst[(size_t)i * H + h] = gd;
    }
}

// ------------------------------------------------------- backward (src)
// CSR by source: sptr[j]..sptr[j+1] lists dst-CSR positions p of j's out-edges.
template <typename T>
__global__ void __launch_bounds__(kWave * kGatWaves)
    gat_bwd_src_kernel(int Nt, int H, int C, const int32_t* __restrict__ sptr, const int32_t* __restrict__ spos,
                       const int32_t* __restrict__ sdst, const float* __restrict__ alpha,
                       const float* __restrict__ dlogit, const float* __restrict__ gout, T* __restrict__ gxh,
                       float* __restrict__ ga_src) {
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    const int j = blockIdx.x * kGatWaves + w;
    if (j >= Nt) return;
    const int HC = H * C;
    const int nq = HC / 4;
    const int beg = sptr[j], deg = sptr[j + 1] - beg;
    float4 acc[kMaxChunks];
#pragma unroll
    for (int k = 0; k < kMaxChunks; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t = 0; t < deg; ++t) {
        const int p = spos[beg + t];
        const int i = sdst[beg + t];
        const float* gr = gout + (size_t)i * HC;
#pragma unroll
        for (int k = 0; k < kMaxChunks; ++k) {
            const int q = lane + kWave * k;
            if (q < nq) {
                const float al = alpha[(size_t)p * H + (4 * q) / C];
                float4 g = *reinterpret_cast<const float4*>(gr + 4 * q);
                acc[k].x += al * g.x;
                acc[k].y += al * g.y;
                acc[k].z += al * g.z;
                acc[k].w += al * g.w;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxChunks; ++k) {
        const int q = lane + kWave * k;
        if (q < nq) store4<T>(gxh + (size_t)j * HC + 4 * q, acc[k]);  // grad in xh's dtype (RNE to bf16)
    }
    for (int h = lane; h < H; h += kWave) {
        float s = 0.0f;
        for (int t = 0; t < deg; ++t) s += dlogit[(size_t)spos[beg + t] * H + h];
        ga_src[(size_t)j * H + h] = s;
    }
}

hipError_t launch_gat_forward(int Nt, int H, int C, const int32_t* rowptr, const int32_t* src, const void* xh,
                              int bf16, const float* a_src, const float* a_dst, const float* a_edge, float slope,
                              const float* bias, float* out, float* alpha, hipStream_t stream) {
    dim3 grid((Nt + kGatWaves - 1) / kGatWaves), block(kWave * kGatWaves);
    if (bf16)
        hipLaunchKernelGGL(gat_fwd_kernel<__hip_bfloat16>, grid, block, 0, stream, Nt, H, C, rowptr, src,
                           static_cast<const __hip_bfloat16*>(xh), a_src, a_dst, a_edge, slope, bias, out, alpha);
    else
        hipLaunchKernelGGL(gat_fwd_kernel<float>, grid, block, 0, stream, Nt, H, C, rowptr, src,
                           static_cast<const float*>(xh), a_src, a_dst, a_edge, slope, bias, out, alpha);
    return hipGetLastError();
}

hipError_t launch_gat_backward(int Nt, int H, int C, const int32_t* rowptr, const int32_t* src, const int32_t* sptr,
                               const int32_t* spos, const int32_t* sdst, const void* xh, int bf16, const float* a_src,
                               const float* a_dst, const float* a_edge, float slope, const float* alpha,
                               const float* gout, void* gxh, float* ga_src, float* ga_dst, float* ga_edge,
                               hipStream_t stream) {
    dim3 grid((Nt + kGatWaves - 1) / kGatWaves), block(kWave * kGatWaves);
    if (bf16)
        hipLaunchKernelGGL(gat_bwd_dst_kernel<__hip_bfloat16>, grid, block, 0, stream, Nt, H, C, rowptr, src,
                           static_cast<const __hip_bfloat16*>(xh), a_src, a_dst, a_edge, slope, alpha, gout, ga_edge,
                           ga_dst);
    else
        hipLaunchKernelGGL(gat_bwd_dst_kernel<float>, grid, block, 0, stream, Nt, H, C, rowptr, src,
                           static_cast<const float*>(xh), a_src, a_dst, a_edge, slope, alpha, gout, ga_edge, ga_dst);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (bf16)
        hipLaunchKernelGGL(gat_bwd_src_kernel<__hip_bfloat16>, grid, block, 0, stream, Nt, H, C, sptr, spos, sdst,
                           alpha, ga_edge, gout, static_cast<__hip_bfloat16*>(gxh), ga_src);
    else
        hipLaunchKernelGGL(gat_bwd_src_kernel<float>, grid, block, 0, stream, Nt, H, C, sptr, spos, sdst, alpha,
                           ga_edge, gout, static_cast<float*>(gxh), ga_src);
    return hipGetLastError();
}

}  // namespace trx

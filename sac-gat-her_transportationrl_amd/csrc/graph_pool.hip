// graph_pool.hip -- global mean | max pooling of GATEncoder (src/models/
// gat_encoder.py:50-52, PyG global_mean_pool / global_max_pool + cat) for a
// regular batch (graph b owns nodes [b*n, (b+1)*n)), training path.
// Forward: one thread per (graph, feature) -> out [B, 2F] = mean | max, the
// max and its tie count kept for the backward.  Backward: one thread per
// (node, feature): g_mean / n + (x == max ? g_max / ties : 0) -- torch's
// amax backward spreads the gradient evenly over ties.  Replaces ~3 forward
// and ~7 backward torch launches per encoder.
// Also here: trx_bf16_round, the multi-tensor bf16 rounding of the small
// weight blocks the fused inference passes read (one launch per pass).
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

__global__ void __launch_bounds__(256) graph_pool_fwd_kernel(int B, int n, int F, const float* __restrict__ x,
                                                             float* __restrict__ out, float* __restrict__ ties) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= B * F) return;
    const int b = idx / F, f = idx - b * F;
    const float* col = x + (size_t)b * n * F + f;
    float s = 0.0f, mx = -__builtin_huge_valf();
    for (int i = 0; i < n; ++i) {
        const float v = col[(size_t)i * F];
        s += v;
        mx = fmaxf(mx, v);
    }
    float cnt = 0.0f;
    for (int i = 0; i < n; ++i) cnt += col[(size_t)i * F] == mx ? 1.0f : 0.0f;
    out[(size_t)b * 2 * F + f] = s / (float)n;
    out[(size_t)b * 2 * F + F + f] = mx;
    ties[idx] = cnt;
}

__global__ void __launch_bounds__(256) graph_pool_bwd_kernel(int B, int n, int F, const float* __restrict__ x,
                                                             const float* __restrict__ out,
                                                             const float* __restrict__ ties,
                                                             const float* __restrict__ g, float* __restrict__ gx) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)B * n * F) return;
    const int f = (int)(idx % F);
    const int b = (int)(idx / ((size_t)n * F));
    const float gm = g[(size_t)b * 2 * F + f] / (float)n;
    const float mx = out[(size_t)b * 2 * F + F + f];
    gx[idx] = gm + (x[idx] == mx ? g[(size_t)b * 2 * F + F + f] / ties[(size_t)b * F + f] : 0.0f);
}

}  // namespace

hipError_t launch_graph_pool_fwd(int B, int n, int F, const float* x, float* out, float* ties, hipStream_t stream) {
    hipLaunchKernelGGL(graph_pool_fwd_kernel, dim3((B * F + 255) / 256), dim3(256), 0, stream, B, n, F, x, out, ties);
    return hipGetLastError();
}

hipError_t launch_graph_pool_bwd(int B, int n, int F, const float* x, const float* out, const float* ties,
                                 const float* g, float* gx, hipStream_t stream) {
    const size_t total = (size_t)B * n * F;
    hipLaunchKernelGGL(graph_pool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, B, n, F, x,
                       out, ties, g, gx);
    return hipGetLastError();
}

}  // namespace trx

// ------------------------------------------------------------------------
// Multi-tensor bf16 rounding (trx_bf16_round): the fused inference passes
// need bf16 copies (or bf16-rounded float32 copies) of ~10 small weight
// blocks per pass; one launch for all of them instead of one or two each.
namespace trx {
namespace {
__global__ void __launch_bounds__(256) bf16_round_kernel(trx_round_list l) {
    const int k = blockIdx.y;
    if (k >= l.count) return;
    // 32-bit index arithmetic (every tensor < 2^31 elements, checked at launch);
    // four consecutive elements of one row per thread when the row length allows
    const uint32_t cols = (uint32_t)l.cols[k], n = (uint32_t)(l.rows[k] * l.cols[k]);
    const float* src = l.src[k];
    const int64_t ss = l.src_stride[k];
    const uint32_t ds = l.dst_stride[k] > 0 ? (uint32_t)l.dst_stride[k] : cols;  // dst row stride (elements)
    // 0 bf16-rounded float32, 1 bf16 bits, 2 exact float32 copy, 3 bf16 bits of the
    // remainder x - bf16(x) (the low half of a two-term bf16 split); 16 + bits: the
    // three pieces of a split operand from one read of x (piece p = the remainder
    // when bit p is set, else bf16(x)), pieces `poff` elements apart
    const int mode = l.out_bf16[k];
    const bool bf = mode == 1 || mode == 3;
    auto lo = [](float x, __bf16 h) -> __bf16 { return (__bf16)(x - (float)h); };
    const uint32_t step = gridDim.x * 256u;
    auto pk = [](__bf16 a, __bf16 b) -> uint32_t {
        return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
    };
    if (mode >= 16) {
        const uint32_t poff = l.dst_stride[k] > 0 ? cols : n;
        uint16_t* dst = static_cast<uint16_t*>(l.dst[k]);
        if ((cols & 3u) == 0 && (ss & 3) == 0 && (ds & 3u) == 0 && (poff & 3u) == 0 && ((uintptr_t)src & 15) == 0 &&
            ((uintptr_t)dst & 7) == 0) {
            for (uint32_t q = blockIdx.x * 256u + threadIdx.x; 4 * q < n; q += step) {
                const uint32_t i0 = 4 * q, r = i0 / cols, c = i0 - r * cols, i = r * ds + c;
                const float4 v = *reinterpret_cast<const float4*>(src + r * ss + c);
                const __bf16 h0 = (__bf16)v.x, h1 = (__bf16)v.y, h2 = (__bf16)v.z, h3 = (__bf16)v.w;
                uint2 uh, ul;
                uh.x = pk(h0, h1);
                uh.y = pk(h2, h3);
                ul.x = pk(lo(v.x, h0), lo(v.y, h1));
                ul.y = pk(lo(v.z, h2), lo(v.w, h3));
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    *reinterpret_cast<uint2*>(dst + i + p * poff) = (mode >> p) & 1 ? ul : uh;
            }
            return;
        }
        for (uint32_t i0 = blockIdx.x * 256u + threadIdx.x; i0 < n; i0 += step) {
            const uint32_t r = i0 / cols, c = i0 - r * cols, i = r * ds + c;
            const float x = src[r * ss + c];
            const __bf16 h = (__bf16)x, w = lo(x, h);
#pragma unroll
            for (int p = 0; p < 3; ++p) dst[i + p * poff] = __builtin_bit_cast(uint16_t, (mode >> p) & 1 ? w : h);
        }
        return;
    }
    if ((cols & 3u) == 0 && (ss & 3) == 0 && (ds & 3u) == 0 && ((uintptr_t)src & 15) == 0 &&
        ((uintptr_t)l.dst[k] & 15) == 0) {
        for (uint32_t q = blockIdx.x * 256u + threadIdx.x; 4 * q < n; q += step) {
            const uint32_t i0 = 4 * q, r = i0 / cols, c = i0 - r * cols;
            const uint32_t i = r * ds + c;  // destination element
            const float4 v = *reinterpret_cast<const float4*>(src + r * ss + c);
            __bf16 h0 = (__bf16)v.x, h1 = (__bf16)v.y, h2 = (__bf16)v.z, h3 = (__bf16)v.w;
            if (mode == 3) {
                h0 = lo(v.x, h0);
                h1 = lo(v.y, h1);
                h2 = lo(v.z, h2);
                h3 = lo(v.w, h3);
            }
            if (bf) {
                uint2 u;
                u.x = pk(h0, h1);
                u.y = pk(h2, h3);
                *reinterpret_cast<uint2*>(static_cast<uint16_t*>(l.dst[k]) + i) = u;
            } else if (mode == 2) {
                *reinterpret_cast<float4*>(static_cast<float*>(l.dst[k]) + i) = v;
            } else {
                *reinterpret_cast<float4*>(static_cast<float*>(l.dst[k]) + i) =
                    make_float4((float)h0, (float)h1, (float)h2, (float)h3);
            }
        }
        return;
    }
    for (uint32_t i0 = blockIdx.x * 256u + threadIdx.x; i0 < n; i0 += step) {
        const uint32_t r = i0 / cols, c = i0 - r * cols, i = r * ds + c;
        const float x = src[r * ss + c];
        const __bf16 h = mode == 3 ? lo(x, (__bf16)x) : (__bf16)x;
        if (bf)
            static_cast<uint16_t*>(l.dst[k])[i] = __builtin_bit_cast(uint16_t, h);
        else
            static_cast<float*>(l.dst[k])[i] = mode == 2 ? x : (float)h;
    }
}
}  // namespace

hipError_t launch_bf16_round(const trx_round_list& l, hipStream_t stream) {
    int64_t mx = 1;
    for (int k = 0; k < l.count; ++k) {
        const int64_t n = l.rows[k] * l.cols[k];
        if ((l.out_bf16[k] >= 16 ? 3 * n : n) >= ((int64_t)1 << 31) || l.rows[k] * l.src_stride[k] >= ((int64_t)1 << 31) ||
            l.rows[k] * l.dst_stride[k] >= ((int64_t)1 << 31))
            return hipErrorInvalidValue;
        mx = n > mx ? n : mx;
    }
    const int64_t blocks = (mx + 1023) / 1024;  // ~4 elements per thread
    const unsigned bx = (unsigned)(blocks < 1024 ? blocks : 1024);
    hipLaunchKernelGGL(bf16_round_kernel, dim3(bx, l.count), dim3(256), 0, stream, l);
    return hipGetLastError();
}
}  // namespace trx

// ------------------------------------------------------------------------
// Multi-buffer device copy (trx_multi_copy): the trainer writes ~13 fields of
// every step's transitions into the replay ring; one launch instead of one
// memcpy / index_copy each.
namespace trx {
namespace {
__global__ void __launch_bounds__(256) multi_copy_kernel(trx_copy_list l) {
    const int k = blockIdx.y;
    if (k >= l.count) return;
    const char* src = static_cast<const char*>(l.src[k]);
    char* dst = static_cast<char*>(l.dst[k]);
    const int64_t nb = l.bytes[k];
    const int64_t stride = (int64_t)gridDim.x * 256;
    if ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)nb) & 15) == 0) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nb / 16; i += stride) d4[i] = s4[i];
    } else {
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += stride) dst[i] = src[i];
    }
}

// Row gather (trx_multi_gather): dst[k] row r = src[k] row idx[r], rows of
// l.bytes[k] bytes -- the replay sample's ~13 index_selects in one launch.
__global__ void __launch_bounds__(256) multi_gather_kernel(trx_copy_list l, const int64_t* __restrict__ idx) {
    const int k = blockIdx.y;
    if (k >= l.count) return;
    const int64_t rb = l.bytes[k], r = blockIdx.x, sr = idx[r];
    const char* src = static_cast<const char*>(l.src[k]) + sr * rb;
    char* dst = static_cast<char*>(l.dst[k]) + r * rb;
    if ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)rb) & 15) == 0) {
        for (int64_t i = threadIdx.x; i < rb / 16; i += 256)
            reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    } else if ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)rb) & 3) == 0) {
        for (int64_t i = threadIdx.x; i < rb / 4; i += 256)
            reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(src)[i];
    } else {
        for (int64_t i = threadIdx.x; i < rb; i += 256) dst[i] = src[i];
    }
}
}  // namespace

hipError_t launch_multi_gather(const trx_copy_list& l, const int64_t* idx, int nrows, hipStream_t stream) {
    if (nrows <= 0 || l.count <= 0) return hipSuccess;
    hipLaunchKernelGGL(multi_gather_kernel, dim3(nrows, l.count), dim3(256), 0, stream, l, idx);
    return hipGetLastError();
}

hipError_t launch_multi_copy(const trx_copy_list& l, hipStream_t stream) {
    int64_t mx = 16;
    for (int k = 0; k < l.count; ++k) mx = l.bytes[k] > mx ? l.bytes[k] : mx;
    const int64_t blocks = (mx / 16 + 255) / 256;
    const unsigned bx = (unsigned)(blocks < 512 ? (blocks > 0 ? blocks : 1) : 512);
    hipLaunchKernelGGL(multi_copy_kernel, dim3(bx, l.count), dim3(256), 0, stream, l);
    return hipGetLastError();
}
// ------------------------------------------------------------------------
// Per-step episode bookkeeping of the vectorised trainer (src/train.py:916-935:
// reward scaling, episode reward / TSTT sum / AUC, truncation) for all B envs
// in one launch instead of ~12 elementwise torch ops; float64 like the
// reference's Python floats, in the same operation order.
namespace {
__global__ void episode_step_kernel(int B, const double* __restrict__ reward, const uint8_t* __restrict__ done,
                                    const double* __restrict__ tstt, double reward_scale, int64_t max_steps,
                                    double* __restrict__ scaled, float* __restrict__ scaled_f32,
                                    float* __restrict__ done_f32, double* __restrict__ ep_reward,
                                    double* __restrict__ ep_tstt_sum, double* __restrict__ ep_auc,
                                    double* __restrict__ ep_prev_tstt, int64_t* __restrict__ ep_len,
                                    uint8_t* __restrict__ finished) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int64_t ln = ep_len[b] + 1;
    ep_len[b] = ln;
    const double sv = reward[b] * reward_scale;
    scaled[b] = sv;
    scaled_f32[b] = (float)sv;
    done_f32[b] = done[b] ? 1.0f : 0.0f;
    ep_reward[b] = ep_reward[b] + sv;
    const double t = tstt[b];
    ep_tstt_sum[b] = ep_tstt_sum[b] + t;
    ep_auc[b] = ep_auc[b] + (0.5 * (ep_prev_tstt[b] + t)) * (ln > 1 ? 1.0 : 0.0);
    ep_prev_tstt[b] = t;
    finished[b] = (done[b] != 0 || (max_steps > 0 && ln >= max_steps)) ? 1 : 0;
}
}  // namespace

hipError_t launch_episode_step(int B, const double* reward, const uint8_t* done, const double* tstt,
                               double reward_scale, int64_t max_steps, double* scaled, float* scaled_f32,
                               float* done_f32, double* ep_reward, double* ep_tstt_sum, double* ep_auc,
                               double* ep_prev_tstt, int64_t* ep_len, uint8_t* finished, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(episode_step_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, B, reward, done, tstt,
                       reward_scale, max_steps, scaled, scaled_f32, done_f32, ep_reward, ep_tstt_sum, ep_auc,
                       ep_prev_tstt, ep_len, finished);
    return hipGetLastError();
}
}  // namespace trx

// small_ln.hip -- LayerNorm over the 4-/6-wide raw node / link features of
// Actor and Critic (src/rl/sac.py:27-28, 36-37: nn.LayerNorm(node_in / edge_in)) in
// the training (autograd) path.  torch runs such narrow rows either with one
// workgroup per row (nn.LayerNorm) or as ~8 elementwise/reduction launches
// forward and ~12 backward (the vectorised form in rl/sac.py); here one
// thread per row each way.  Backward column sums (weight, bias) are reduced
// per workgroup (DPP wave sums, then the 4 waves in order) into partials and
// summed over workgroups by one more launch in a fixed order.
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kWave = 64;
constexpr int kLnThreads = 256;
constexpr int kLnMax = 8;

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

__global__ void __launch_bounds__(kLnThreads) small_ln_fwd_kernel(int N, int d, const float* __restrict__ x,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b, float eps,
                                                                  float* __restrict__ y, float* __restrict__ stats) {
    const int i = blockIdx.x * kLnThreads + threadIdx.x;
    if (i >= N) return;
    float v[kLnMax];
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < kLnMax; ++j) {
        v[j] = j < d ? x[(size_t)i * d + j] : 0.0f;
        if (j < d) s += v[j];
    }
    const float mu = s / (float)d;
    float s2 = 0.0f;
#pragma unroll
    for (int j = 0; j < kLnMax; ++j)
        if (j < d) {
            const float t = v[j] - mu;
            s2 += t * t;
        }
    const float r = rsqrtf(s2 / (float)d + eps);
#pragma unroll
    for (int j = 0; j < kLnMax; ++j)
        if (j < d) y[(size_t)i * d + j] = (v[j] - mu) * r * w[j] + b[j];
    stats[2 * i] = mu;
    stats[2 * i + 1] = r;
}

__global__ void __launch_bounds__(kLnThreads) small_ln_bwd_kernel(int N, int d, const float* __restrict__ gy,
                                                                  const float* __restrict__ x,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ stats,
                                                                  float* __restrict__ gx, float* __restrict__ part) {
    __shared__ float red[kLnThreads / kWave][2 * kLnMax];
    const int i = blockIdx.x * kLnThreads + threadIdx.x;
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    float gw[kLnMax], gb[kLnMax];
#pragma unroll
    for (int j = 0; j < kLnMax; ++j) gw[j] = gb[j] = 0.0f;
    if (i < N) {
        const float mu = stats[2 * i], r = stats[2 * i + 1];
        float xh[kLnMax], dxh[kLnMax];
        float m1 = 0.0f, m2 = 0.0f;
#pragma unroll
        for (int j = 0; j < kLnMax; ++j) {
            xh[j] = dxh[j] = 0.0f;
            if (j < d) {
                const float g = gy[(size_t)i * d + j];
                xh[j] = (x[(size_t)i * d + j] - mu) * r;
                dxh[j] = g * w[j];
                m1 += dxh[j];
                m2 += dxh[j] * xh[j];
                gw[j] = g * xh[j];
                gb[j] = g;
            }
        }
        m1 /= (float)d;
        m2 /= (float)d;
#pragma unroll
        for (int j = 0; j < kLnMax; ++j)
            if (j < d) gx[(size_t)i * d + j] = r * (dxh[j] - m1 - xh[j] * m2);
    }
#pragma unroll
    for (int j = 0; j < kLnMax; ++j)
        if (j < d) {
            const float a = wave_sum(gw[j]), c = wave_sum(gb[j]);
            if (lane == 0) {
                red[wv][j] = a;
                red[wv][kLnMax + j] = c;
            }
        }
    __syncthreads();
    if (threadIdx.x < 2 * d) {
        const int t = threadIdx.x / d, j = threadIdx.x - t * d;
        float v = 0.0f;
#pragma unroll
        for (int ww = 0; ww < kLnThreads / kWave; ++ww) v += red[ww][t * kLnMax + j];
        part[(size_t)blockIdx.x * 2 * d + threadIdx.x] = v;
    }
}

// gwb[idx] = sum over workgroups of part[blk][idx] (idx < 2d): one wave per output
__global__ void __launch_bounds__(kWave) small_ln_reduce_kernel(int nblk, int n_out, const float* __restrict__ part,
                                                                float* __restrict__ gwb) {
    const int idx = blockIdx.x, lane = threadIdx.x;
    float v = 0.0f;
    for (int blk = lane; blk < nblk; blk += kWave) v += part[(size_t)blk * n_out + idx];
    v = wave_sum(v);
    if (lane == 0) gwb[idx] = v;
}

}  // namespace

int small_ln_blocks(int N) { return (N + kLnThreads - 1) / kLnThreads; }

hipError_t launch_small_ln_fwd(int N, int d, const float* x, const float* w, const float* b, float eps, float* y,
                               float* stats, hipStream_t stream) {
    hipLaunchKernelGGL(small_ln_fwd_kernel, dim3(small_ln_blocks(N)), dim3(kLnThreads), 0, stream, N, d, x, w, b, eps,
                       y, stats);
    return hipGetLastError();
}

hipError_t launch_small_ln_bwd(int N, int d, const float* gy, const float* x, const float* w, const float* stats,
                               float* gx, float* gwb, float* part, hipStream_t stream) {
    const int nblk = small_ln_blocks(N);
    hipLaunchKernelGGL(small_ln_bwd_kernel, dim3(nblk), dim3(kLnThreads), 0, stream, N, d, gy, x, w, stats, gx, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(small_ln_reduce_kernel, dim3(2 * d), dim3(kWave), 0, stream, nblk, 2 * d, part, gwb);
    return hipGetLastError();
}

}  // namespace trx

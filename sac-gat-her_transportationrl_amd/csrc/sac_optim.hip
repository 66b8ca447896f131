// sac_optim.hip -- DiscreteSAC.apply_gradients as three launches, gfx950.
//
// The reference steps three torch.optim.Adam optimizers after clipping each
// one's gradients (src/rl/sac.py:224-240: clip_grad_norm_ + critic_opt.step,
// actor_opt.step, alpha_opt.step), clamps log_alpha and Polyak-averages the
// target critics (263, 288-291).  Through torch that is ~40 launches per
// update (per-tensor norms, stack, norm of norms, foreach scaling, three fused
// Adam multi-tensor launches, foreach Polyak mul/mul/add, clamps).  Here the
// gradients already sit in one flat buffer (the fused update writes every
// parameter gradient into it, for the data-parallel all-reduce), so:
//   1. adam_norm_kernel    per-chunk sums of squares of the gradients
//                          (fixed in-block order), step counts + 1;
//   2. adam_scal_kernel    per optimizer group: total norm in a fixed order,
//                          clip coefficient min(max_norm / (norm + 1e-6), 1),
//                          Adam step size lr / (1 - beta1^t) and
//                          sqrt(1 - beta2^t);
//   3. adam_apply_kernel   per element: g * coef, the Adam moments and
//                          parameter update (torch's fused Adam expression
//                          order), the log_alpha clamps, and for the critics
//                          the Polyak update of the matching target element
//                          (t * (1 - tau) + p * tau, rounded like the foreach
//                          ops) -- the target reads the parameter just written.
// Chunks never straddle a parameter tensor (host-built table), so every
// block knows its tensor, group and target without a search.
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "trx_internal.h"

namespace trx {
namespace {

constexpr int kAT = 256;

__global__ void __launch_bounds__(kAT) adam_norm_kernel(trx_adam_args a) {
    __shared__ float red[kAT];
    const int b = blockIdx.x, tid = threadIdx.x;
    const trx_adam_block blk = a.blocks[b];
    const trx_adam_seg sg = a.segs[blk.seg];
    const float* __restrict__ g = a.g_base + sg.goff;
    float s = 0.0f;
    // unrolled: the loads of eight strided elements in flight, the sum in element order
#pragma unroll 8
    for (int i = blk.begin + tid; i < blk.end; i += kAT) {
        const float v = g[i];
        s += v * v;
    }
    red[tid] = s;
    __syncthreads();
    for (int w = kAT / 2; w > 0; w >>= 1) {  // fixed tree order: deterministic
        if (tid < w) red[tid] += red[tid + w];
        __syncthreads();
    }
    if (tid == 0) a.partial[b] = red[0];
    if (b == 0 && tid < 3) a.step[tid] += 1.0f;
}

__global__ void __launch_bounds__(kAT) adam_scal_kernel(trx_adam_args a) {
    const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
    if (grp >= 3) return;
    float s = 0.0f;  // lane-strided over the chunks of this group, then a fixed shuffle tree
    for (int b = lane; b < a.nblocks; b += 64)
        if (a.segs[a.blocks[b].seg].group == grp) s += a.partial[b];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if (lane == 0) {
        const float norm = sqrtf(s);
        float coef = 1.0f;
        if (a.max_norm[grp] > 0.0f) {
            coef = a.max_norm[grp] / (norm + 1e-6f);
            coef = coef < 1.0f ? coef : 1.0f;
        }
        const double t = (double)a.step[grp];
        a.scal[4 * grp + 0] = coef;
        a.scal[4 * grp + 1] = (float)((double)a.lr[grp] / (1.0 - pow((double)a.beta1, t)));
        a.scal[4 * grp + 2] = (float)sqrt(1.0 - pow((double)a.beta2, t));
        a.scal[4 * grp + 3] = norm;
    }
}

__global__ void __launch_bounds__(kAT) adam_apply_kernel(trx_adam_args a) {
    const int b = blockIdx.x, tid = threadIdx.x;
    const trx_adam_block blk = a.blocks[b];
    const trx_adam_seg sg = a.segs[blk.seg];
    const int grp = sg.group;
    const float coef = a.scal[4 * grp], step_size = a.scal[4 * grp + 1], bc2s = a.scal[4 * grp + 2];
    const float b1 = a.beta1, b2 = a.beta2, eps = a.eps;
    const float omb1 = 1.0f - b1, omb2 = 1.0f - b2, tau = a.tau, omt = 1.0f - a.tau;
    // four strided elements per round: every load of the round issued before its
    // arithmetic and stores (the element's own expression order is unchanged).
    // Out-of-range slots load a valid element (clamped index) and store nothing:
    // no per-element branch around a load.
    const float* g = a.g_base + sg.goff;
    float* m = a.m + sg.moff;
    float* v = a.v + sg.moff;
    float* pp = sg.p;
    float* tt = sg.t;
    constexpr int U = 4;
    auto rounds = [&](auto has_t) {
        constexpr bool HT = decltype(has_t)::value;
        for (int i0 = blk.begin + tid; i0 < blk.end; i0 += U * kAT) {
            float gv[U], mv[U], vv[U], pv[U], tv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + u * kAT < blk.end ? i0 + u * kAT : i0;
                gv[u] = g[i];
                mv[u] = m[i];
                vv[u] = v[i];
                pv[u] = pp[i];
                if constexpr (HT) tv[u] = tt[i];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + u * kAT;
                const float gi = gv[u] * coef;
                const float mi = b1 * mv[u] + omb1 * gi;
                const float vi = b2 * vv[u] + omb2 * gi * gi;
                const float denom = sqrtf(vi) / bc2s + eps;
                float p = pv[u] - step_size * mi / denom;
                if (grp == 2) {  // log_alpha clamps (sac.py:241-246)
                    p = p < a.log_alpha_max ? p : a.log_alpha_max;
                    p = p > a.log_alpha_min ? p : a.log_alpha_min;
                }
                if (i < blk.end) {
                    m[i] = mi;
                    v[i] = vi;
                    pp[i] = p;
                    if constexpr (HT) tt[i] = tv[u] * omt + p * tau;  // Polyak (288-291)
                }
            }
        }
    };
    if (tt)
        rounds(std::true_type{});
    else
        rounds(std::false_type{});
}

}  // namespace

hipError_t launch_sac_adam(const trx_adam_args& a, hipStream_t stream) {
    hipLaunchKernelGGL(adam_norm_kernel, dim3(a.nblocks), dim3(kAT), 0, stream, a);
    hipLaunchKernelGGL(adam_scal_kernel, dim3(1), dim3(kAT), 0, stream, a);
    hipLaunchKernelGGL(adam_apply_kernel, dim3(a.nblocks), dim3(kAT), 0, stream, a);
    return hipGetLastError();
}

}  // namespace trx

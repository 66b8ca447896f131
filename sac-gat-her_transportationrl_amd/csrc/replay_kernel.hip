// replay_kernel.hip -- prioritized-replay sum tree on the GPU.
//
// Replaces the Python sum-tree of src/train.py:27-91 (ReplayBuffer._set_priority,
// sample).  Same array layout: tree[1] is the root, leaves are
// tree[capacity + i], children of k are 2k and 2k+1 (also for a capacity that
// is not a power of two, exactly like the reference).  Differences: the tree is
// float64 and an update recomputes each touched ancestor as the sum of its
// two children (the reference propagates float32 deltas), so sums do not drift.
//
//   trx_per_update: leaves idx[k] <- priority[k] (caller dedups: last wins),
//                   then every ancestor of a touched leaf is recomputed level
//                   by level inside ONE workgroup (a __syncthreads per level).
//   trx_per_sample: per draw k: r = u[k] * tree[1]; descend with the
//                   reference's rule `if r <= tree[left]: go left else r -=
//                   tree[left]; go right` (train.py:67-79).
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {

__global__ void __launch_bounds__(1024) per_update_kernel(double* __restrict__ tree, int64_t capacity,
                                                          const int64_t* __restrict__ idx,
                                                          const double* __restrict__ pri, int n) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) tree[capacity + idx[k]] = pri[k];
    __syncthreads();
    // depth: number of halvings until the root for the deepest leaf index
    int64_t top = 2 * capacity - 1;
    int levels = 0;
    while ((top >> levels) > 1) ++levels;
    for (int l = 1; l <= levels; ++l) {
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            int64_t node = (capacity + idx[k]) >> l;
            if (node >= 1) {
                int64_t a = 2 * node, b = 2 * node + 1;
                double va = a < 2 * capacity ? tree[a] : 0.0;
                double vb = b < 2 * capacity ? tree[b] : 0.0;
                tree[node] = va + vb;  // idempotent: concurrent writers store the same value
            }
        }
        __threadfence_block();
        __syncthreads();
    }
}

// Contiguous leaf range [lo, lo + n) (ring-buffer adds): the ancestors touched at
// level l are exactly the contiguous range ((capacity + lo) >> l, (capacity + lo + n
// - 1) >> l), so each level recomputes its distinct nodes once -- the same node
// updates, in the same level order, as per_update_kernel, without its per-leaf
// redundancy (n / 2^l nodes at level l instead of n).
// max_priority != NULL: the ring add itself (src/train.py:50-58 applied n times):
// leaf k = (max_p + eps * (k + 1)) ** alpha, then max_p += ... (written last).
__global__ void __launch_bounds__(1024) per_update_range_kernel(double* __restrict__ tree, int64_t capacity,
                                                                int64_t lo, const double* __restrict__ pri, int n,
                                                                double* __restrict__ max_priority, double eps,
                                                                double alpha) {
    if (max_priority) {
        const double mp = *max_priority;
        for (int k = threadIdx.x; k < n; k += blockDim.x) tree[capacity + lo + k] = pow(mp + eps * (double)(k + 1), alpha);
        __syncthreads();
        if (threadIdx.x == 0) *max_priority = mp + eps * (double)n;
    } else {
        for (int k = threadIdx.x; k < n; k += blockDim.x) tree[capacity + lo + k] = pri[k];
    }
    __syncthreads();
    int64_t top = 2 * capacity - 1;
    int levels = 0;
    while ((top >> levels) > 1) ++levels;
    for (int l = 1; l <= levels; ++l) {
        const int64_t a = (capacity + lo) >> l, b = (capacity + lo + n - 1) >> l;
        for (int64_t node = a + threadIdx.x; node <= b; node += blockDim.x) {
            if (node >= 1) {
                const int64_t c0 = 2 * node, c1 = 2 * node + 1;
                const double va = c0 < 2 * capacity ? tree[c0] : 0.0;
                const double vb = c1 < 2 * capacity ? tree[c1] : 0.0;
                tree[node] = va + vb;
            }
        }
        __threadfence_block();
        __syncthreads();
    }
}

__global__ void per_sample_kernel(const double* __restrict__ tree, int64_t capacity, const double* __restrict__ u,
                                  int n, int64_t* __restrict__ out_idx, double* __restrict__ out_pri) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    double r = u[k] * tree[1];
    int64_t node = 1;
    while (node < capacity) {
        int64_t left = 2 * node;
        double tl = left < 2 * capacity ? tree[left] : 0.0;
        if (r <= tl) {
            node = left;
        } else {
            r -= tl;
            node = left + 1;
        }
    }
    out_idx[k] = node - capacity;
    out_pri[k] = node < 2 * capacity ? tree[node] : 0.0;
}

hipError_t launch_per_update(double* tree, int64_t capacity, const int64_t* idx, const double* pri, int n,
                             hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(per_update_kernel, dim3(1), dim3(1024), 0, stream, tree, capacity, idx, pri, n);
    return hipGetLastError();
}

hipError_t launch_per_update_range(double* tree, int64_t capacity, int64_t lo, const double* pri, int n,
                                   hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(per_update_range_kernel, dim3(1), dim3(1024), 0, stream, tree, capacity, lo, pri, n,
                       static_cast<double*>(nullptr), 0.0, 0.0);
    return hipGetLastError();
}

hipError_t launch_per_add_range(double* tree, int64_t capacity, int64_t lo, int n, double* max_priority, double eps,
                                double alpha, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(per_update_range_kernel, dim3(1), dim3(1024), 0, stream, tree, capacity, lo,
                       static_cast<const double*>(nullptr), n, max_priority, eps, alpha);
    return hipGetLastError();
}

hipError_t launch_per_sample(const double* tree, int64_t capacity, const double* u, int n, int64_t* out_idx,
                             double* out_pri, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(per_sample_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, tree, capacity, u, n, out_idx,
                       out_pri);
    return hipGetLastError();
}

}  // namespace trx

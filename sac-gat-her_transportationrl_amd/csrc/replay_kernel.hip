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

// ---------------------------------------------------------------- float32 tree
// The reference's own sum tree, bit for bit (src/train.py:27-91 under numpy 2
// / NEP 50 scalar rules): tree float32; _set_priority adds the float32 delta
// fl32(p) - leaf to the leaf and to every ancestor in turn (train.py:43-48), so
// each node accumulates its subtree's deltas sequentially, in update order.
// A parallel restatement has to keep that order per node: every touched node is
// owned by one thread that walks the deltas of the leaves below it in update
// order.  max_priority stays a float64 accumulated sequentially (train.py:52-54).
//
// Leaves of a capacity that is not a power of two sit at two depths: leaf t in
// [capacity, 2 capacity) has bit length d1 = bitlen(capacity) or d2 =
// bitlen(2 capacity - 1); the ancestor of t with bit length b is t >> (bitlen(t) - b).

__device__ __forceinline__ int bitlen64(int64_t x) { return 64 - __clzll((unsigned long long)x); }

constexpr int kPer32Chunk = 2048;   // ring-add leaves per pass (deltas staged in LDS)
constexpr int kPer32MaxUpd = 2048;  // update_priorities entries per launch

// Node m (internal, bit length b) += deltas of the leaves t in [T0, T1) below it,
// in t order (depth d1 leaves precede depth d2 leaves in t, and t order is
// update order for a ring add).
__device__ __forceinline__ float per32_node_sum(float acc, int64_t m, int b, int64_t T0, int64_t T1, int d1, int d2,
                                                const float* __restrict__ sdelta) {
    for (int d = d1; d <= d2; ++d) {
        if (d <= b) continue;
        const int s = d - b;
        int64_t lo = m << s, hi = ((m + 1) << s) - 1;
        if (lo < T0) lo = T0;
        if (hi > T1 - 1) hi = T1 - 1;
        int64_t t = lo;
        for (; t + 3 <= hi; t += 4) {   // order kept: ((acc + a) + b) + c ...
            const float a0 = sdelta[t - T0], a1 = sdelta[t + 1 - T0], a2 = sdelta[t + 2 - T0], a3 = sdelta[t + 3 - T0];
            acc = acc + a0;
            acc = acc + a1;
            acc = acc + a2;
            acc = acc + a3;
        }
        for (; t <= hi; ++t) acc = acc + sdelta[t - T0];
    }
    return acc;
}

// n sequential ReplayBuffer.add(item) calls at ring slots lo .. lo+n-1
// (lo + n <= capacity): priority_k = max_p_{k-1} + eps, max_p_k = priority_k,
// leaf += fl32(priority_k ** alpha) - leaf, ancestors += the same delta.
__global__ void __launch_bounds__(1024) per32_add_range_kernel(float* __restrict__ tree, int64_t capacity, int64_t lo,
                                                               int n, double* __restrict__ max_priority, double eps,
                                                               double alpha) {
    __shared__ double smp[kPer32Chunk];
    __shared__ float sdelta[kPer32Chunk];
    __shared__ double s_mp;
    if (threadIdx.x == 0) s_mp = *max_priority;
    const int d1 = bitlen64(capacity), d2 = bitlen64(2 * capacity - 1);
    for (int c0 = 0; c0 < n; c0 += kPer32Chunk) {
        const int cn = min(kPer32Chunk, n - c0);
        __syncthreads();
        if (threadIdx.x == 0) {   // the float64 running max_priority: sequential, as in the reference
            double m = s_mp;
            for (int k = 0; k < cn; ++k) {
                m = m + eps;
                smp[k] = m;
            }
            s_mp = m;
        }
        __syncthreads();
        const int64_t T0 = capacity + lo + c0, T1 = T0 + cn;
        for (int k = threadIdx.x; k < cn; k += blockDim.x) {
            const float p32 = (float)pow(smp[k], alpha);
            const float old = tree[T0 + k];
            const float d = p32 - old;
            sdelta[k] = d;
            tree[T0 + k] = old + d;
        }
        __syncthreads();
        // internal ancestors, bit length 1 .. d2-1; each node owned by one thread
        for (int b = 1; b < d2; ++b) {
            // ancestors of the depth-d1 leaves [T0, min(T1, 2^d1)) and of the depth-d2
            // leaves [max(T0, 2^d1), T1) (d2 > d1 only)
            const int64_t split = (int64_t)1 << d1;
            int64_t a1 = 1, z1 = 0, a2 = 1, z2 = 0;   // empty ranges
            if (d1 > b && T0 < split) {
                a1 = T0 >> (d1 - b);
                z1 = (min(T1, split) - 1) >> (d1 - b);
            }
            if (d2 > d1 && d2 > b && T1 > split) {
                a2 = max(T0, split) >> (d2 - b);
                z2 = (T1 - 1) >> (d2 - b);
            }
            const int64_t c1 = z1 >= a1 ? z1 - a1 + 1 : 0, c2 = z2 >= a2 ? z2 - a2 + 1 : 0;
            for (int64_t j = threadIdx.x; j < c1 + c2; j += blockDim.x) {
                const int64_t m = j < c1 ? a1 + j : a2 + (j - c1);
                if (j >= c1 && m >= a1 && m <= z1) continue;   // owned through the first range
                tree[m] = per32_node_sum(tree[m], m, b, T0, T1, d1, d2, sdelta);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *max_priority = s_mp;
}

// ReplayBuffer.update_priorities(idx, err) (train.py:86-91) for n <= kPer32MaxUpd
// entries in order: priority_k = |err_k| + eps, max_p = max(max_p, priority_k),
// leaf += fl32(priority_k ** alpha) - leaf (a repeated leaf sees the value its
// earlier occurrences left), ancestors += the same deltas in k order.
__global__ void __launch_bounds__(1024) per32_update_kernel(float* __restrict__ tree, int64_t capacity,
                                                            const int64_t* __restrict__ idx,
                                                            const double* __restrict__ err, int n,
                                                            double* __restrict__ max_priority, double eps,
                                                            double alpha) {
    __shared__ int64_t st[kPer32MaxUpd];
    __shared__ float sp[kPer32MaxUpd], sd[kPer32MaxUpd], sval[kPer32MaxUpd];
    __shared__ int sprev[kPer32MaxUpd], sround[kPer32MaxUpd];
    __shared__ unsigned char slast[kPer32MaxUpd];
    __shared__ double smax[32];
    __shared__ int s_pending;
    double mymax = 0.0;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const double pr = fabs(err[k]) + eps;
        mymax = fmax(mymax, pr);
        st[k] = capacity + idx[k];
        sp[k] = (float)pow(pr, alpha);
        sround[k] = -1;
        slast[k] = 1;
    }
    for (int o = 32; o > 0; o >>= 1) mymax = fmax(mymax, __shfl_xor(mymax, o));
    if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = mymax;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = *max_priority;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = fmax(m, smax[w]);
        *max_priority = m;
    }
    for (int k = threadIdx.x; k < n; k += blockDim.x) {   // previous occurrence of the same leaf
        int p = -1;
        for (int q = k - 1; q >= 0; --q)
            if (st[q] == st[k]) {
                p = q;
                break;
            }
        sprev[k] = p;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += blockDim.x)
        if (sprev[k] >= 0) slast[sprev[k]] = 0;
    // leaf chains: round r resolves the entries whose previous occurrence was
    // resolved in an earlier round (depth = longest run of one repeated leaf)
    for (int r = 0;; ++r) {
        if (threadIdx.x == 0) s_pending = 0;
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            if (sround[k] >= 0) continue;
            const int p = sprev[k];
            float before;
            if (p < 0) {
                before = tree[st[k]];
            } else if (sround[p] >= 0 && sround[p] < r) {
                before = sval[p];
            } else {
                s_pending = 1;
                continue;
            }
            const float d = sp[k] - before;
            sd[k] = d;
            sval[k] = before + d;
            sround[k] = r;
        }
        __syncthreads();
        if (!s_pending) break;
        __syncthreads();
    }
    for (int k = threadIdx.x; k < n; k += blockDim.x)
        if (slast[k]) tree[st[k]] = sval[k];
    // ancestors: pair (b, k) owns node anc(t_k, b) when no earlier k' has it
    const int d2 = bitlen64(2 * capacity - 1);
    for (int64_t j = threadIdx.x; j < (int64_t)n * (d2 - 1); j += blockDim.x) {
        const int b = 1 + (int)(j / n), k = (int)(j % n);
        const int64_t t = st[k];
        const int bt = bitlen64(t);
        if (bt <= b) continue;
        const int64_t m = t >> (bt - b);
        bool owner = true;
        for (int q = 0; q < k && owner; ++q) {
            const int bq = bitlen64(st[q]);
            owner = !(bq > b && (st[q] >> (bq - b)) == m);
        }
        if (!owner) continue;
        float acc = tree[m];
        for (int q = k; q < n; ++q) {
            const int bq = bitlen64(st[q]);
            if (bq > b && (st[q] >> (bq - b)) == m) acc = acc + sd[q];
        }
        tree[m] = acc;
    }
}

// ReplayBuffer.sample's descent (train.py:67-79): r = np.random.rand() * total is
// a Python float, so NEP 50 rounds it to float32 at the first comparison with a
// float32 node; from there on r and the subtraction are float32.
__global__ void per32_sample_kernel(const float* __restrict__ tree, int64_t capacity, const double* __restrict__ u,
                                    int n, int64_t* __restrict__ out_idx, float* __restrict__ out_pri) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    float r = (float)(u[k] * (double)tree[1]);
    int64_t node = 1;
    while (node < capacity) {
        const int64_t left = 2 * node;
        const float tl = tree[left];
        if (r <= tl) {
            node = left;
        } else {
            r = r - tl;
            node = left + 1;
        }
    }
    out_idx[k] = node - capacity;
    out_pri[k] = tree[node];
}

hipError_t launch_per32_add_range(float* tree, int64_t capacity, int64_t lo, int n, double* max_priority, double eps,
                                  double alpha, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(per32_add_range_kernel, dim3(1), dim3(1024), 0, stream, tree, capacity, lo, n, max_priority,
                       eps, alpha);
    return hipGetLastError();
}

hipError_t launch_per32_update(float* tree, int64_t capacity, const int64_t* idx, const double* err, int n,
                               double* max_priority, double eps, double alpha, hipStream_t stream) {
    for (int c0 = 0; c0 < n; c0 += kPer32MaxUpd) {   // sequential chunks keep the update order
        const int cn = n - c0 < kPer32MaxUpd ? n - c0 : kPer32MaxUpd;
        hipLaunchKernelGGL(per32_update_kernel, dim3(1), dim3(1024), 0, stream, tree, capacity, idx + c0, err + c0,
                           cn, max_priority, eps, alpha);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_per32_sample(const float* tree, int64_t capacity, const double* u, int n, int64_t* out_idx,
                               float* out_pri, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(per32_sample_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, tree, capacity, u, n,
                       out_idx, out_pri);
    return hipGetLastError();
}

}  // namespace trx

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
// order.  Nodes of different tree levels are independent, so each level gets
// its own workgroup (the long chains near the root run side by side on
// different CUs); the deltas are computed from the leaves as they were before
// the call, so the leaves themselves are written by a second launch.
// max_priority stays a float64 accumulated sequentially (train.py:52-54).
//
// Leaves of a capacity that is not a power of two sit at two depths: leaf t in
// [capacity, 2 capacity) has bit length d1 = bitlen(capacity) or d2 =
// bitlen(2 capacity - 1); the ancestor of t with bit length b is t >> (bitlen(t) - b).

__device__ __forceinline__ int bitlen64(int64_t x) { return 64 - __clzll((unsigned long long)x); }

constexpr int kPer32Chunk = 8192;   // ring-add leaves per launch pair (deltas staged in LDS)
constexpr int kPer32MaxUpd = 2048;  // update_priorities entries per launch pair

// The float64 running max_priority of k sequential adds, mp_k = fl(mp_{k-1} +
// eps) (train.py:52-54).  Inside one binade, away from a rounding tie, every
// step adds the same s = fl(mp_0 + eps) - mp_0, so mp_k = mp_0 + k s exactly;
// otherwise the sequence is replayed.
struct MpSeq {
    double mp0, step;
    bool closed;
};

__device__ inline MpSeq mp_sequence(double mp0, double eps, int n) {
    MpSeq q{mp0, (mp0 + eps) - mp0, false};
    int e0, e1;
    frexp(mp0, &e0);
    frexp(mp0 + (double)n * q.step, &e1);
    const double u = ldexp(1.0, e0 - 53);     // ulp of mp0
    const double r = eps / u;                 // exact (power-of-two scaling)
    q.closed = mp0 > 0.0 && e0 == e1 && (r - floor(r)) != 0.5;
    return q;
}

__device__ inline double mp_at(const MpSeq& q, double eps, int k) {   // mp after k + 1 adds
    if (q.closed) return q.mp0 + (double)(k + 1) * q.step;
    double m = q.mp0;
    for (int i = 0; i <= k; ++i) m = m + eps;
    return m;
}

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
        // order kept: ((acc + a) + b) + c ...; the long chains near the root are
        // the critical path, so 16-float LDS groups are fetched one group ahead
        int64_t t = lo;
        for (; t <= hi && ((t - T0) & 3); ++t) acc = acc + sdelta[t - T0];
        const float4* v = reinterpret_cast<const float4*>(sdelta + (t - T0));
        const int64_t nq = (hi - t + 1) >> 2;   // whole float4s
        int64_t i = 0;
        if (nq >= 4) {
            float4 c0 = v[0], c1 = v[1], c2 = v[2], c3 = v[3];
            for (; i + 8 <= nq; i += 4) {
                const float4 n0 = v[i + 4], n1 = v[i + 5], n2 = v[i + 6], n3 = v[i + 7];
                acc = acc + c0.x; acc = acc + c0.y; acc = acc + c0.z; acc = acc + c0.w;
                acc = acc + c1.x; acc = acc + c1.y; acc = acc + c1.z; acc = acc + c1.w;
                acc = acc + c2.x; acc = acc + c2.y; acc = acc + c2.z; acc = acc + c2.w;
                acc = acc + c3.x; acc = acc + c3.y; acc = acc + c3.z; acc = acc + c3.w;
                c0 = n0; c1 = n1; c2 = n2; c3 = n3;
            }
            acc = acc + c0.x; acc = acc + c0.y; acc = acc + c0.z; acc = acc + c0.w;
            acc = acc + c1.x; acc = acc + c1.y; acc = acc + c1.z; acc = acc + c1.w;
            acc = acc + c2.x; acc = acc + c2.y; acc = acc + c2.z; acc = acc + c2.w;
            acc = acc + c3.x; acc = acc + c3.y; acc = acc + c3.z; acc = acc + c3.w;
            i += 4;
        }
        for (; i < nq; ++i) {
            const float4 c = v[i];
            acc = acc + c.x; acc = acc + c.y; acc = acc + c.z; acc = acc + c.w;
        }
        for (t += 4 * nq; t <= hi; ++t) acc = acc + sdelta[t - T0];
    }
    return acc;
}

// n sequential ReplayBuffer.add(item) calls at ring slots lo .. lo+n-1
// (lo + n <= capacity, n <= kPer32Chunk): priority_k = max_p_{k-1} + eps,
// max_p_k = priority_k, leaf += fl32(priority_k ** alpha) - leaf, ancestors +=
// the same delta.  Launch 1: workgroup w owns the ancestors of bit length w + 1.
__global__ void __launch_bounds__(1024) per32_add_levels_kernel(float* __restrict__ tree, int64_t capacity, int64_t lo,
                                                               int n, const double* __restrict__ max_priority,
                                                               double eps, double alpha) {
    __shared__ __attribute__((aligned(16))) float sdelta[kPer32Chunk];
    const MpSeq q = mp_sequence(*max_priority, eps, n);
    const int64_t T0 = capacity + lo, T1 = T0 + n;
    for (int k = threadIdx.x; k < n; k += blockDim.x)
        sdelta[k] = (float)pow(mp_at(q, eps, k), alpha) - tree[T0 + k];
    __syncthreads();
    const int d1 = bitlen64(capacity), d2 = bitlen64(2 * capacity - 1);
    const int b = blockIdx.x + 1;
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

// Launch 2 (one workgroup): the leaves, then max_priority.
__global__ void __launch_bounds__(1024) per32_add_leaves_kernel(float* __restrict__ tree, int64_t capacity,
                                                                int64_t lo, int n, double* __restrict__ max_priority,
                                                                double eps, double alpha) {
    const MpSeq q = mp_sequence(*max_priority, eps, n);
    const int64_t T0 = capacity + lo;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const float old = tree[T0 + k];
        tree[T0 + k] = old + ((float)pow(mp_at(q, eps, k), alpha) - old);
    }
    __syncthreads();   // every thread has read *max_priority
    if (threadIdx.x == 0) *max_priority = mp_at(q, eps, n - 1);
}

// ReplayBuffer.update_priorities(idx, err) (train.py:86-91) for n <= kPer32MaxUpd
// entries in order: priority_k = |err_k| + eps, max_p = max(max_p, priority_k),
// leaf += fl32(priority_k ** alpha) - leaf (a repeated leaf sees the value its
// earlier occurrences left), ancestors += the same deltas in k order.
struct UpdLds {
    int64_t st[kPer32MaxUpd];
    float sp[kPer32MaxUpd], sd[kPer32MaxUpd], sval[kPer32MaxUpd];
    int sprev[kPer32MaxUpd], sround[kPer32MaxUpd];
    unsigned char sbl[kPer32MaxUpd], slast[kPer32MaxUpd];
    int pending;
};

// Leaf chains of the batch from the tree's leaves as they are on entry: sd[k]
// (delta of entry k), sval[k] (leaf after entry k), slast[k] (k is the last
// entry for its leaf).
__device__ void per32_leaf_chains(UpdLds& L, const float* __restrict__ tree, int64_t capacity,
                                  const int64_t* __restrict__ idx, const double* __restrict__ err, int n, double eps,
                                  double alpha) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const int64_t t = capacity + idx[k];
        L.st[k] = t;
        L.sbl[k] = (unsigned char)bitlen64(t);
        L.sp[k] = (float)pow(fabs(err[k]) + eps, alpha);
        L.sround[k] = -1;
        L.slast[k] = 1;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += blockDim.x) {   // previous occurrence of the same leaf
        const int64_t t = L.st[k];
        int p = -1;
#pragma unroll 8
        for (int q = 0; q < k; ++q) p = L.st[q] == t ? q : p;
        L.sprev[k] = p;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += blockDim.x)
        if (L.sprev[k] >= 0) L.slast[L.sprev[k]] = 0;
    // round r resolves the entries whose previous occurrence was resolved in an
    // earlier round (rounds = longest run of one repeated leaf)
    for (int r = 0;; ++r) {
        if (threadIdx.x == 0) L.pending = 0;
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            if (L.sround[k] >= 0) continue;
            const int p = L.sprev[k];
            float before;
            if (p < 0) {
                before = tree[L.st[k]];
            } else if (L.sround[p] >= 0 && L.sround[p] < r) {
                before = L.sval[p];
            } else {
                L.pending = 1;
                continue;
            }
            const float d = L.sp[k] - before;
            L.sd[k] = d;
            L.sval[k] = before + d;
            L.sround[k] = r;
        }
        __syncthreads();
        const int more = L.pending;
        __syncthreads();
        if (!more) break;
    }
}

// Launch 1: workgroup w owns the touched ancestors of bit length w + 1; entry k
// owns node anc(t_k) when no earlier entry has it, and adds every member's
// delta in entry order.
__global__ void __launch_bounds__(256) per32_update_levels_kernel(float* __restrict__ tree, int64_t capacity,
                                                                  const int64_t* __restrict__ idx,
                                                                  const double* __restrict__ err, int n, double eps,
                                                                  double alpha) {
    __shared__ UpdLds L;
    __shared__ int64_t anc[kPer32MaxUpd];   // entry k's ancestor at this level, -1 above its leaf
    per32_leaf_chains(L, tree, capacity, idx, err, n, eps, alpha);
    const int b = blockIdx.x + 1;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const int bt = L.sbl[k];
        anc[k] = bt > b ? L.st[k] >> (bt - b) : (int64_t)-1;
    }
    __syncthreads();
    // the scans below are branch-free selects over broadcast LDS reads: written
    // as short-circuit tests they compiled to one dependent LDS round trip per
    // entry (42 us for a 256-entry batch)
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const int64_t m = anc[k];
        if (m < 0) continue;
        int taken = 0;
#pragma unroll 8
        for (int q = 0; q < k; ++q) taken |= (int)(anc[q] == m);   // an earlier entry below m owns it
        if (taken) continue;
        float acc = tree[m];
#pragma unroll 8
        for (int q = k; q < n; ++q) {   // members in entry order (k itself first)
            const float s = acc + L.sd[q];
            acc = anc[q] == m ? s : acc;
        }
        tree[m] = acc;
    }
}

// Launch 2 (one workgroup): the leaves and max_priority.
__global__ void __launch_bounds__(1024) per32_update_leaves_kernel(float* __restrict__ tree, int64_t capacity,
                                                                   const int64_t* __restrict__ idx,
                                                                   const double* __restrict__ err, int n,
                                                                   double* __restrict__ max_priority, double eps,
                                                                   double alpha) {
    __shared__ UpdLds L;
    __shared__ double smax[16];
    per32_leaf_chains(L, tree, capacity, idx, err, n, eps, alpha);
    double mymax = 0.0;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        mymax = fmax(mymax, fabs(err[k]) + eps);
        if (L.slast[k]) tree[L.st[k]] = L.sval[k];
    }
    for (int o = 32; o > 0; o >>= 1) mymax = fmax(mymax, __shfl_xor(mymax, o));
    if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = mymax;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = *max_priority;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = fmax(m, smax[w]);
        *max_priority = m;
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

// float32 x ** e as torch's pow_tensor_scalar (the weights' op on the device):
// exponents 2, 3, -2, -1, 0.5 and -0.5 by their closed forms, every other by powf
__device__ __forceinline__ float pow_scalar_f32(float x, float e) {
    if (e == 2.0f) return x * x;
    if (e == 3.0f) return x * x * x;
    if (e == -2.0f) return 1.0f / (x * x);
    if (e == -1.0f) return 1.0f / x;
    if (e == 0.5f) return sqrtf(x);
    if (e == -0.5f) return rsqrtf(x);
    return powf(x, e);
}

// sample + importance weights in ONE workgroup (train.py:61-84 in float32):
// the descent above for every k, then w_k = (size * (pri_k / total)) ** -beta
// and w /= max(w) when that max is > 0 (a NaN max leaves w unscaled, as
// torch.where(wmax > 0, wmax, 1) does).  One block so the max needs no second
// launch; a batch of n samples takes ceil(n / 1024) descents per lane.
__global__ void __launch_bounds__(1024) per32_sample_weighted_kernel(const float* __restrict__ tree, int64_t capacity,
                                                                     const double* __restrict__ u, int n,
                                                                     const double* __restrict__ size, float neg_beta,
                                                                     int64_t* __restrict__ out_idx,
                                                                     float* __restrict__ out_pri,
                                                                     float* __restrict__ out_w) {
    __shared__ float wmax[16];
    const float total = tree[1];
    const float sz = (float)size[0];
    float m = -INFINITY;
    bool nan = false;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        float r = (float)(u[k] * (double)total);
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
        const float pri = tree[node];
        out_idx[k] = node - capacity;
        out_pri[k] = pri;
        const float w = pow_scalar_f32(sz * (pri / total), neg_beta);
        out_w[k] = w;
        nan |= w != w;
        m = fmaxf(m, w);
    }
    for (int o = 32; o > 0; o >>= 1) {
        m = fmaxf(m, __shfl_xor(m, o, 64));
        nan |= __shfl_xor((int)nan, o, 64) != 0;
    }
    const int wave = threadIdx.x >> 6, waves = (blockDim.x + 63) >> 6;
    if ((threadIdx.x & 63) == 0) wmax[wave] = nan ? __int_as_float(0x7fc00000) : m;
    __syncthreads();
    float mx = wmax[0];
    for (int w = 1; w < waves; ++w) mx = (mx != mx || wmax[w] != wmax[w]) ? __int_as_float(0x7fc00000) : fmaxf(mx, wmax[w]);
    const float d = mx > 0.0f ? mx : 1.0f;
    for (int k = threadIdx.x; k < n; k += blockDim.x) out_w[k] = out_w[k] / d;   // this lane's own stores
}

static int tree_levels(int64_t capacity) {   // internal bit lengths 1 .. d2-1
    int d2 = 0;
    while ((2 * capacity - 1) >> d2) ++d2;
    return d2 - 1;
}

hipError_t launch_per32_add_range(float* tree, int64_t capacity, int64_t lo, int n, double* max_priority, double eps,
                                  double alpha, hipStream_t stream) {
    const int levels = tree_levels(capacity);
    for (int c0 = 0; c0 < n; c0 += kPer32Chunk) {   // sequential chunks keep the add order
        const int cn = n - c0 < kPer32Chunk ? n - c0 : kPer32Chunk;
        if (levels > 0)
            hipLaunchKernelGGL(per32_add_levels_kernel, dim3(levels), dim3(1024), 0, stream, tree, capacity, lo + c0,
                               cn, max_priority, eps, alpha);
        hipLaunchKernelGGL(per32_add_leaves_kernel, dim3(1), dim3(1024), 0, stream, tree, capacity, lo + c0, cn,
                           max_priority, eps, alpha);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_per32_update(float* tree, int64_t capacity, const int64_t* idx, const double* err, int n,
                               double* max_priority, double eps, double alpha, hipStream_t stream) {
    const int levels = tree_levels(capacity);
    for (int c0 = 0; c0 < n; c0 += kPer32MaxUpd) {   // sequential chunks keep the update order
        const int cn = n - c0 < kPer32MaxUpd ? n - c0 : kPer32MaxUpd;
        if (levels > 0)
            hipLaunchKernelGGL(per32_update_levels_kernel, dim3(levels), dim3(256), 0, stream, tree, capacity,
                               idx + c0, err + c0, cn, eps, alpha);
        hipLaunchKernelGGL(per32_update_leaves_kernel, dim3(1), dim3(1024), 0, stream, tree, capacity, idx + c0,
                           err + c0, cn, max_priority, eps, alpha);
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

hipError_t launch_per32_sample_weighted(const float* tree, int64_t capacity, const double* u, int n, const double* size,
                                        double beta, int64_t* out_idx, float* out_pri, float* out_w,
                                        hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int threads = n >= 1024 ? 1024 : ((n + 63) / 64) * 64;
    hipLaunchKernelGGL(per32_sample_weighted_kernel, dim3(1), dim3(threads), 0, stream, tree, capacity, u, n, size,
                       (float)(-beta), out_idx, out_pri, out_w);
    return hipGetLastError();
}

}  // namespace trx

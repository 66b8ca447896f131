// device_common.h -- device helpers shared by the gfx950 env kernels:
// BPR cost, numpy pairwise float32 sum, the exact scipy Fibonacci-heap SSSP
// replay, and the reward formula.
#pragma once
#include <hip/hip_runtime.h>

#include "trx_internal.h"

namespace trx {
namespace {  // internal linkage: each kernel TU gets its own copy

constexpr float kInfF = __builtin_huge_valf();
constexpr double kInfD = __builtin_huge_val();
constexpr uint8_t kNoPred = 0xFF;

__device__ __forceinline__ float bpr_cost(float flow, float cap, float t0, float dmg, float alpha, float beta) {
    // repair_env.py:670-677
    const float floor6 = 1e-6f;
    float c = cap > floor6 ? cap : floor6;
    float vc = __fdiv_rn(flow, c);
    vc = vc < 0.0f ? 0.0f : (vc > 10.0f ? 10.0f : vc);
    float pw;
    if (beta == 4.0f) {
        double v = (double)vc;
        double v2 = __dmul_rn(v, v);
        pw = (float)__dmul_rn(v2, v2);
    } else {  // integer beta (checked by the host): left-to-right float64 product
        double v = (double)vc, acc = 1.0;
        const int n = (int)beta;
        for (int i = 0; i < n; ++i) acc = __dmul_rn(acc, v);
        pw = (float)acc;
    }
    float t = __fmul_rn(t0, __fadd_rn(1.0f, __fmul_rn(alpha, pw)));
    return dmg > 0.5f ? 1e6f : t;
}

// numpy pairwise_sum (float32) over a[0..n) with stride-1 LDS reads.
__device__ float pairwise_block(const float* a, int n) {
    if (n < 8) {
        float r = 0.0f;
        for (int i = 0; i < n; ++i) r = __fadd_rn(r, a[i]);
        return r;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], a[i + j]);
    }
    float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                          __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
    for (; i < n; ++i) res = __fadd_rn(res, a[i]);
    return res;
}

// numpy's recursive pairwise_sum for n > 128, unrolled to a fixed depth
// (n <= 128 * 2^D); no stack arrays, so it costs no VGPRs for the kernel.
template <int D>
__device__ __forceinline__ float pairwise_rec(const float* a, int n) {
    if constexpr (D == 0) {
        return pairwise_block(a, n);
    } else {
        if (n <= 128) return pairwise_block(a, n);
        int n2 = n / 2;
        n2 -= n2 % 8;
        return __fadd_rn(pairwise_rec<D - 1>(a, n2), pairwise_rec<D - 1>(a + n2, n - n2));
    }
}
__device__ __forceinline__ float pairwise_sum(const float* a, int n) { return pairwise_rec<4>(a, n); }

// Same recursion for any n, evaluated iteratively (explicit post-order stack)
// so that large-graph kernels do not inline 2^depth copies of the block sum.
[[maybe_unused]] __device__ __noinline__ float pairwise_sum_any(const float* a, int n) {
    if (n <= 128) return pairwise_block(a, n);
    int off[32], cnt[32];
    float lft[32];
    uint8_t st[32];
    int sp = 0;
    off[0] = 0;
    cnt[0] = n;
    st[0] = 0;
    float ret = 0.0f;
    bool have = false;
    for (;;) {
        if (!have) {
            const int c = cnt[sp];
            if (c <= 128) {
                ret = pairwise_block(a + off[sp], c);
                have = true;
                --sp;
            } else {  // descend into the left half
                int n2 = c / 2;
                n2 -= n2 % 8;
                st[sp] = 1;
                off[sp + 1] = off[sp];
                cnt[sp + 1] = n2;
                st[sp + 1] = 0;
                ++sp;
            }
        } else {
            if (sp < 0) return ret;
            if (st[sp] == 1) {  // left done: keep it, descend into the right half
                const int c = cnt[sp];
                int n2 = c / 2;
                n2 -= n2 % 8;
                lft[sp] = ret;
                st[sp] = 2;
                off[sp + 1] = off[sp] + n2;
                cnt[sp + 1] = c - n2;
                st[sp + 1] = 0;
                ++sp;
                have = false;
            } else {  // both halves done
                ret = __fadd_rn(lft[sp], ret);
                --sp;
            }
        }
    }
}

// ------------------------------------------- exact scipy heap (rare path)
// Restates scipy 1.15.3 _shortest_path.pyx FibonacciHeap on index links.
// HT is a heap-storage type exposing val/parent/left/right/child/rank/state/
// roots arrays (FibLane: per-lane LDS, int8 links, N <= 32; FibBig: per-wave
// global scratch, int16 links, N <= 16383) and its link type idx_t.
template <typename HT>
struct Heap {
    HT* h;
    int min;
};

template <typename HT>
__device__ void fh_add_sibling(HT* h, int node, int ns) {
    using I = typename HT::idx_t;
    int r = h->right[node];
    if (r >= 0) h->left[r] = (I)ns;
    h->right[ns] = (I)r;
    h->left[ns] = (I)node;
    h->right[node] = (I)ns;
    int par = h->parent[node];
    h->parent[ns] = (I)par;
    if (par >= 0) h->rank[par] += 1;
}
template <typename HT>
__device__ void fh_add_child(HT* h, int node, int c) {
    using I = typename HT::idx_t;
    h->parent[c] = (I)node;
    int ch = h->child[node];
    if (ch >= 0) {
        fh_add_sibling(h, ch, c);
    } else {
        h->child[node] = (I)c;
        h->right[c] = -1;
        h->left[c] = -1;
        h->rank[node] = 1;
    }
}
template <typename HT>
__device__ void fh_remove(HT* h, int node) {
    using I = typename HT::idx_t;
    int par = h->parent[node];
    if (par >= 0) {
        h->rank[par] -= 1;
        if (h->child[par] == node) h->child[par] = h->right[node];
    }
    int l = h->left[node], r = h->right[node];
    if (l >= 0) h->right[l] = (I)r;
    if (r >= 0) h->left[r] = (I)l;
    h->left[node] = -1;
    h->right[node] = -1;
    h->parent[node] = -1;
}
template <typename HT>
__device__ void fh_insert(Heap<HT>& H, int node) {
    using I = typename HT::idx_t;
    HT* h = H.h;
    if (H.min >= 0) {
        if (h->val[node] < h->val[H.min]) {
            h->left[node] = -1;
            h->right[node] = (I)H.min;
            h->left[H.min] = (I)node;
            H.min = node;
        } else {
            fh_add_sibling(h, H.min, node);
        }
    } else {
        H.min = node;
    }
}
template <typename HT>
__device__ void fh_decrease(Heap<HT>& H, int node, double nv) {
    using I = typename HT::idx_t;
    HT* h = H.h;
    h->val[node] = nv;
    int par = h->parent[node];
    if (par >= 0 && h->val[par] >= nv) {
        fh_remove(h, node);
        fh_insert(H, node);
    } else if (h->val[H.min] > nv) {
        fh_remove(h, node);
        h->right[node] = (I)H.min;
        h->left[H.min] = (I)node;
        H.min = node;
    }
}
template <typename HT>
__device__ void fh_link(Heap<HT>& H, int node) {
    using I = typename HT::idx_t;
    HT* h = H.h;
    for (;;) {
        int rk = h->rank[node];
        int ln = h->roots[rk];
        if (ln < 0) {
            h->roots[rk] = (I)node;
            return;
        }
        h->roots[rk] = -1;
        if (h->val[node] < h->val[ln] || node == H.min) {
            fh_remove(h, ln);
            fh_add_child(h, node, ln);
        } else {
            fh_remove(h, node);
            fh_add_child(h, ln, node);
            node = ln;
        }
    }
}
template <typename HT>
__device__ int fh_remove_min(Heap<HT>& H) {
    using I = typename HT::idx_t;
    HT* h = H.h;
    int temp = h->child[H.min];
    while (temp >= 0) {
        int tr = h->right[temp];
        fh_remove(h, temp);
        fh_add_sibling(h, H.min, temp);
        temp = tr;
    }
    int out = H.min;
    temp = h->right[H.min];
    fh_remove(h, H.min);
    H.min = temp;
    if (temp < 0) return out;
    for (int i = 0; i < 32; ++i) h->roots[i] = -1;
    while (temp >= 0) {
        if (h->val[temp] < h->val[H.min]) H.min = temp;
        int tr = h->right[temp];
        fh_link(H, temp);
        temp = tr;
    }
    temp = H.min;
    while (h->left[temp] >= 0) temp = h->left[temp];
    if (H.min != temp) {
        fh_remove(h, H.min);
        h->right[H.min] = (I)temp;
        h->left[temp] = (I)H.min;
    }
    return out;
}

// Exact scipy-order SSSP for one lane; writes scan order and predecessors
// (node-major [v][L] LDS layout) and returns the number of scanned nodes.
template <typename HT, typename CostFn>
__device__ int exact_sssp(const int N, const int32_t* __restrict__ indptr, const int32_t* __restrict__ indices,
                          CostFn cost, int origin, HT* h, uint8_t* ord, uint8_t* pred, int L, int lane) {
    for (int k = 0; k < N; ++k) {
        h->val[k] = 0.0;
        h->parent[k] = h->left[k] = h->right[k] = h->child[k] = -1;
        h->rank[k] = 0;
        h->state[k] = 0;
        pred[k * L + lane] = kNoPred;
    }
    Heap<HT> H{h, -1};
    fh_insert(H, origin);
    int k = 0;
    while (H.min >= 0) {
        int v = fh_remove_min(H);
        h->state[v] = 2;
        if (ord) ord[k * L + lane] = (uint8_t)v;
        ++k;
        double vv = h->val[v];
        for (int j = indptr[v]; j < indptr[v + 1]; ++j) {
            int jc = indices[j];
            int st = h->state[jc];
            if (st != 2) {
                double nv = vv + (double)cost(v, jc);
                if (st == 0) {
                    h->state[jc] = 1;
                    h->val[jc] = nv;
                    fh_insert(H, jc);
                    pred[jc * L + lane] = (uint8_t)v;
                } else if (h->val[jc] > nv) {
                    fh_decrease(H, jc, nv);
                    pred[jc * L + lane] = (uint8_t)v;
                }
            }
        }
    }
    return k;
}

// Same replay, recording each node's predecessor as a packed
// (link id | tail node << 16) word (-1 = unreached / origin) instead of the
// node: the large-graph kernel walks paths by link.  cost(j) is the weight of
// CSR entry j.
template <typename HT, typename CostFn>
__device__ void exact_sssp_links(const int N, const int32_t* __restrict__ indptr, const int32_t* __restrict__ indices,
                                 const int32_t* __restrict__ csr_eid, CostFn cost, int origin, HT* h,
                                 int32_t* pred_packed) {
    for (int k = 0; k < N; ++k) {
        h->val[k] = 0.0;
        h->parent[k] = h->left[k] = h->right[k] = h->child[k] = -1;
        h->rank[k] = 0;
        h->state[k] = 0;
        pred_packed[k] = -1;
    }
    Heap<HT> H{h, -1};
    fh_insert(H, origin);
    while (H.min >= 0) {
        int v = fh_remove_min(H);
        h->state[v] = 2;
        double vv = h->val[v];
        for (int j = indptr[v]; j < indptr[v + 1]; ++j) {
            int jc = indices[j];
            int st = h->state[jc];
            if (st != 2) {
                double nv = vv + (double)cost(j);
                if (st == 0) {
                    h->state[jc] = 1;
                    h->val[jc] = nv;
                    fh_insert(H, jc);
                    pred_packed[jc] = csr_eid[j] | (v << 16);
                } else if (h->val[jc] > nv) {
                    fh_decrease(H, jc, nv);
                    pred_packed[jc] = csr_eid[j] | (v << 16);
                }
            }
        }
    }
}

// compute_reward_with_goal (repair_env.py:244-291)
__device__ double reward_fn(const trx_params& p, double prev, double curr, double init, bool complete) {
    double bonus = complete ? p.reward_beta : 0.0;
    double r;
    if (p.reward_mode == TRX_REWARD_MINIMIZE_TSTT || p.reward_mode == TRX_REWARD_REL_IMPROVE) {
        double base = init;
        double bb = base > 1.0 ? base : 1.0;
        if (p.reward_mode == TRX_REWARD_MINIMIZE_TSTT) {
            r = -p.reward_alpha * (curr / bb);
        } else {
            double delta_pct = ((prev - curr) / bb) * 100.0;
            double ratio = curr / bb;
            r = p.reward_alpha * delta_pct - 1.0 * ratio;
        }
        r = r + bonus;
    } else {
        double delta;
        if (p.reward_mode == TRX_REWARD_NEG_TSTT) {
            delta = -curr;
        } else if (p.reward_mode == TRX_REWARD_LOG_DELTA) {
            delta = log10(prev > 1.0 ? prev : 1.0) - log10(curr > 1.0 ? curr : 1.0);
        } else {
            delta = prev - curr;
        }
        r = p.reward_alpha * delta + bonus - p.reward_gamma;
    }
    if (p.reward_clip > 0) r = r < -p.reward_clip ? -p.reward_clip : (r > p.reward_clip ? p.reward_clip : r);
    return r;
}

}  // namespace
}  // namespace trx

// trx_internal.h -- shared declarations between the C-ABI host code and the
// gfx950 kernels of libtrafficrl.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "trafficrl.h"


namespace trx {

// records the message trx_last_error() returns (capi.hip); returns code
int set_error(int code, const char* fmt, ...);


// Largest node count handled by the register-resident small-graph kernel
// (dist labels live in VGPRs, one lane per (env, origin) SSSP).
constexpr int kSmallMaxNodes = 32;
// Largest node count of the LDS-resident large-graph kernel (14-bit node ids
// in the packed in-link entries; the LDS budget is checked per graph).
constexpr int kBigMaxNodes = 16382;  // node id 16382 < 2^14 - 1; N itself is the dummy node

// Device-resident, immutable graph description (built by trx_graph_create).
struct DevGraph {
    int N, E, Z, NP;            // nodes, edges, origins (zones with demand), padded nodes
    int P;                      // OD entries
    const int32_t* src;         // [E]
    const int32_t* dst;         // [E]
    const float* t0;            // [E]
    const float* cap0;          // [E]
    const int32_t* indptr;      // [N+1]  CSR rows sorted by column (scipy order)
    const int32_t* indices;     // [E]
    const int32_t* csr_eid;     // [E]
    const int16_t* eid_of;      // [NP*NP] (u,v) -> edge id, -1 = no edge
    const float* dem;           // [Z*N]  demand origin zone zi -> node v (fp32, exact ints)
    const int32_t* origins;     // [Z]    node id of origin zone zi
    const int32_t* nx_order;    // [N]    networkx node insertion order (observation)
    const int32_t* out_ptr;     // [N+1]  successors in networkx adjacency (file) order
    const int32_t* out_dst;     // [E]
    const int32_t* out_eid;     // [E]
    const int32_t* in_ptr;      // [N+1]  predecessors (any order: distinct tails)
    const int32_t* in_src;      // [E]
    const int32_t* in_eid;      // [E]
    // large-graph kernel (N > kSmallMaxNodes): in-links grouped per node, nodes
    // dealt to lanes in contiguous chunks of a DFS order (see capi.hip)
    int KMAX;                   // packed entries per lane
    int big_g;                  // lanes per shortest-path tree (32 or 64)
    const uint32_t* blist;      // [KMAX][big_g] u | v<<16 | first<<30 | last<<31 (DFS positions)
    const int16_t* blink;       // [KMAX][big_g] link id of the entry, -1 = padding / no in-link
    // node ids of the large-graph kernels are DFS positions (capi.hip):
    const int32_t* b_origin;    // [Z]    origin of zone zi
    const int32_t* b_od_dst;    // [P]    OD destination
    const int16_t* b_lsrc;      // [E]    tail of each link
    const int32_t* b_indptr;    // [N+1]  scipy CSR, rows by DFS position, entries in scipy order
    const int32_t* b_indices;   // [E]
    const int32_t* b_csr_eid;   // [E]
    const int32_t* od_ptr;      // [Z+1]  OD entries of origin zone zi (dict order)
    const int32_t* od_dst;      // [P]
    const float* od_dem;        // [P]
    double total_demand;        // float(np.sum(list(od_demand.values())))
    float max_t0, max_cap;      // RepairEnv.max_t0 / max_capacity
    float min_t0;               // smallest free-flow time (exact-label headroom, assign_sparse.hip)
    int max_out_deg, max_in_deg;  // largest out-/in-degree (sparse-relaxation kernel tables)
    int reach_all;              // every origin reaches every node (N <= kSmallMaxNodes; env_kernel_pair FULL)
};

// Per-lane Fibonacci-heap state for the exact (scipy-order) SSSP fallback.
struct FibLane {
    using idx_t = int8_t;
    double val[kSmallMaxNodes];
    int8_t parent[kSmallMaxNodes], left[kSmallMaxNodes], right[kSmallMaxNodes], child[kSmallMaxNodes];
    uint8_t rank[kSmallMaxNodes], state[kSmallMaxNodes];
    int8_t roots[32];
};

// Per-wave Fibonacci-heap scratch of the large-graph kernel, carved from the
// caller's workspace (global memory): int16 links, N <= kBigMaxNodes.
struct FibBig {
    using idx_t = int16_t;
    double* val;
    int16_t *parent, *left, *right, *child;
    uint8_t *rank, *state;
    int16_t* roots;  // [32]
};

// Path-based (GP) assignment state: one row per env (trx_state.gp).
constexpr int kGpMaxHops = 32;   // links per path (N <= 32)
constexpr int kGpMaxPaths = 4;   // gp_keep_paths + 1 while a new path is priced
struct GpLayout {
    size_t nkeys, ord, np, flow, mask, len, edges, total;
};
__host__ __device__ inline GpLayout gp_layout(int P, int keep) {
    const size_t KP = (size_t)keep + 1;
    GpLayout o{};
    size_t off = 0;
    auto take = [&off](size_t b) {
        size_t r = off;
        off = (off + b + 15) & ~(size_t)15;
        return r;
    };
    o.nkeys = take(16);                      // i32 keys inserted so far
    o.ord = take((size_t)P * 2);             // i16 key ids in insertion (dict) order
    o.np = take((size_t)P);                  // u8 paths per key
    o.flow = take((size_t)P * KP * 8);       // f64 path flows
    o.mask = take((size_t)P * KP * 16);      // uint4 link bitmask per path (E <= 128)
    o.len = take((size_t)P * KP);            // u8 links per path
    o.edges = take((size_t)P * KP * kGpMaxHops);  // u8 link ids in path order
    o.total = (off + 255) & ~(size_t)255;
    return o;
}

enum RunMode { kModeAssign = 0, kModeReset = 1, kModeStep = 2 };

struct LaunchCfg {
    int np;        // template node padding
    int epw;       // envs per workgroup
    int threads;   // block size
    size_t smem;   // dynamic LDS bytes
    int blocks;    // grid
};

// Small-graph (N <= kSmallMaxNodes) env kernels, selected per graph and
// parameters by capi.hip select_env_kernel():
//   scipy rule: env_kernel_pair (assign_pair.hip) when pair_ok(), else
//               env_kernel_s (assign_sparse.hip) when sparse_ok(), else
//               env_kernel_q (assign_quad.hip, no exact-label / degree limits);
//   torch rule: env_kernel_t (assign_torch.hip) when torch_kernel_ok(), else
//               env_kernel_q's torch-rule instantiation.
LaunchCfg quad_launch_cfg(const DevGraph& g, int num_envs, int sp_rule);
bool quad_ok(const DevGraph& g, int sp_rule);  // LDS / block-size budget of env_kernel_q
bool exact_label_ok(const DevGraph& g, const trx_params& p);
bool sparse_ok(const DevGraph& g, const trx_params& p);
LaunchCfg sparse_launch_cfg(const DevGraph& g, int num_envs, int method);
hipError_t launch_env_kernel_sparse(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs,
                                    int mode, const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                    const uint8_t* env_mask, void* workspace, hipStream_t stream);
size_t sparse_workspace_bytes(const DevGraph& g, int num_envs);  // exact-heap scratch, one FibLane per tree
bool pair_ok(const DevGraph& g, const trx_params& p);
LaunchCfg pair_launch_cfg(const DevGraph& g, int num_envs, int method);
hipError_t launch_env_kernel_pair(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                  const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                  const uint8_t* env_mask, hipStream_t stream);
hipError_t launch_env_kernel_quad(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                  const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                  const uint8_t* env_mask, hipStream_t stream);

bool torch_kernel_ok(const DevGraph& g);
hipError_t launch_env_kernel_torch(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                   const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                   const uint8_t* env_mask, hipStream_t stream);

size_t big_smem_bytes(const DevGraph& g, int waves);
int big_waves(const DevGraph& g);  // waves per workgroup that fit the LDS budget (0 = none)
size_t big_workspace_bytes(const DevGraph& g, int num_envs);
hipError_t launch_env_kernel_big(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                                 const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                                 const uint8_t* env_mask, void* workspace, hipStream_t stream);

hipError_t launch_gp_kernel(const DevGraph& g, const trx_params& p, const trx_state& s, int num_envs, int mode,
                            const int32_t* action, double* reward, uint8_t* done, uint8_t* valid,
                            const uint8_t* env_mask, hipStream_t stream);
hipError_t launch_observe_big(const DevGraph& g, int num_envs, const trx_state& s, float* node_x, float* edge_x,
                              float* mask, hipStream_t stream);
hipError_t launch_observe_kernel(const DevGraph& g, int num_envs, const trx_state& s, float* node_x, float* edge_x,
                                 float* mask, hipStream_t stream);

hipError_t launch_gat_forward(int Nt, int H, int C, const int32_t* rowptr, const int32_t* src, const void* xh,
                              int bf16, const float* a_src, const float* a_dst, const float* a_edge, float slope,
                              const float* bias, float* out, float* alpha, hipStream_t stream);
hipError_t launch_gat_backward(int Nt, int H, int C, const int32_t* rowptr, const int32_t* src, const int32_t* sptr,
                               const int32_t* spos, const int32_t* sdst, const void* xh, int bf16, const float* a_src,
                               const float* a_dst, const float* a_edge, float slope, const float* alpha,
                               const float* gout, void* gxh, float* ga_src, float* ga_dst, float* ga_edge,
                               hipStream_t stream);

size_t gat_layer_infer_smem(const trx_gat_layer_args& a);
// several networks' passes in one launch (blockIdx.y = network): the argument
// blocks travel by value in the kernel arguments, indexed by blockIdx.y
template <class A>
struct NetList {
    A a[TRX_MAX_NETS];
};
template <class A>
inline NetList<A> net_list(const A* a, int count) {
    NetList<A> l{};
    for (int k = 0; k < count; ++k) l.a[k] = a[k];
    return l;
}
struct EdgeHeadBwdItem {
    trx_edge_head_args a;
    trx_edge_head_bwd_io io;
};
hipError_t launch_gat_layer_infer(const trx_gat_layer_args* a, int count, hipStream_t stream);
hipError_t launch_edge_head_infer(const trx_edge_head_args* a, int count, hipStream_t stream);
size_t gat_layer0_smem(const trx_gat_layer0_args& a);
hipError_t launch_gat_layer0(const trx_gat_layer0_args& a, hipStream_t stream);
size_t gat_mid_smem(const trx_gat_mid_args& a);
hipError_t launch_gat_mid(const trx_gat_mid_args& a, hipStream_t stream);
hipError_t launch_gat_layer0_prepare(int H, int C, const float* w0, const float* att_src, const float* att_dst,
                                     const float* bias, float* u, double* stats, hipStream_t stream);
size_t edge_head_infer_smem(const trx_edge_head_args& a);
size_t gat_tail_smem(const trx_gat_tail_args& a);
int gat_tail_mtiles(int nodes_per_graph);
hipError_t launch_gat_tail_infer(const trx_gat_tail_args& a, hipStream_t stream);
size_t edge_head_bwd_smem(const trx_edge_head_args& a);
hipError_t launch_edge_head_bwd(const EdgeHeadBwdItem* items, int count, hipStream_t stream);
int layer_tail_blocks(int N);
int att_dots_blocks(int N);
int small_ln_blocks(int N);
hipError_t launch_bf16_round(const trx_round_list& l, hipStream_t stream);
hipError_t launch_episode_step(int B, const double* reward, const uint8_t* done, const double* tstt,
                               double reward_scale, int64_t max_steps, double* scaled, float* scaled_f32,
                               float* done_f32, double* ep_reward, double* ep_tstt_sum, double* ep_auc,
                               double* ep_prev_tstt, int64_t* ep_len, uint8_t* finished, hipStream_t stream);
hipError_t launch_multi_gather(const trx_copy_list& l, const int64_t* idx, int nrows, hipStream_t stream);
hipError_t launch_multi_copy(const trx_copy_list& l, hipStream_t stream);
hipError_t launch_graph_pool_fwd(int B, int n, int F, const float* x, float* out, float* ties, hipStream_t stream);
hipError_t launch_graph_pool_bwd(int B, int n, int F, const float* x, const float* out, const float* ties,
                                 const float* g, float* gx, hipStream_t stream);
hipError_t launch_small_ln_fwd(int N, int d, const float* x, const float* w, const float* b, float eps, float* y,
                               float* stats, hipStream_t stream);
hipError_t launch_small_ln_bwd(int N, int d, const float* gy, const float* x, const float* w, const float* stats,
                               float* gx, float* gwb, float* part, hipStream_t stream);
hipError_t launch_att_dots_fwd(int N, int H, int C, const void* xh, int bf16, const float* att_src,
                               const float* att_dst, float* a_src, float* a_dst, hipStream_t stream);
hipError_t launch_att_dots_bwd(int N, int H, int C, const void* xh, int bf16, const float* att_src,
                               const float* att_dst, const float* g_src, const float* g_dst, void* g_xh,
                               float* g_att, float* part, hipStream_t stream);
hipError_t launch_layer_tail_fwd(int N, int F, int act, int res_bf16, const float* out, const float* bias,
                                 const float* w, const float* b, float eps, const void* res, float* y, float* stats,
                                 hipStream_t stream);
hipError_t launch_layer_tail_bwd(int N, int F, int act, int res_bf16, const float* gy, const float* out,
                                 const float* bias, const float* w, const float* y, const float* stats, float* gout,
                                 void* gres, float* part, float* grads, hipStream_t stream);
hipError_t launch_gat_prologue(const trx_gat_prologue_args* a, int count, hipStream_t stream);
size_t gat_prologue_smem(const trx_gat_prologue_args& a);
hipError_t patch_graph_memsets(hipGraph_t graph, int* n_patched);
size_t gat_layer_bwd_smem(const trx_gat_layer_bwd_args& a);
hipError_t launch_gat_layer_bwd(const trx_gat_layer_bwd_args* a, int count, hipStream_t stream);
hipError_t launch_partial_sum(const float* part, int rows, int width, int64_t stride, float* out, hipStream_t stream);
hipError_t launch_partial_sum_multi(const trx_psum_list& l, hipStream_t stream);
hipError_t launch_edge_att_weights_bwd(const trx_gat_prologue_args& a, const float* gm, int gm_stride, float* out,
                                       hipStream_t stream);
size_t gat_prologue_bwd_smem(const trx_gat_prologue_bwd_args& a);
hipError_t launch_gat_prologue_bwd(const trx_gat_prologue_bwd_args* a, int count, hipStream_t stream);
hipError_t launch_sac_loss(const trx_sac_loss_args& a, hipStream_t stream);
hipError_t launch_sac_adam(const trx_adam_args& a, hipStream_t stream);
hipError_t launch_per_update(double* tree, int64_t capacity, const int64_t* idx, const double* pri, int n,
                             hipStream_t stream);
hipError_t launch_per_update_range(double* tree, int64_t capacity, int64_t lo, const double* pri, int n,
                                   hipStream_t stream);
hipError_t launch_per_add_range(double* tree, int64_t capacity, int64_t lo, int n, double* max_priority, double eps,
                                double alpha, hipStream_t stream);
hipError_t launch_per_sample(const double* tree, int64_t capacity, const double* u, int n, int64_t* out_idx,
                             double* out_pri, hipStream_t stream);
hipError_t launch_per32_add_range(float* tree, int64_t capacity, int64_t lo, int n, double* max_priority, double eps,
                                  double alpha, hipStream_t stream);
hipError_t launch_per32_update(float* tree, int64_t capacity, const int64_t* idx, const double* err, int n,
                               double* max_priority, double eps, double alpha, hipStream_t stream);
hipError_t launch_per32_sample(const float* tree, int64_t capacity, const double* u, int n, int64_t* out_idx,
                               float* out_pri, hipStream_t stream);
hipError_t launch_per32_sample_weighted(const float* tree, int64_t capacity, const double* u, int n, const double* size,
                                        double beta, int64_t* out_idx, float* out_pri, float* out_w,
                                        hipStream_t stream);

}  // namespace trx

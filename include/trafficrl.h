/*
 * trafficrl.h -- C ABI of libtrafficrl.so, the MI355X (gfx950) implementation
 * of the reference's per-step user-equilibrium hot path.
 *
 * The reference's boundary is Python (pop-pop-pOp-dev/SAC-GAT-HER_transportationRL,
 * src/env/repair_env.py); every entry point below names the reference
 * function/statement range it replaces.  INTEGRATION.md shows the ctypes
 * binding the reference side would add; trafficrl/_lib.py is that binding.
 *
 * Conventions
 *  - All buffers are CALLER-OWNED DEVICE pointers (e.g. torch tensors'
 *    data_ptr()), row-major [B, E] / [B] unless noted.  Graph inputs to
 *    trx_graph_create are HOST pointers (copied to the device).
 *  - Every call is stream-ordered and asynchronous on `stream` (a
 *    hipStream_t passed as void*; NULL = the null stream).  No call
 *    allocates, frees or synchronises (hipGraph-capturable), except
 *    trx_graph_create/destroy.
 *  - A graph handle is bound to the device current at creation.  Handles are
 *    immutable after creation and may be shared by threads; one stream per
 *    host thread.
 *  - Return 0 on success, <0 on error; trx_last_error() gives a thread-local
 *    message.  No C++ exception crosses this boundary.
 */
#ifndef TRAFFICRL_H
#define TRAFFICRL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TRX_ABI_VERSION 12  /* 12: trx_bf16_round modes 16..23 (a three-piece split from one read);
                                 11: *_multi entry points (several networks' passes per launch);
                                 10: `exact` (float32) mode of the fused forward/backward kernels;
                                  9: fp32 edge scorer after its p GEMM; trx_gat_layer0_* */

/* error codes */
#define TRX_OK 0
#define TRX_EINVAL (-1)   /* bad argument (ValueError on the Python side)   */
#define TRX_EHIP (-2)     /* HIP runtime failure (RuntimeError)             */
#define TRX_EUNSUP (-3)   /* input outside what a kernel supports           */

/* assignment methods: RepairEnv(assignment_method=...) repair_env.py:55,304-335 */
#define TRX_METHOD_MSA 0
#define TRX_METHOD_FW 1
#define TRX_METHOD_CFW 2
#define TRX_METHOD_GP 3   /* path-based: _compute_flow_assignment_gp, repair_env.py:351-419 */

/* reward modes: RepairEnv.compute_reward_with_goal repair_env.py:244-291 */
#define TRX_REWARD_DELTA 0
#define TRX_REWARD_LOG_DELTA 1
#define TRX_REWARD_NEG_TSTT 2
#define TRX_REWARD_MINIMIZE_TSTT 3
#define TRX_REWARD_REL_IMPROVE 4

/* shortest-path rule of the all-or-nothing step: RepairEnv(sp_backend=...)
 * repair_env.py:34, 111-161, 421-573.  SCIPY: scipy.sparse.csgraph.dijkstra
 * (float64 labels, scipy heap order on ties; what sp_backend="auto"/"scipy"
 * resolves to without cupy/cugraph).  TORCH: _all_or_nothing_torch, float32
 * Floyd-Warshall (k ascending, strict <) + next_hop walk (sp_backend="torch"
 * on a GPU device: configs/sioux_falls.yaml, run_greedy.py).  TORCH needs
 * N <= 32; GP assignment always uses SCIPY (as _shortest_paths_from_origin). */
#define TRX_SP_SCIPY 0
#define TRX_SP_TORCH 1

typedef struct trx_graph trx_graph;

/* Env constants of RepairEnv.__init__ (repair_env.py:23-50). */
typedef struct trx_params {
    int32_t method;             /* TRX_METHOD_*                      assignment_method   */
    int32_t iters;              /* K > 0                             assignment_iters    */
    float bpr_alpha;            /* 0.15                              bpr_alpha           */
    float bpr_beta;             /* 4.0                               bpr_beta            */
    float capacity_damage;      /* 1e-3                              capacity_damage     */
    float _pad0;
    double unassigned_penalty;  /* 2e7 (yaml: 1e4)                   unassigned_penalty  */
    int32_t reward_mode;        /* TRX_REWARD_*                      reward_mode         */
    int32_t sp_rule;            /* TRX_SP_*                          sp_backend          */
    double reward_alpha, reward_beta, reward_gamma, reward_clip;
    double gp_step;             /* 1.0; <= 0 means 1/(it+1)          gp_step (GP only)   */
    int32_t gp_keep_paths;      /* 3 (yaml: 2); 1..3 supported       gp_keep_paths       */
    int32_t _pad2;
} trx_params;

/* Per-env state of B vectorised envs: device pointers, caller-owned.
 * Mirrors RepairEnv attributes (repair_env.py:167-205):
 *   flow          [B,E] f32  self.flow          (warm start in, result out)
 *   capacity      [B,E] f32  self.capacities
 *   damaged       [B,E] f32  self.is_damaged    (0/1)
 *   goal          [B,E] f32  self.goal_mask     (0/1)
 *   t             [B,E] f32  BPR(final flow)    (may be NULL)
 *   tstt          [B]   f64  self.tstt
 *   initial_tstt  [B]   f64  self.initial_tstt
 *   unassigned    [B]   f64  self.unassigned_demand                          */
typedef struct trx_state {
    float* flow;
    float* capacity;
    float* damaged;
    float* goal;
    float* t;
    double* tstt;
    double* initial_tstt;
    double* unassigned;
    void* gp;       /* TRX_METHOD_GP only: per-env path sets, i.e. RepairEnv.od_paths /
                     * od_path_flows (repair_env.py:199-200, 351-404), trx_gp_state_bytes()
                     * per env, caller-owned, kept between calls (cleared by trx_reset) */
} trx_state;

/* ---------------------------------------------------------------- misc */
int32_t trx_abi_version(void);
const char* trx_last_error(void);

/* ----------------------------------------------------------------- graph
 * Replaces RepairEnv.__init__ array setup (repair_env.py:85-96, 106-109) over
 * GraphData from src/data/tntp_parser.py:102-105.
 *   src,dst   [E] 0-based node ids (file order = edge id order)
 *   t0,cap0   [E] free-flow time, capacity (float32, like repair_env.py:89-91)
 *   od_o,od_d,od_v [P] OD entries in dict order (0-based), demand > 0
 * Fails (TRX_EUNSUP) on parallel links (scipy's csr_matrix would sum them)
 * or on non-integral / >= 2^24 total demand (the exact fp32 AON contract). */
int trx_graph_create(int32_t num_nodes, int32_t num_edges, const int32_t* src, const int32_t* dst,
                     const float* t0, const float* cap0, int32_t num_od, const int32_t* od_o,
                     const int32_t* od_d, const double* od_v, trx_graph** out);
int trx_graph_destroy(trx_graph* g);
/* num_nodes, num_edges, num_origins (zones with demand), total_demand */
int trx_graph_info(const trx_graph* g, int32_t* num_nodes, int32_t* num_edges, int32_t* num_origins,
                   double* total_demand);
/* Device scratch bytes needed by trx_reset/step/assign for B envs. */
int64_t trx_workspace_bytes(const trx_graph* g, int32_t num_envs);
/* Bytes of trx_state.gp for num_envs envs with gp_keep_paths = keep_paths
 * (envs are contiguous rows of equal size: row b starts at b * bytes(1)).
 * GP needs N <= 32, E <= 128 and 1 <= keep_paths <= 3 (else TRX_EUNSUP). */
int64_t trx_gp_state_bytes(const trx_graph* g, int32_t num_envs, int32_t keep_paths);

/* Which env kernel trx_assign/trx_reset/trx_step launch for this graph and
 * params: "env_kernel_s" (scipy rule, N <= 32, within the exact-label and
 * out-degree <= 16 preconditions), "env_kernel_q" (the general N <= 32 kernel,
 * both rules), "env_kernel_t" (torch rule), "env_kernel_big" (N > 32),
 * "gp_kernel", or "" when no kernel takes the pair (the calls then fail with
 * TRX_EUNSUP).  No device work; the string is static. */
const char* trx_env_kernel_name(const trx_graph* g, const trx_params* p);

/* ----------------------------------------------------------- hot path
 * trx_assign: RepairEnv.compute_flow_assignment (repair_env.py:299-345) for
 * every env b with env_mask[b] != 0 (env_mask NULL = all): warm start from
 * state.flow, K iterations of BPR (667-677) -> all-or-nothing over every OD
 * pair (scipy branch 481-503, 707-722) -> MSA/FW/CFW averaging (315-343),
 * then TSTT (724-735).  Writes flow, t, tstt, unassigned.  Used by the
 * greedy baseline's what-if batches (src/baselines/__init__.py:51-67). */
int trx_assign(const trx_graph* g, const trx_params* p, int32_t num_envs, trx_state* s, const uint8_t* env_mask,
               void* workspace, void* stream);

/* trx_reset: RepairEnv.reset (repair_env.py:167-205) after damage sampling.
 * The caller writes the sampled 0/1 mask into state.damaged (numpy PCG64
 * sampling + strong-connectivity retries stay on the host, 168-192).  Sets
 * capacity (cap0 or capacity_damage), goal = damaged, flow = 0, runs the
 * assignment and sets tstt = initial_tstt.  env_mask as in trx_assign. */
int trx_reset(const trx_graph* g, const trx_params* p, int32_t num_envs, trx_state* s, const uint8_t* env_mask,
              void* workspace, void* stream);

/* trx_step: RepairEnv.step (repair_env.py:207-237) for all B envs.
 *   action [B] int32 edge ids; must be in [0,E) (the host checks the range
 *   and raises ValueError, 208-209).  An already-repaired edge gives
 *   reward -1, done 0 and no assignment (210-212); otherwise the edge is
 *   repaired, the assignment runs, reward = compute_reward_with_goal
 *   (220-230), done = is_goal_complete (236).
 *   reward [B] f64, done [B] u8, valid [B] u8 (1 if an assignment ran). */
int trx_step(const trx_graph* g, const trx_params* p, int32_t num_envs, trx_state* s, const int32_t* action,
             double* reward, uint8_t* done, uint8_t* valid, void* workspace, void* stream);

/* trx_observe: RepairEnv.get_state (repair_env.py:751-819) for B envs.
 *   node_x [B,N,4] f32: betweenness of the active subgraph / its max,
 *                      remaining goal ratio, avg undamaged flow norm, log10 tstt
 *   edge_x [B,E,6] f32: t0_norm, cap_norm, clip(log1p(v/c)), damaged, goal, id/(E-1)
 *   mask   [B,E]   f32: action_mask = damaged (may be NULL)                     */
int trx_observe(const trx_graph* g, int32_t num_envs, const trx_state* s, float* node_x, float* edge_x,
                float* mask, void* workspace, void* stream);

/* ------------------------------------------------------------------ GAT
 * Edge softmax + neighbour aggregation of torch_geometric GATConv as used by
 * GATEncoder (src/models/gat_encoder.py:22-25, 36-42; PyG GATConv.forward
 * after `lin`): over a graph in CSR-by-destination form (self loops included)
 *   logit[e,h] = leaky_relu(a_src[src[e],h] + a_dst[i,h] + a_edge[e,h], negative_slope)
 *   alpha[e,h] = softmax over the in-edges of i (max-shifted, +1e-16 denominator)
 *   out[i,h*C:(h+1)*C] = sum_e alpha[e,h] * xh[src[e], h*C:(h+1)*C]  (+ bias, may be NULL)
 * xh [N, heads*channels] float32 (xh_bf16=0) or bfloat16 (1); a_src/a_dst
 * [N,heads], a_edge/alpha [num_edges,heads] in CSR order, out [N,heads*channels].
 * Constraints: heads <= 8, channels % 4 == 0, heads*channels <= 2048,
 * channels divides 256 or is a multiple of 256. */
int trx_gat_forward(int32_t num_nodes, int32_t heads, int32_t channels, const int32_t* rowptr, const int32_t* src,
                    const void* xh, int32_t xh_bf16, const float* a_src, const float* a_dst, const float* a_edge,
                    float negative_slope, const float* bias, float* out, float* alpha, void* stream);
/* Backward of trx_gat_forward (without bias).  (sptr, spos, sdst) is the same
 * graph in CSR by SOURCE: for node j, entries sptr[j]..sptr[j+1] give the
 * dst-CSR position and destination of each out-edge (fixed order =>
 * deterministic, no float atomics).  grad_xh [N,heads*channels] in xh's dtype
 * (float32, or bfloat16 rounded to nearest even when xh_bf16). */
int trx_gat_backward(int32_t num_nodes, int32_t heads, int32_t channels, const int32_t* rowptr, const int32_t* src,
                     const int32_t* sptr, const int32_t* spos, const int32_t* sdst, const void* xh, int32_t xh_bf16,
                     const float* a_src, const float* a_dst, const float* a_edge, float negative_slope,
                     const float* alpha, const float* grad_out, void* grad_xh, float* grad_a_src, float* grad_a_dst,
                     float* grad_a_edge, void* stream);

/* ------------------------------------------------ fused GAT inference
 * Acting (and the no-grad target/next-state passes of the SAC update) run
 * the whole GATEncoder layer (src/models/gat_encoder.py:36-52) as ONE kernel
 * per layer, one workgroup per graph: the graph's xh rows are staged in LDS
 * once, then attention logits (PyG GATConv: <xh,att_src>, <xh,att_dst>,
 * a_edge, leaky_relu, softmax over in-edges +1e-16), neighbour aggregation,
 * + bias, LayerNorm, residual (layer 0: input_proj(x) computed in-kernel;
 * later layers: the previous layer's output), ReLU / ELU and, on the last
 * layer, global mean|max pooling.  The dense `lin` projection of layers >= 1
 * stays a bf16 MFMA GEMM on the torch side.  Batches must be regular: graph
 * b owns nodes [b*n, (b+1)*n) and its CSR-by-destination range, n <= 32,
 * <= 256 edges (self loops included) per graph.  Numerics follow the
 * bf16-autocast torch path (bf16 roundings at the same points).             */
typedef struct trx_gat_layer_args {
    int32_t num_graphs, nodes_per_graph, heads, channels, concat;
    int32_t max_graph_edges;    /* CSR positions per graph (self loops included), <= 256;
                                   a graph with more gets NaN outputs */
    int32_t in_dim;             /* 4: layer 0, xh = bf16(x0 @ w0^T) in-kernel; 0: xh given */
    const void* xh;             /* bf16 [N, heads*channels]                   (in_dim == 0) */
    const float* x0;            /* [N, in_dim] layer input                    (in_dim > 0)  */
    const float* w0;            /* [heads*channels, in_dim] lin.weight, bf16-representable  */
    const int32_t* rowptr;      /* [N+1] CSR by destination (self loops included)           */
    const int32_t* col;         /* [Et]  source node of each CSR position                   */
    const float* a_edge;        /* [Et, a_edge_stride] edge logits in CSR order             */
    int32_t a_edge_stride, a_edge_offset;
    const float* att_src;       /* [heads*channels] */
    const float* att_dst;       /* [heads*channels] */
    const float* bias;          /* [out] (out = concat ? heads*channels : channels)         */
    float negative_slope;
    const float* ln_weight;     /* [out] */
    const float* ln_bias;       /* [out] */
    float ln_eps;
    int32_t residual;           /* 0 none, 1 res [N,out] fp32, 2 bf16(x0 @ wp^T + bp)       */
    const float* res;
    const float* wp;            /* [out, in_dim] bf16-representable */
    const float* bp;            /* [out] bf16-representable */
    int32_t activation;         /* 0 relu, 1 elu */
    float* out_f32;             /* [N, out] or NULL */
    void* out_bf16;             /* [N, out] bf16 or NULL */
    float* pool;                /* [num_graphs, 2*out] mean | max, or NULL */
    /* training forward (trx_gat_layer_backward's saved tensors), each NULL = not saved: */
    float* save_alpha;          /* [Et, heads] attention weights in CSR order             */
    float* save_asd;            /* [N, 2*heads] a_src | a_dst                              */
    float* save_v;              /* [N, out] aggregate + bias (LayerNorm input)             */
    float* save_stats;          /* [N, 2] LayerNorm mean, rstd                             */
    int32_t exact;              /* ABI 10: 1 = float32 throughout (xh float [N, out], layer 0 computes
                                   xh and the input projection unrounded, x0 unrounded; heads*channels
                                   <= 1024); 0 = the bf16-autocast rounding points above */
} trx_gat_layer_args;
int trx_gat_layer_infer(const trx_gat_layer_args* a, void* stream);
/* ABI 11: the same layer for `count` (1..TRX_MAX_NETS) networks in ONE launch
 * (workgroup (g, k) = graph g of network k): a[k] are complete argument
 * blocks that must agree in num_graphs, nodes_per_graph, heads, channels,
 * max_graph_edges, in_dim, exact and the presence of pool; every buffer is
 * per network.  Results equal `count` separate trx_gat_layer_infer calls --
 * the SAC update evaluates its same-shaped networks (the next-state actor and
 * target critics, the two critics) this way. */
#define TRX_MAX_NETS 6
int trx_gat_layer_infer_multi(const trx_gat_layer_args* a, int32_t count, void* stream);

/* Layer 0 of GATEncoder for inference (no saved intermediates), in its linear
 * form (gat_layer0.hip): 4 raw features per node, heads*channels = 256, 512 or
 * 1024, concat, LayerNorm, relu(x + input_proj(x_in)); fp32 throughout.  The
 * attention logits are 4-dots with u = W0_h^T att_h, the aggregate is
 * W0_h (sum_j alpha_jh x_j) + b, the LayerNorm statistics are float64 forms
 * of that per-head 4-vector (`stats`).  u and stats come from
 * trx_gat_layer0_prepare whenever the weights change. */
typedef struct trx_gat_layer0_args {
    int32_t num_graphs, nodes_per_graph, heads, channels;  /* nodes_per_graph <= 32 */
    int32_t max_graph_edges;    /* CSR positions per graph (self loops included), <= 256 */
    const float* x0;            /* [N, 4] raw (normalised) node features */
    const float* w0;            /* [heads*channels, 4] lin.weight */
    const int32_t* rowptr;      /* [N+1] CSR by destination (self loops included) */
    const int32_t* col;         /* [Et] */
    const float* a_edge;        /* [Et, a_edge_stride] edge logits in CSR order */
    int32_t a_edge_stride, a_edge_offset;
    const float* bias;          /* [heads*channels] */
    float negative_slope;
    const float* ln_weight;     /* [heads*channels] */
    const float* ln_bias;
    float ln_eps;
    const float* wp;            /* [heads*channels, 4] input_proj.weight */
    const float* bp;            /* [heads*channels] input_proj.bias */
    const float* u;             /* [2, heads, 4] W0_h^T att_src_h | W0_h^T att_dst_h */
    const double* stats;        /* [heads*24 + 2] (trx_gat_layer0_prepare) */
    float* out_f32;             /* [N, heads*channels] or NULL */
    void* out_bf16;             /* [N, heads*channels] bf16 or NULL */
    float* desc;                /* [N, 4*heads + 8] per-node descriptor (xbar [heads][4], x [4], mean,
                                   rstd, 0, 0) for trx_gat_mid_infer, or NULL */
} trx_gat_layer0_args;
int trx_gat_layer0_infer(const trx_gat_layer0_args* a, void* stream);
/* The middle GAT layer whose residual input is layer 0's output (GATEncoder
 * layer 1), for inference: xh = bf16(x_in @ lin.weight^T) given, channels
 * == 256, heads*channels = layer 0's; the residual rows are regenerated from
 * layer 0's descriptor (trx_gat_layer0_infer's desc) and parameters with the
 * expression that kernel evaluates (bit-identical), not read from HBM. */
typedef struct trx_gat_mid_args {
    int32_t num_graphs, nodes_per_graph, heads, channels;
    int32_t max_graph_edges;
    const void* xh;             /* bf16 [N, heads*channels] */
    const int32_t* rowptr;
    const int32_t* col;
    const float* a_edge;
    int32_t a_edge_stride, a_edge_offset;
    const float* att_src;       /* [heads*channels] */
    const float* att_dst;
    const float* bias;
    float negative_slope;
    const float* ln_weight;
    const float* ln_bias;
    float ln_eps;
    const float* desc;          /* [N, 4*l0_heads + 8] */
    int32_t l0_heads;
    const float* l0_w0;         /* layer 0: [heads*channels, 4] lin.weight (the same float32 buffers */
    const float* l0_bias;       /*   trx_gat_layer0_infer read)                                      */
    const float* l0_ln_weight;
    const float* l0_ln_bias;
    const float* l0_wp;         /* [heads*channels, 4] input_proj.weight */
    const float* l0_bp;
    float* out_f32;             /* [N, heads*channels] or NULL */
    void* out_bf16;             /* [N, heads*channels] bf16 or NULL */
} trx_gat_mid_args;
int trx_gat_mid_infer(const trx_gat_mid_args* a, void* stream);
/* u [2*heads*4] float32 and stats [heads*24 + 2] float64 of one weight set:
 * per head h (channels c of h, in order) s_h = sum W0[c], t_h = sum b_c W0[c],
 * G_h = sum W0[c] W0[c]^T (4x4 row-major) at stats[24h + 0/4/8], then
 * sum b_c and sum b_c^2.  heads + 1 workgroups, fixed-order float64 sums. */
int trx_gat_layer0_prepare(int32_t heads, int32_t channels, const float* w0, const float* att_src,
                           const float* att_dst, const float* bias, float* u, double* stats, void* stream);

/* Edge scorer of Actor/Critic (src/rl/sac.py:42-46, 69-78) for regular
 * batches, one workgroup per graph:
 *   z = ((p[src,:H] + p[dst,H:]) + ea @ we^T) + c[graph]      (fp32)
 *   logit = relu(z) . w2 + b2                                   (fp32)
 * p [N, 2H] bf16 = node_emb @ [W_src; W_dst]^T (the bf16 GEMM), c [B, H] fp32 =
 * bf16(ctx @ W_ctx^T) + b1; everything after those products is fp32.
 * softmax != 0: logits masked (mask <= 0 -> -1e9) and soft-maxed per graph
 * (Actor probs); else raw logits (Critic Q).  hidden <= 512, edge_dim <= 8,
 * nodes_per_graph * hidden <= 32768 (the graph's p rows are staged in LDS). */
typedef struct trx_edge_head_args {
    int32_t num_graphs, edges_per_graph, hidden, edge_dim;
    const int32_t* src;         /* [B*E] global node ids */
    const int32_t* dst;
    const void* p;              /* bf16 [N, 2*hidden] */
    const float* c;             /* [B, hidden] */
    const float* ea;            /* [B*E, edge_dim] normalised edge features */
    const float* we;            /* [hidden, edge_dim] */
    const float* w2;            /* [hidden] */
    const float* b2;            /* [1] (device: no host read) */
    const float* mask;          /* [B*E] (softmax only) */
    int32_t softmax;
    float* out;                 /* [B*E] probs (softmax) or logits */
    float* logits;              /* [B*E] masked logits when softmax, or NULL */
    int32_t nodes_per_graph;    /* n: graph g's links join nodes [g*n, g*n + n) (regular batch) */
    const float* u;             /* [B] uniforms in [0,1) or NULL: with softmax != 0, also draw one link
                                   per graph from the probs (inverse CDF: the first link whose running
                                   sum of exp(logit - max) exceeds u * total) into `action` */
    int64_t* action;            /* [B] drawn graph-local link (u != NULL) */
    int32_t exact;              /* ABI 10: 1 = p is float [N, 2*hidden] (and the backward's grad_p float) */
} trx_edge_head_args;
int trx_edge_head_infer(const trx_edge_head_args* a, void* stream);
/* ABI 11: `count` networks in one launch (same num_graphs, edges_per_graph,
 * nodes_per_graph, hidden, edge_dim, exact, softmax and draw). */
int trx_edge_head_infer_multi(const trx_edge_head_args* a, int32_t count, void* stream);

/* Fused tail of the Actor/Critic inference pass (ABI 8): the last GATConv of
 * GATEncoder (src/models/gat_encoder.py:22-25, 47-53: heads 1, concat False,
 * LayerNorm, ELU, global mean|max pool) followed by the edge scorer of
 * trx_edge_head_infer (src/rl/sac.py:38-46, 69-78), four graphs per workgroup:
 *   xh = bf16(x @ w_lin^T)                  (bf16 MFMA, fp32 accumulation)
 *   attention / aggregation / bias / LayerNorm / ELU / pool as trx_gat_layer_infer
 *   p  = bf16(bf16(y) @ w_nodes^T), c = bf16(bf16(ctx) @ w_ctx^T) + b1   (MFMA)
 *   logits / masked softmax / draw as trx_edge_head_infer
 * Replaces lin GEMM + trx_gat_layer_infer + two GEMMs + trx_edge_head_infer of
 * the last layer; outputs equal theirs up to the GEMMs' accumulation order.
 * channels == hidden == 256, in_dim % 128 == 0 (<= 8192), nodes_per_graph
 * 1..32, edges_per_graph 1..128, max_graph_edges 1..256, edge_dim 1..8.     */
typedef struct trx_gat_tail_args {
    int32_t num_graphs, nodes_per_graph, edges_per_graph, in_dim, channels, hidden, edge_dim, max_graph_edges;
    const void* x;              /* bf16 [N, in_dim] the previous layer's output */
    const void* w_lin;          /* bf16 [channels, in_dim] lin.weight */
    const int32_t* rowptr;      /* [N+1] CSR by destination (self loops included) */
    const int32_t* col;         /* [Et] */
    const float* a_edge;        /* [Et, a_edge_stride] edge logits in CSR order */
    int32_t a_edge_stride, a_edge_offset;
    const float* att_src;       /* [channels] */
    const float* att_dst;       /* [channels] */
    const float* bias;          /* [channels] */
    float negative_slope;
    const float* ln_weight;     /* [channels] */
    const float* ln_bias;       /* [channels] */
    float ln_eps;
    const void* w_nodes;        /* bf16 [2*hidden, channels]: rows [0, hidden) src, [hidden, 2*hidden) dst */
    const void* w_ctx;          /* bf16 [hidden, 2*channels] */
    const float* b1;            /* [hidden] */
    const int32_t* src;         /* [B*E] global node ids of the links */
    const int32_t* dst;
    const float* ea;            /* [B*E, edge_dim] normalised link features */
    const float* we;            /* [hidden, edge_dim] bf16-representable */
    const float* w2;            /* [hidden] bf16-representable */
    const float* b2;            /* [1] bf16-representable */
    const float* mask;          /* [B*E] (softmax only) */
    int32_t softmax;            /* as trx_edge_head_args */
    float* out;                 /* [B*E] probs (softmax) or logits */
    float* logits;              /* [B*E] masked logits (softmax) or NULL */
    const float* u;             /* [B] uniforms or NULL: draw one link per graph into action */
    int64_t* action;            /* [B] */
    void* emb_bf16;             /* [N, channels] bf16 node embeddings, or NULL */
    float* pool;                /* [B, 2*channels] mean | max, or NULL */
} trx_gat_tail_args;
int trx_gat_tail_infer(const trx_gat_tail_args* a, void* stream);
/* Backward of the edge scorer's logits (softmax = 0) for training, one
 * workgroup per graph (hidden <= 256): from grad_logits [B*E] float32 and the
 * same args (p, c, ea, we, w2, src, dst, nodes_per_graph) it writes grad_p
 * [N, 2H] bf16 (fp32 sums over the graph's links, rounded once), grad_c
 * [B, H] float32, grad_w2_part [B, H] float32 (per-graph partial sums of the
 * 256->1 weight gradient), grad_we_part [B, H, edge_dim] float32 (per-graph
 * partial sums of the link-feature weight gradient) and grad_ea [B*E,
 * edge_dim] float32 (the link features' gradient); grad_z [B*E, H] bf16 (the
 * gradient at the link pre-activation) only when non-NULL.  fp32 after the p
 * GEMM, as the forward (and the general path of trafficrl/rl/sac.py
 * _EdgeHead.edge_scores). */
int trx_edge_head_backward(const trx_edge_head_args* a, const float* grad_logits, void* grad_p, float* grad_c,
                           void* grad_z, float* grad_w2_part, float* grad_we_part, float* grad_ea, void* stream);
/* ABI 11: trx_edge_head_backward for `count` networks in one launch; io[k]
 * holds network k's gradient buffers (the arguments of the single call).  The
 * networks must agree on num_graphs, edges_per_graph, nodes_per_graph, hidden,
 * edge_dim, exact, softmax, the presence of u and the presence of grad_z
 * (TRX_EINVAL otherwise). */
typedef struct trx_edge_head_bwd_io {
    const float* grad_logits;
    void* grad_p;
    float* grad_c;
    void* grad_z;
    float* grad_w2_part;
    float* grad_we_part;
    float* grad_ea;
} trx_edge_head_bwd_io;
int trx_edge_head_backward_multi(const trx_edge_head_args* a, const trx_edge_head_bwd_io* io, int32_t count,
                                 void* stream);

/* Input stage of Actor/Critic (src/rl/sac.py:36-37) plus every layer's edge
 * attention logits (src/models/gat_encoder.py:36-52: PyG GATConv with
 * edge_dim and add_self_loops fill_value='mean') for regular batches:
 *   x0 = LayerNorm(node_x), ea = LayerNorm(edge_x)                  (fp32)
 *   loop[i] = mean of ea over the links entering i with src != dst (0 if none)
 *   M_l[h, :] = sum_c lin_edge_l.weight[h*C + c, :] * att_edge_l[h, c]
 *   a_edge[p, off_l + h] = bf16(bf16(full[p]) . bf16(M_l[h, :]))
 * full[p] is ea of the link, or the node's loop attr, at CSR position p
 * (pos_src); off_l = heads_0 + ... + heads_{l-1}.  bf16-autocast numerics.
 * node_dim, edge_dim <= 8, num_layers <= 4, sum of heads <= 32,
 * nodes_per_graph <= 64, edges_per_graph <= 1024.                          */
#define TRX_MAX_GAT_LAYERS 4
typedef struct trx_gat_prologue_args {
    int32_t num_graphs, nodes_per_graph, edges_per_graph, node_dim, edge_dim;
    const float* node_x;        /* [B*n, node_dim] raw node features */
    const float* edge_x;        /* [B*e, edge_dim] raw link features */
    const float* node_ln_w;     /* [node_dim] */
    const float* node_ln_b;
    float node_ln_eps;
    const float* edge_ln_w;     /* [edge_dim] */
    const float* edge_ln_b;
    float edge_ln_eps;
    const int32_t* src;         /* [B*e] global node ids of the input links */
    const int32_t* dst;
    const int32_t* rowptr;      /* [N+1] CSR by destination, self loops included */
    const int32_t* pos_src;     /* [Et] per CSR position: input link id (>= 0) or -(node + 1) for a self loop */
    int32_t num_layers;
    int32_t heads[TRX_MAX_GAT_LAYERS];
    int32_t channels[TRX_MAX_GAT_LAYERS];
    const float* lin_edge_w[TRX_MAX_GAT_LAYERS];  /* [heads*channels, edge_dim] */
    const float* att_edge[TRX_MAX_GAT_LAYERS];    /* [heads*channels] */
    float* m_work;              /* [sum heads, edge_dim] scratch: the M rows */
    float* x0;                  /* out [B*n, node_dim] */
    float* ea;                  /* out [B*e, edge_dim] */
    float* a_edge;              /* out [Et, sum heads], CSR order; a graph whose CSR range references
                                   links or nodes of another graph gets NaN rows */
    int32_t exact;              /* ABI 10: 1 = M rows, link / loop features and a_edge unrounded (fp32) */
} trx_gat_prologue_args;
int trx_gat_prologue_infer(const trx_gat_prologue_args* a, void* stream);
/* ABI 11: `count` networks in one launch (same sizes, layer shapes and exact). */
int trx_gat_prologue_infer_multi(const trx_gat_prologue_args* a, int32_t count, void* stream);

/* ------------------------------------------ fused SAC-update backward
 * The SAC update (src/rl/sac.py:157-243) runs its training forwards through
 * the fused inference kernels above with the save_* outputs set; these
 * kernels are their backward (csrc/gat_train.hip), one workgroup per graph.
 *
 * trx_gat_layer_backward: a whole GATConv layer + tail of GATEncoder
 * (src/models/gat_encoder.py:36-49): activation (0 relu / 1 elu), residual
 * (0 none, 1 res input [N,F] fp32 -> g_res, 2 layer 0's bf16(x0 @ wp^T + bp)),
 * LayerNorm, bias, aggregation, edge softmax, leaky ReLU, attention dots;
 * in_dim 4 = layer 0 (xh recomputed from x0 and w0, g_x0 written), the last
 * layer may take the pooled-context gradient g_pool [B, 2F] (mean | max).
 * Inputs: gy fp32 [N,F] and/or gy_bf16 bf16 [N,F] (summed), the forward's
 * saved alpha / asd / v / stats and its output y fp32.  Outputs: g_xh bf16
 * [N,F] (gradient of the lin output, rounded once), g_res fp32 [N,F] (always
 * written: the gradient at the activation input; the residual's gradient for
 * residual 1), g_a_edge [Et, a_edge_stride] at a_edge_offset, g_x0 [N,4]
 * (in_dim 4), part [num_graphs, trx_gat_layer_backward_part_floats()]
 * per-graph partial sums: bias, ln weight, ln bias, att_src, att_dst (F each)
 * and, for in_dim 4, lin.weight (F x 4), input_proj weight (F x 4) and bias.
 * F = heads*channels in {256, 512, 1024}; sptr/spos = the same graph in CSR by
 * source (dst-CSR position of each out-edge, fixed order: deterministic).   */
typedef struct trx_gat_layer_bwd_args {
    int32_t num_graphs, nodes_per_graph, heads, channels, max_graph_edges, in_dim;
    const int32_t* rowptr;      /* [N+1] CSR by destination (self loops included) */
    const int32_t* col;         /* [Et] */
    const int32_t* sptr;        /* [N+1] CSR by source */
    const int32_t* spos;        /* [Et] dst-CSR position per source entry */
    const void* xh;             /* bf16 [N, F] lin output (in_dim 0) */
    const float* x0;            /* [N, in_dim] (in_dim 4) */
    const float* w0;            /* [F, in_dim] bf16-rounded lin.weight (in_dim 4) */
    const float* a_edge;        /* [Et, a_edge_stride] forward edge logits */
    int32_t a_edge_stride, a_edge_offset;
    const float* att_src;       /* [F] */
    const float* att_dst;       /* [F] */
    const float* ln_weight;     /* [F] */
    float negative_slope;
    int32_t activation, residual;
    const float* wp;            /* [F, in_dim] bf16-rounded input_proj weight (residual 2) */
    const float* alpha;         /* saved by the forward: [Et, heads] */
    const float* asd;           /* [N, 2*heads] */
    const float* v;             /* [N, F] */
    const float* stats;         /* [N, 2] */
    const float* y;             /* [N, F] forward output (fp32) */
    const float* gy;            /* [N, F] or NULL */
    const void* gy_bf16;        /* bf16 [N, F] or NULL */
    const float* g_pool;        /* [B, 2F] or NULL */
    void* g_xh;                 /* bf16 [N, F] */
    float* g_res;               /* [N, F] */
    float* g_x0;                /* [N, in_dim] (in_dim 4) */
    float* g_a_edge;            /* [Et, a_edge_stride] */
    float* part;                /* [num_graphs, part_floats] */
    int32_t exact;              /* ABI 10: 1 = backward of the exact forward: xh and g_xh float [N, F],
                                   w0 / wp unrounded, no bf16 rounding anywhere (at heads*channels 1024 xh
                                   is read from global memory, layer 0 recomputes it) */
} trx_gat_layer_bwd_args;
int trx_gat_layer_backward(const trx_gat_layer_bwd_args* a, void* stream);
/* ABI 11: `count` networks in one launch (same sizes, in_dim, residual,
 * activation, exact and pooling). */
int trx_gat_layer_backward_multi(const trx_gat_layer_bwd_args* a, int32_t count, void* stream);
int64_t trx_gat_layer_backward_part_floats(int32_t heads, int32_t channels, int32_t in_dim);
/* out[k] = sum over r < rows (ascending) of part[r * stride + k], k < width. */
int trx_partial_sum(const float* part, int32_t rows, int32_t width, int64_t stride, float* out, void* stream);
/* ABI 10: up to TRX_MAX_PSUM such column sums (same rows) in one launch, same
 * order per column; out index k -> out + (k / out_cols) * out_ld + k % out_cols
 * when out_cols > 0 (a column block of a larger matrix), else out + k. */
#define TRX_MAX_PSUM 32
typedef struct trx_psum_list {
    int32_t count, rows;
    int32_t width[TRX_MAX_PSUM];
    int32_t out_cols[TRX_MAX_PSUM];
    int64_t stride[TRX_MAX_PSUM];
    int64_t out_ld[TRX_MAX_PSUM];
    const float* part[TRX_MAX_PSUM];
    float* out[TRX_MAX_PSUM];
} trx_psum_list;
int trx_partial_sum_multi(const trx_psum_list* l, void* stream);

/* trx_gat_prologue_backward: backward of trx_gat_prologue_infer (input
 * LayerNorms, PyG mean self-loop attrs, every layer's a_edge) from g_a_edge
 * [Et, A] (A = sum of heads), g_x0 [N, node_dim] and the edge head's link-
 * feature gradient g_ea_head [B*e, edge_dim] (or NULL).  part [num_graphs,
 * 8A + 32]: rows of 8 floats -- dL/dM_k (k < A, the bf16-rounded M rows of
 * the forward's m_work), edge LN weight, edge LN bias, node LN weight, node
 * LN bias (node_dim / edge_dim <= 8).                                       */
typedef struct trx_gat_prologue_bwd_args {
    int32_t num_graphs, nodes_per_graph, edges_per_graph, node_dim, edge_dim, A;
    const float* node_x;
    const float* edge_x;
    const float* node_ln_w;
    const float* node_ln_b;
    float node_ln_eps;
    const float* edge_ln_w;
    const float* edge_ln_b;
    float edge_ln_eps;
    const int32_t* src;
    const int32_t* dst;
    const int32_t* rowptr;
    const int32_t* pos_src;
    const float* m_work;        /* [A, edge_dim] the forward's M rows */
    const float* g_a_edge;      /* [Et, A] */
    const float* g_x0;          /* [N, node_dim] */
    const float* g_ea_head;     /* [B*e, edge_dim] or NULL */
    float* part;                /* [num_graphs, 8A + 32] */
    int32_t exact;              /* ABI 10: backward of the exact prologue (no bf16 rounding) */
} trx_gat_prologue_bwd_args;
int trx_gat_prologue_backward(const trx_gat_prologue_bwd_args* a, void* stream);
/* ABI 11: `count` networks in one launch (same sizes and exact). */
int trx_gat_prologue_backward_multi(const trx_gat_prologue_bwd_args* a, int32_t count, void* stream);
/* Backward of every layer's edge-attention rows M (trx_gat_prologue_infer's
 * M_l[h, :] = sum_c lin_edge_l.weight[h*C + c, :] * att_edge_l[h, c]; PyG
 * GATConv's lin_edge + att_edge, src/models/gat_encoder.py:22-25) from
 * g_m [sum heads, g_m_stride] (trx_gat_prologue_backward's summed rows):
 * out holds, per layer in order, g_lin_edge [heads*channels, edge_dim] then
 * g_att_edge [heads*channels] (ABI 8; reads num_layers, heads, channels,
 * edge_dim, lin_edge_w, att_edge of the args).                             */
int trx_edge_att_weights_backward(const trx_gat_prologue_args* a, const float* g_m, int32_t g_m_stride, float* out,
                                  void* stream);

/* trx_sac_loss: DiscreteSAC.update's losses (src/rl/sac.py:184-219) for B
 * graphs of e links (e <= 256) and their gradients: soft V target from the
 * next-state actor probs and target critics, the PER-weighted twin-Q MSE
 * (dL/dq1, dL/dq2 [B*e], non-zero at the taken action), the actor loss through
 * the masked softmax of the raw logits (dL/dlogits), the alpha loss
 * (dL/dlog_alpha).  out[8]: critic_loss, actor_loss, alpha_loss, entropy,
 * q_taken, q_mean, logp_mean, alpha; td_error [B] = |target - q1|.
 * target_entropy_given = 0: target entropy = ratio * mean log(valid + 1e-8). */
typedef struct trx_sac_loss_args {
    int32_t num_graphs, edges_per_graph;
    const float* next_probs;    /* [B*e] */
    const float* qt1;           /* [B*e] target critics */
    const float* qt2;
    const float* reward;        /* [B] */
    const float* done;          /* [B] */
    const float* q1;            /* [B*e] critics */
    const float* q2;
    const float* logits;        /* [B*e] actor raw logits */
    const float* mask;          /* [B*e] action mask */
    const int64_t* action;      /* [B] graph-local link */
    const float* weights;       /* [B] PER importance weights */
    const float* log_alpha;     /* [1] */
    float gamma, target_entropy, target_entropy_ratio;
    int32_t target_entropy_given;
    float* g_q1;                /* [B*e] */
    float* g_q2;
    float* g_logits;
    float* td_error;            /* [B] */
    float* part;                /* [B, 8] scratch */
    float* out;                 /* [8] */
    float* g_log_alpha;         /* [1] */
} trx_sac_loss_args;
int trx_sac_loss(const trx_sac_loss_args* a, void* stream);

/* trx_sac_adam: DiscreteSAC.apply_gradients (src/rl/sac.py:224-263) after
 * the gradients of one update sit in one flat buffer: clip_grad_norm_ per
 * optimizer group (0 critics, 1 actor, 2 log_alpha), the three Adam steps
 * (torch.optim.Adam, no weight decay), the log_alpha clamps and the Polyak
 * update of the target critics, in three launches.  Segment k: parameter
 * p (n floats), gradient at g_base + goff, moments at m / v + moff, Polyak
 * target t (or NULL), group.  blocks: (segment, begin, end) chunks of one
 * segment each (the host splits tensors into <= 8192-float chunks).  step[3]
 * is incremented on the device (graph-capturable). */
typedef struct trx_adam_seg {
    float* p;
    float* t;
    int64_t goff, moff, n;
    int32_t group, _pad;
} trx_adam_seg;
typedef struct trx_adam_block {
    int32_t seg, begin, end, _pad;
} trx_adam_block;
typedef struct trx_adam_args {
    const trx_adam_seg* segs;     /* device [nseg] */
    const trx_adam_block* blocks; /* device [nblocks] */
    int32_t nseg, nblocks;
    const float* g_base;
    float* m;                     /* [total] first moments */
    float* v;                     /* [total] second moments */
    float* partial;               /* [nblocks] scratch */
    float* step;                  /* [3] step counts */
    float* scal;                  /* [12] scratch: coef, step size, sqrt(bias correction 2), grad norm */
    float lr[3], max_norm[3];     /* max_norm <= 0: no clipping */
    float beta1, beta2, eps, tau;
    float log_alpha_min, log_alpha_max;
} trx_adam_args;
int trx_sac_adam(const trx_adam_args* a, void* stream);

/* ------------------------------------------------- prioritized replay
 * Sum tree of src/train.py:27-91 (ReplayBuffer) on the device: tree[1] is the
 * root, leaf i is tree[capacity + i], children of k are 2k, 2k+1; float64.
 * trx_per_update: tree[capacity + idx[k]] = priority[k] (priority already
 *   raised to alpha; idx distinct -- the caller keeps the last of duplicates)
 *   and every ancestor recomputed as the sum of its children.
 * trx_per_sample: for each u[k] in [0,1): r = u[k]*tree[1], descend with
 *   `r <= tree[left] ? left : (r -= tree[left], right)` (train.py:67-79);
 *   out_idx[k] = leaf - capacity, out_priority[k] = tree[leaf]. */
int trx_per_update(double* tree, int64_t capacity, const int64_t* idx, const double* priority, int32_t n,
                   void* stream);
int trx_per_sample(const double* tree, int64_t capacity, const double* u, int32_t n, int64_t* out_idx,
                   double* out_priority, void* stream);
/* trx_per_update for the contiguous leaves lo .. lo+n-1 (lo + n <= capacity):
 * the ring-buffer add of n new transitions; same tree values as trx_per_update
 * with idx = lo + k, each touched ancestor recomputed once per level.      */
int trx_per_update_range(double* tree, int64_t capacity, int64_t lo, const double* priority, int32_t n,
                         void* stream);
/* The ring add of n new transitions at leaves lo .. lo+n-1 (lo + n <= capacity)
 * as n sequential reference adds (src/train.py:50-58): leaf k = (max_p + eps *
 * (k+1)) ** alpha with max_p = *max_priority on entry; *max_priority becomes
 * max_p + eps * n.  One launch (the ancestors as in trx_per_update_range).  */
int trx_per_add_range(double* tree, int64_t capacity, int64_t lo, int32_t n, double* max_priority, double eps,
                      double alpha, void* stream);

/* The reference's float32 sum tree, bit for bit (src/train.py:27-91 under
 * numpy >= 2 scalar rules): _set_priority adds the float32 delta fl32(p) - leaf
 * to the leaf and to each ancestor in sequence (train.py:43-48); *max_priority
 * is the reference's float64 max_priority.
 * trx_per32_add_range: n sequential ReplayBuffer.add() calls at ring slots
 *   lo .. lo+n-1 (lo + n <= capacity; replaces train.py:50-59): priority_k =
 *   max_p + eps (float64, accumulated one add at a time), p_k = priority_k **
 *   alpha.
 * trx_per32_update: ReplayBuffer.update_priorities(idx, td_error) (train.py:
 *   86-91), entries applied in order (a repeated idx sees the value left by
 *   its earlier occurrences); td_error is float64 (the reference's .tolist()
 *   of the float32 TD errors).  O(n^2) in LDS per 2048-entry chunk.
 * trx_per32_sample: the descent of ReplayBuffer.sample (train.py:67-79) for
 *   u[k] in [0,1): r = fl32(u[k] * tree[1]), then float32 `r <= tree[left] ?
 *   left : (r -= tree[left], right)`; out_priority[k] = tree[leaf].        */
int trx_per32_add_range(float* tree, int64_t capacity, int64_t lo, int32_t n, double* max_priority, double eps,
                        double alpha, void* stream);
int trx_per32_update(float* tree, int64_t capacity, const int64_t* idx, const double* td_error, int32_t n,
                     double* max_priority, double eps, double alpha, void* stream);
int trx_per32_sample(const float* tree, int64_t capacity, const double* u, int32_t n, int64_t* out_idx,
                     float* out_priority, void* stream);
/* trx_per32_sample_weighted: trx_per32_sample plus ReplayBuffer.sample's
 *   importance weights (train.py:80-82) in float32, as the device path states
 *   them: w_k = (fl32(*size) * (out_priority[k] / tree[1])) ** (float)-beta,
 *   then w /= max(w) when that max is > 0 -- one launch (one workgroup) instead
 *   of the sample kernel and eight elementwise / reduction launches.  *size is
 *   the buffer's current fill (float64, device memory, read at run time so a
 *   captured graph sees the live value).                                    */
int trx_per32_sample_weighted(const float* tree, int64_t capacity, const double* u, int32_t n, const double* size,
                              double beta, int64_t* out_idx, float* out_priority, float* out_weight, void* stream);

/* ------------------------------------------------------- damage draws (host)
 * RepairEnv.reset's damage draw (src/env/repair_env.py:167-192) for num_envs
 * envs, each with its own numpy Generator (PCG64) passed by state and updated
 * in place -- the masks and the generator states afterwards are numpy's own:
 * up to max_tries draws of rng.choice(num_edges, count, replace=False) until
 * the active links' DiGraph (one arc per (u, v), the last link added for it,
 * repair_env.py:107-109) is strongly connected, else one more draw unchecked.
 * out_mask: float32 [num_envs, num_edges], 1 = damaged.  Host memory only; no
 * device needed.  nthreads <= 0: min(16, hardware threads).
 * The state fields are numpy's bit_generator.state: state/inc split in 64-bit
 * halves, has_uint32/uinteger its buffered half-draw.  num_edges <= 10000
 * (numpy's Floyd branch of choice). */
typedef struct trx_pcg64 {
    uint64_t state_hi, state_lo, inc_hi, inc_lo;
    uint32_t has_uint32, uinteger;
} trx_pcg64;
int trx_damage_sample(int32_t num_nodes, int32_t num_edges, const int32_t* src, const int32_t* dst, int32_t count,
                      int32_t max_tries, int32_t num_envs, trx_pcg64* rngs, float* out_mask, int32_t nthreads);

/* ------------------------------------------------ GAT layer tail (training)
 * The autograd path's post-aggregation tail of a GATEncoder layer
 * (src/models/gat_encoder.py:40-49): z = out + bias, h = LayerNorm(z; ln_w,
 * ln_b, eps) (biased variance, like torch), then act 0: y = relu(h + res)
 * (middle layers; res float32 or bfloat16 per res_dtype) or act 1: y = elu(h)
 * (last layer).  out, y: float32 [N, F]; stats: float32 [N, 2] (mean, rstd)
 * saved for the backward.  Backward: grad_out = dL/dz [N, F] float32,
 * grad_res = dL/dres [N, F] in res_dtype (act 0), grads = [3, F] float32 sums
 * over rows of dL/dz (bias), dL/dh * xhat (ln_w) and dL/dh (ln_b), reduced
 * in a fixed order from workspace (trx_layer_tail_workspace_floats).  F <= 1024,
 * F % 4 == 0.                                                              */
int trx_layer_tail_forward(int32_t N, int32_t F, int32_t act, int32_t res_dtype, const float* out, const float* bias,
                           const float* ln_w, const float* ln_b, float eps, const void* res, float* y, float* stats,
                           void* stream);
int64_t trx_layer_tail_workspace_floats(int32_t N, int32_t F);
int trx_layer_tail_backward(int32_t N, int32_t F, int32_t act, int32_t res_dtype, const float* grad_y,
                            const float* out, const float* bias, const float* ln_w, const float* y, const float* stats,
                            float* grad_out, void* grad_res, float* grads, float* workspace, void* stream);

/* -------------------------------------------- GAT attention dot products
 * Training-path a_src[i,h] = <xh[i, h*C:(h+1)*C], att_src[h*C:(h+1)*C]> and
 * a_dst likewise (PyG GATConv inside src/models/gat_encoder.py), float32
 * [N, H].  xh [N, H*C] float32 (dtype 0) or bfloat16 (1).  Backward:
 * grad_xh [N, H*C] in xh's dtype = grad_src[i,h] att_src + grad_dst[i,h]
 * att_dst; grad_att float32 [2, H*C] (att_src, att_dst) = column sums over
 * nodes, reduced in a fixed order from workspace
 * (trx_att_dots_workspace_floats).  H <= 8, C % 4 == 0, H*C <= 1024.        */
int trx_att_dots_forward(int32_t N, int32_t H, int32_t C, const void* xh, int32_t xh_dtype, const float* att_src,
                         const float* att_dst, float* a_src, float* a_dst, void* stream);
int64_t trx_att_dots_workspace_floats(int32_t N, int32_t H, int32_t C);
int trx_att_dots_backward(int32_t N, int32_t H, int32_t C, const void* xh, int32_t xh_dtype, const float* att_src,
                          const float* att_dst, const float* grad_src, const float* grad_dst, void* grad_xh,
                          float* grad_att, float* workspace, void* stream);

/* ------------------------------------------------- narrow-row LayerNorm
 * Training-path LayerNorm of the 4-/6-wide raw node / link features
 * (src/rl/sac.py:27-28, 36-37): y = (x - mean) * rsqrt(var + eps) * w + b per row
 * (biased variance), x, y float32 [N, d], d <= 8; stats [N, 2] (mean,
 * rstd) for the backward.  Backward: grad_x [N, d]; grad_wb float32 [2, d]
 * = column sums of grad_y * xhat and grad_y, reduced in a fixed order from
 * workspace (trx_small_ln_workspace_floats).                              */
int trx_small_ln_forward(int32_t N, int32_t d, const float* x, const float* w, const float* b, float eps, float* y,
                         float* stats, void* stream);
int64_t trx_small_ln_workspace_floats(int32_t N, int32_t d);
int trx_small_ln_backward(int32_t N, int32_t d, const float* grad_y, const float* x, const float* w,
                          const float* stats, float* grad_x, float* grad_wb, float* workspace, void* stream);

/* --------------------------------------------------- global graph pooling
 * GATEncoder's readout (src/models/gat_encoder.py:50-52) for a regular batch:
 * out [B, 2F] = mean over the graph's n nodes | max over them, x [B*n, F]
 * float32; ties [B, F] = how many nodes reach the max (saved for the
 * backward, which spreads the max gradient evenly over ties like torch's
 * amax).  grad_x [B*n, F] = grad_mean / n + (x == max) * grad_max / ties.   */
int trx_graph_pool_forward(int32_t B, int32_t n, int32_t F, const float* x, float* out, float* ties, void* stream);
int trx_graph_pool_backward(int32_t B, int32_t n, int32_t F, const float* x, const float* out, const float* ties,
                            const float* grad_out, float* grad_x, void* stream);

/* ------------------------------------------------ multi-tensor bf16 round
 * dst[k] = bf16(src[k]) for up to TRX_MAX_ROUND row-major blocks in one launch
 * (src rows x cols float32 with row stride src_stride; dst rows dst_stride apart;
 * out_bf16[k] = 1: bf16 bits, 0: the bf16-rounded value as float32, 2: the
 * float32 value unrounded -- a plain strided copy, 3 (ABI 10): bf16 bits of
 * the remainder x - bf16(x), the low half of a two-term split x ~ hi + lo),
 * 16 + b (ABI 12): the three bf16 pieces of a split GEMM operand from one read
 * of x -- piece p is the remainder when bit p of b is set, else bf16(x); the
 * pieces lie cols elements apart when dst_stride > 0 (side by side in each
 * row; dst_stride >= 3 cols) and rows x cols elements apart when it is 0
 * (stacked blocks).
 * Used to prepare the small weight blocks of the fused inference passes and
 * the split operands of the update's three-product float32 GEMMs.          */
#define TRX_MAX_ROUND 48  /* ABI 11: 48 (was 16): every weight block of five networks in one launch */
typedef struct trx_round_list {
    int32_t count;
    int32_t out_bf16[TRX_MAX_ROUND];
    int64_t rows[TRX_MAX_ROUND], cols[TRX_MAX_ROUND], src_stride[TRX_MAX_ROUND];
    const float* src[TRX_MAX_ROUND];
    void* dst[TRX_MAX_ROUND];
    int64_t dst_stride[TRX_MAX_ROUND];  /* ABI 10: dst row stride in elements (0: cols, contiguous) --
                                           the column blocks of the split GEMM operands */
} trx_round_list;
int trx_bf16_round(const trx_round_list* l, void* stream);

/* ------------------------------------------------------ multi-buffer copy
 * dst[k][0:bytes[k]) = src[k][0:bytes[k]) for up to TRX_MAX_COPY device
 * buffers in one launch (non-overlapping).  The trainer's replay-ring writes
 * (src/train.py:27-58 ReplayBuffer.add, vectorised over the envs).         */
#define TRX_MAX_COPY 16
typedef struct trx_copy_list {
    int32_t count, _pad;
    int64_t bytes[TRX_MAX_COPY];
    const void* src[TRX_MAX_COPY];
    void* dst[TRX_MAX_COPY];
} trx_copy_list;
int trx_multi_copy(const trx_copy_list* l, void* stream);
/* Row gather: for r < nrows, dst[k] bytes [r*bytes[k], (r+1)*bytes[k]) =
 * src[k] bytes [idx[r]*bytes[k], ...) -- bytes[k] is the ROW size here; the
 * caller guarantees idx[r] is a valid row of every src[k].  The replay
 * sample's field gathers (src/train.py:83 `[self.data[i] for i in indices]`)
 * in one launch.                                                          */
int trx_multi_gather(const trx_copy_list* l, const int64_t* idx, int32_t nrows, void* stream);

/* --------------------------------------------- trainer episode bookkeeping
 * One vector step of src/train.py's per-env bookkeeping (916-935) for all envs:
 * ep_len += 1; scaled = reward * reward_scale (float64; scaled_f32 its float32
 * replay copy); done_f32 = done; ep_reward += scaled; ep_tstt_sum += tstt;
 * ep_auc += 0.5 * (ep_prev_tstt + tstt) * (ep_len > 1); ep_prev_tstt = tstt;
 * finished = done | (max_steps > 0 && ep_len >= max_steps).            */
int trx_episode_step(int32_t num_envs, const double* reward, const uint8_t* done, const double* tstt,
                     double reward_scale, int64_t max_steps, double* scaled, float* scaled_f32, float* done_f32,
                     double* ep_reward, double* ep_tstt_sum, double* ep_auc, double* ep_prev_tstt, int64_t* ep_len,
                     uint8_t* finished, void* stream);

/* ------------------------------------------------------ graph support
 * Rewrites every memset node of a captured, not yet instantiated hipGraph_t
 * (passed as void*) into an equivalent fill-kernel node with the same
 * dependencies.  Works around ROCm 7.2's packet-capture replay of small
 * memset nodes (torch's reduction semaphores), see csrc/graph_patch.hip.
 * Used by the trainer's HIP-graph SAC update (train.py:GraphedUpdate); the
 * reference has no counterpart (its update is eager, src/rl/sac.py:157-263). */
int trx_graph_patch_memsets(void* hip_graph, int32_t* n_patched);

#ifdef __cplusplus
}
#endif
#endif /* TRAFFICRL_H */

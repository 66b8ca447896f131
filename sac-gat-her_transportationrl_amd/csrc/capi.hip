// capi.hip -- C ABI of libtrafficrl.so (declared in include/trafficrl.h).
//
// Host-side runtime: validates inputs the way the reference raises, builds the
// immutable device graph (scipy-ordered CSR, dense demand table, edge-id
// table) once, and launches the stream-ordered gfx950 kernels.  No call but
// trx_graph_create/destroy allocates or synchronises.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "trx_internal.h"

using trx::DevGraph;

struct trx_graph {
    DevGraph dg;
    int device;
    std::vector<void*> allocs;
};

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace

int trx::set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

namespace {

template <typename T>
int upload(trx_graph* g, const std::vector<T>& host, const T** out) {
    void* d = nullptr;
    size_t bytes = host.size() * sizeof(T);
    if (bytes == 0) bytes = sizeof(T);
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) return fail(TRX_EHIP, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    g->allocs.push_back(d);
    if (!host.empty()) {
        e = hipMemcpy(d, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) return fail(TRX_EHIP, "hipMemcpy: %s", hipGetErrorString(e));
    }
    *out = static_cast<const T*>(d);
    return TRX_OK;
}

int check_params(const trx_params* p) {
    if (!p) return fail(TRX_EINVAL, "params is NULL");
    if (p->iters <= 0) return fail(TRX_EINVAL, "assignment_iters must be > 0 to update TSTT.");  // repair_env.py:300-301
    if (p->method < TRX_METHOD_MSA || p->method > TRX_METHOD_GP)
        return fail(TRX_EINVAL, "unsupported assignment_method %d", p->method);
    if (p->method == TRX_METHOD_GP && (p->gp_keep_paths < 1 || p->gp_keep_paths > trx::kGpMaxPaths - 1))
        return fail(TRX_EUNSUP, "gp_keep_paths %d: this build supports 1..%d", p->gp_keep_paths,
                    trx::kGpMaxPaths - 1);
    if (!(p->bpr_beta >= 0.0f && p->bpr_beta <= 16.0f) || p->bpr_beta != std::floor(p->bpr_beta))
        return fail(TRX_EUNSUP, "bpr_beta %g: only integer BPR powers 0..16 are supported (the reference uses 4)",
                    (double)p->bpr_beta);
    if (p->reward_mode < TRX_REWARD_DELTA || p->reward_mode > TRX_REWARD_REL_IMPROVE)
        return fail(TRX_EINVAL, "unsupported reward_mode %d", p->reward_mode);
    if (p->sp_rule != TRX_SP_SCIPY && p->sp_rule != TRX_SP_TORCH)
        return fail(TRX_EINVAL, "unsupported sp_rule %d", p->sp_rule);
    return TRX_OK;
}

int check_state(const trx_state* s, bool need_initial) {
    if (!s) return fail(TRX_EINVAL, "state is NULL");
    if (!s->flow || !s->capacity || !s->damaged || !s->goal || !s->tstt || !s->unassigned)
        return fail(TRX_EINVAL, "state has a NULL required buffer");
    if (need_initial && !s->initial_tstt) return fail(TRX_EINVAL, "state.initial_tstt is NULL");
    return TRX_OK;
}

// The env kernel a (graph, params) pair runs.  TRX_KERNEL=quad forces the
// general quad kernel for both rules, TRX_KERNEL=sparse the quad-per-tree
// sparse kernel instead of the pair kernel (A/B runs, fallback tests).
enum EnvKernel { kEnvNone = 0, kEnvSparse, kEnvQuad, kEnvTorch, kEnvBig, kEnvGp, kEnvPair };

const std::string& kernel_override() {
    static const std::string k = [] {
        const char* e = getenv("TRX_KERNEL");
        return std::string(e ? e : "");
    }();
    return k;
}
bool force_quad() { return kernel_override() == "quad"; }

EnvKernel select_env_kernel(const trx::DevGraph& g, const trx_params& p) {
    const bool small = g.N <= trx::kSmallMaxNodes;
    if (p.method == TRX_METHOD_GP) return small && g.E <= 128 && g.Z <= 256 ? kEnvGp : kEnvNone;
    if (!small) return p.sp_rule == TRX_SP_SCIPY ? kEnvBig : kEnvNone;  // torch rule: N <= 32 only
    if (!force_quad()) {
        if (p.sp_rule == TRX_SP_TORCH && trx::torch_kernel_ok(g)) return kEnvTorch;
        if (p.sp_rule == TRX_SP_SCIPY && kernel_override() != "sparse" && trx::pair_ok(g, p)) return kEnvPair;
        if (p.sp_rule == TRX_SP_SCIPY && trx::sparse_ok(g, p)) return kEnvSparse;
    }
    return trx::quad_ok(g, p.sp_rule) ? kEnvQuad : kEnvNone;
}

const char* env_kernel_label(EnvKernel k) {
    switch (k) {
        case kEnvPair: return "env_kernel_pair";
        case kEnvSparse: return "env_kernel_s";
        case kEnvQuad: return "env_kernel_q";
        case kEnvTorch: return "env_kernel_t";
        case kEnvBig: return "env_kernel_big";
        case kEnvGp: return "gp_kernel";
        default: return "";
    }
}

int run(const trx_graph* g, const trx_params* p, int32_t B, trx_state* s, int mode, const int32_t* action,
        double* reward, uint8_t* done, uint8_t* valid, const uint8_t* env_mask, void* ws, void* stream) {
    int rc;
    if (!g) return fail(TRX_EINVAL, "graph is NULL");
    if ((rc = check_params(p)) || (rc = check_state(s, mode != trx::kModeAssign))) return rc;
    if (B < 0) return fail(TRX_EINVAL, "num_envs < 0");
    if (B == 0) return TRX_OK;
    if (!ws) return fail(TRX_EINVAL, "workspace is NULL (size it with trx_workspace_bytes)");
    hipError_t e = hipSetDevice(g->device);
    if (e != hipSuccess) return fail(TRX_EHIP, "hipSetDevice: %s", hipGetErrorString(e));
    const EnvKernel k = select_env_kernel(g->dg, *p);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    switch (k) {
        case kEnvGp:
            if (!s->gp) return fail(TRX_EINVAL, "state.gp is NULL (size it with trx_gp_state_bytes)");
            e = trx::launch_gp_kernel(g->dg, *p, *s, B, mode, action, reward, done, valid, env_mask, st);
            break;
        case kEnvTorch:
            e = trx::launch_env_kernel_torch(g->dg, *p, *s, B, mode, action, reward, done, valid, env_mask, st);
            break;
        case kEnvSparse:
            e = trx::launch_env_kernel_sparse(g->dg, *p, *s, B, mode, action, reward, done, valid, env_mask, ws, st);
            break;
        case kEnvPair:
            e = trx::launch_env_kernel_pair(g->dg, *p, *s, B, mode, action, reward, done, valid, env_mask, st);
            break;
        case kEnvQuad:
            e = trx::launch_env_kernel_quad(g->dg, *p, *s, B, mode, action, reward, done, valid, env_mask, st);
            break;
        case kEnvBig:
            e = trx::launch_env_kernel_big(g->dg, *p, *s, B, mode, action, reward, done, valid, env_mask, ws, st);
            break;
        default:
            if (p->method == TRX_METHOD_GP)
                return fail(TRX_EUNSUP, "GP assignment supports N <= %d, E <= 128 (got N=%d E=%d)",
                            trx::kSmallMaxNodes, g->dg.N, g->dg.E);
            if (p->sp_rule == TRX_SP_TORCH && g->dg.N > trx::kSmallMaxNodes)
                return fail(TRX_EUNSUP, "sp_rule TORCH (all-pairs Floyd-Warshall) supports N <= %d (got N=%d)",
                            trx::kSmallMaxNodes, g->dg.N);
            return fail(TRX_EUNSUP, "graph (N=%d, E=%d) exceeds every env kernel's LDS budget", g->dg.N, g->dg.E);
    }
    if (e != hipSuccess) return fail(TRX_EHIP, "kernel launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

}  // namespace

extern "C" {

int32_t trx_abi_version(void) { return TRX_ABI_VERSION; }

const char* trx_last_error(void) { return g_err; }

int trx_graph_create(int32_t N, int32_t E, const int32_t* src, const int32_t* dst, const float* t0,
                     const float* cap0, int32_t P, const int32_t* od_o, const int32_t* od_d, const double* od_v,
                     trx_graph** out) {
    if (!out) return fail(TRX_EINVAL, "out is NULL");
    *out = nullptr;
    if (N <= 0 || E < 0 || P < 0) return fail(TRX_EINVAL, "bad sizes N=%d E=%d P=%d", N, E, P);
    if (E > 0 && (!src || !dst || !t0 || !cap0)) return fail(TRX_EINVAL, "NULL edge array");
    if (P > 0 && (!od_o || !od_d || !od_v)) return fail(TRX_EINVAL, "NULL OD array");
    if (N > trx::kBigMaxNodes)
        return fail(TRX_EUNSUP, "graph has %d nodes; this build supports <= %d", N, trx::kBigMaxNodes);
    if (E > 32767) return fail(TRX_EUNSUP, "graph has %d links; this build supports <= 32767", E);
    const bool small = N <= trx::kSmallMaxNodes;
    const int NP = !small ? 0 : N <= 8 ? 8 : N <= 16 ? 16 : N <= 24 ? 24 : 32;

    for (int e = 0; e < E; ++e) {
        if (src[e] < 0 || src[e] >= N || dst[e] < 0 || dst[e] >= N)
            return fail(TRX_EINVAL, "edge %d endpoint out of range", e);
        if (!(t0[e] > 0.0f) || !std::isfinite(t0[e]))
            return fail(TRX_EUNSUP, "edge %d has non-positive free-flow time %g", e, (double)t0[e]);
    }
    // scipy CSR: rows by source, columns ascending (csr_matrix((w,(row,col))))
    std::vector<int32_t> order(E);
    for (int e = 0; e < E; ++e) order[e] = e;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        return src[a] != src[b] ? src[a] < src[b] : dst[a] < dst[b];
    });
    std::vector<int32_t> indptr(N + 1, 0), indices(E), csr_eid(E);
    for (int k = 0; k < E; ++k) {
        const int e = order[k];
        if (k > 0 && src[order[k - 1]] == src[e] && dst[order[k - 1]] == dst[e])
            return fail(TRX_EUNSUP, "parallel links %d->%d (scipy csr_matrix would sum them)", src[e], dst[e]);
        indices[k] = dst[e];
        csr_eid[k] = e;
        indptr[src[e] + 1]++;
    }
    for (int u = 0; u < N; ++u) indptr[u + 1] += indptr[u];
    std::vector<int16_t> eid_of(small ? (size_t)NP * NP : 1, -1);
    if (small)
        for (int e = 0; e < E; ++e) eid_of[(size_t)src[e] * NP + dst[e]] = (int16_t)e;
    // origins = nodes with at least one OD entry (repair_env.py:490-493)
    std::vector<int> has(N, 0);
    double total = 0.0;
    for (int k = 0; k < P; ++k) {
        if (od_o[k] < 0 || od_o[k] >= N || od_d[k] < 0 || od_d[k] >= N)
            return fail(TRX_EINVAL, "OD entry %d out of range", k);
        double v = od_v[k];
        if (!(v > 0.0) || v != std::floor(v))
            return fail(TRX_EUNSUP, "OD demand %g is not a positive integer (exact fp32 AON contract)", v);
        has[od_o[k]] = 1;
        total += v;
    }
    if (total >= 16777216.0) return fail(TRX_EUNSUP, "total demand %g >= 2^24 (exact fp32 AON contract)", total);
    std::vector<int32_t> origins;
    std::vector<int> zone_of(N, -1);
    for (int u = 0; u < N; ++u)
        if (has[u]) {
            zone_of[u] = (int)origins.size();
            origins.push_back(u);
        }
    const int Z = (int)origins.size();
    if (Z == 0) return fail(TRX_EUNSUP, "no OD demand");
    std::vector<float> dem(small ? (size_t)Z * N : 1, 0.0f);
    if (small)
        for (int k = 0; k < P; ++k) dem[(size_t)zone_of[od_o[k]] * N + od_d[k]] = (float)od_v[k];
    // OD entries grouped per origin zone, dict order kept (repair_env.py:491)
    std::vector<int32_t> od_ptr(Z + 1, 0), od_dst(P > 0 ? P : 1), od_pos(Z, 0);
    std::vector<float> od_dem(P > 0 ? P : 1);
    for (int k = 0; k < P; ++k) od_ptr[zone_of[od_o[k]] + 1]++;
    for (int z = 0; z < Z; ++z) od_ptr[z + 1] += od_ptr[z];
    for (int k = 0; k < P; ++k) {
        int z = zone_of[od_o[k]];
        int at = od_ptr[z] + od_pos[z]++;
        od_dst[at] = od_d[k];
        od_dem[at] = (float)od_v[k];
    }
    // networkx node insertion order (repair_env.py:106-109)
    std::vector<int32_t> nx_order;
    std::vector<int> seen(N, 0);
    for (int e = 0; e < E; ++e)
        for (int n : {src[e], dst[e]})
            if (!seen[n]) {
                seen[n] = 1;
                nx_order.push_back(n);
            }
    for (int n = 0; n < N; ++n)
        if (!seen[n]) nx_order.push_back(n);
    // adjacency views (file order within a node) for the observation kernels
    std::vector<int32_t> out_ptr(N + 1, 0), out_dst(E > 0 ? E : 1), out_eid(E > 0 ? E : 1), in_ptr(N + 1, 0),
        in_src(E > 0 ? E : 1), in_eid(E > 0 ? E : 1);
    for (int e = 0; e < E; ++e) {
        out_ptr[src[e] + 1]++;
        in_ptr[dst[e] + 1]++;
    }
    for (int u = 0; u < N; ++u) {
        out_ptr[u + 1] += out_ptr[u];
        in_ptr[u + 1] += in_ptr[u];
    }
    {
        std::vector<int32_t> op(out_ptr.begin(), out_ptr.end() - 1), ip(in_ptr.begin(), in_ptr.end() - 1);
        for (int e = 0; e < E; ++e) {
            int a = op[src[e]]++;
            out_dst[a] = dst[e];
            out_eid[a] = e;
            int b = ip[dst[e]]++;
            in_src[b] = src[e];
            in_eid[b] = e;
        }
    }
    if (!small)
        for (int u = 0; u < N; ++u)
            if (out_ptr[u + 1] - out_ptr[u] > 64)
                return fail(TRX_EUNSUP, "node %d has %d out-links; the large-graph kernels take <= 64", u,
                            out_ptr[u + 1] - out_ptr[u]);
    // large-graph kernel: packed in-link lists.  Nodes in DFS preorder of the
    // undirected graph (neighbours ascending) are dealt to the 64 lanes in
    // contiguous chunks balanced by entry count, so consecutive nodes of a
    // lane are mostly adjacent and one Gauss-Seidel sweep carries a label
    // along the whole chunk (assign_big.hip).
    int KMAX = 0, big_g = 64;
    std::vector<int32_t> b_origin(1, 0), b_od_dst(1, 0), b_indptr(1, 0), b_indices(1, 0), b_csr_eid(1, 0);
    std::vector<int16_t> b_lsrc(1, 0);
    std::vector<uint32_t> blist(1, 0);
    std::vector<int16_t> blink(1, -1);
    if (!small) {
        std::vector<std::vector<int>> und(N);
        for (int e = 0; e < E; ++e) {
            und[src[e]].push_back(dst[e]);
            und[dst[e]].push_back(src[e]);
        }
        for (auto& a : und) {
            std::sort(a.begin(), a.end());
            a.erase(std::unique(a.begin(), a.end()), a.end());
        }
        std::vector<int32_t> perm;
        std::vector<char> vis(N, 0);
        for (int r = 0; r < N; ++r) {
            if (vis[r]) continue;
            std::vector<int> stack{r};
            while (!stack.empty()) {
                int v = stack.back();
                stack.pop_back();
                if (vis[v]) continue;
                vis[v] = 1;
                perm.push_back(v);
                for (auto it = und[v].rbegin(); it != und[v].rend(); ++it)
                    if (!vis[*it]) stack.push_back(*it);
            }
        }
        // the large-graph kernels number nodes by DFS position: a lane's chunk
        // is then a run of consecutive label slots, so the 64 lanes' LDS label
        // reads spread over the banks instead of colliding at random
        std::vector<int32_t> inv(N);
        for (int i = 0; i < N; ++i) inv[perm[i]] = i;
        b_origin.resize(Z);
        for (int z = 0; z < Z; ++z) b_origin[z] = inv[origins[z]];
        b_od_dst.resize(P > 0 ? P : 1);
        for (int q = 0; q < P; ++q) b_od_dst[q] = inv[od_dst[q]];
        b_lsrc.resize(E > 0 ? E : 1);
        for (int e = 0; e < E; ++e) b_lsrc[e] = (int16_t)inv[src[e]];
        b_indptr.assign(N + 1, 0);
        b_indices.clear();
        b_csr_eid.clear();
        for (int r = 0; r < N; ++r) {  // rows by DFS position, entries in scipy order
            const int o = perm[r];
            for (int j = indptr[o]; j < indptr[o + 1]; ++j) {
                b_indices.push_back(inv[indices[j]]);
                b_csr_eid.push_back(csr_eid[j]);
            }
            b_indptr[r + 1] = (int32_t)b_indices.size();
        }
        // chunk the DFS order over the G lanes of a tree, balanced by entry
        // count (every node owns >= 1 entry: a dummy if it has no in-link)
        static const int lanes_env = [] {
            const char* e = getenv("TRX_BIG_LANES");  // tuning knob (A/B runs): 32 or 64
            return e ? atoi(e) : 0;
        }();
        big_g = lanes_env == 64 ? 64 : lanes_env == 16 ? 16 : 32;
        auto cost = [&](int v) { return std::max(1, in_ptr[v + 1] - in_ptr[v]); };
        int tot = 0;
        for (int v = 0; v < N; ++v) tot += cost(v);
        std::vector<int> lane_start;
        for (int T = (tot + big_g - 1) / big_g;; ++T) {
            lane_start.assign(1, 0);
            int acc = 0;
            for (int i = 0; i < N; ++i) {
                if (acc > 0 && acc + cost(perm[i]) > T) {
                    lane_start.push_back(i);
                    acc = 0;
                }
                acc += cost(perm[i]);
            }
            if ((int)lane_start.size() <= big_g) {
                KMAX = T;
                break;
            }
        }
        while ((int)lane_start.size() < big_g) lane_start.push_back(N);
        lane_start.push_back(N);
        blist.assign((size_t)KMAX * big_g, 0u);
        blink.assign((size_t)KMAX * big_g, -1);
        for (int l = 0; l < big_g; ++l) {
            int k = 0;
            for (int i = lane_start[l]; i < lane_start[l + 1]; ++i) {
                const int v = perm[i];
                const int n = in_ptr[v + 1] - in_ptr[v];
                for (int q = 0; q < std::max(1, n); ++q) {
                    const int u = n ? in_src[in_ptr[v] + q] : v;
                    uint32_t word = (uint32_t)inv[u] | ((uint32_t)inv[v] << 16);
                    if (q == 0) word |= 1u << 30;
                    if (q == std::max(1, n) - 1) word |= 1u << 31;
                    blist[(size_t)k * big_g + l] = word;
                    blink[(size_t)k * big_g + l] = (int16_t)(n ? in_eid[in_ptr[v] + q] : -1);
                    ++k;
                }
            }
            // padding entries: node N (the dummy label slot, always +inf)
            for (; k < KMAX; ++k) blist[(size_t)k * big_g + l] = (uint32_t)N | ((uint32_t)N << 16) | (3u << 30);
        }
    }

    trx_graph* g = new trx_graph();
    hipError_t he = hipGetDevice(&g->device);
    if (he != hipSuccess) {
        delete g;
        return fail(TRX_EHIP, "hipGetDevice: %s", hipGetErrorString(he));
    }
    DevGraph& d = g->dg;
    d.N = N;
    d.E = E;
    d.Z = Z;
    d.NP = NP;
    d.P = P;
    d.KMAX = KMAX;
    d.big_g = big_g;
    d.total_demand = total;
    float mt = 0.f, mc = 0.f, mn = E > 0 ? t0[0] : 1.0f;
    for (int e = 0; e < E; ++e) {
        mt = std::max(mt, t0[e]);
        mc = std::max(mc, cap0[e]);
        mn = std::min(mn, t0[e]);
    }
    d.max_t0 = E > 0 ? mt : 1.0f;
    d.max_cap = E > 0 ? mc : 1.0f;
    d.min_t0 = mn;
    d.max_out_deg = d.max_in_deg = 0;
    for (int u = 0; u < N; ++u) {
        d.max_out_deg = std::max(d.max_out_deg, out_ptr[u + 1] - out_ptr[u]);
        d.max_in_deg = std::max(d.max_in_deg, in_ptr[u + 1] - in_ptr[u]);
    }
    // every origin reaches every node: link costs stay finite (a damaged link costs
    // 1e6, repair_env.py:677), so this is a property of the graph, and the pair
    // kernel's trees then scan exactly N nodes (assign_pair.hip FULL)
    d.reach_all = 0;
    if (small) {
        d.reach_all = 1;
        for (int z = 0; z < Z && d.reach_all; ++z) {
            std::vector<char> vis(N, 0);
            std::vector<int> q{origins[z]};
            vis[origins[z]] = 1;
            for (size_t h = 0; h < q.size(); ++h)
                for (int a = out_ptr[q[h]]; a < out_ptr[q[h] + 1]; ++a)
                    if (!vis[out_dst[a]]) {
                        vis[out_dst[a]] = 1;
                        q.push_back(out_dst[a]);
                    }
            if ((int)q.size() != N) d.reach_all = 0;
        }
    }
    int rc = TRX_OK;
    std::vector<int32_t> vsrc(src, src + E), vdst(dst, dst + E);
    std::vector<float> vt0(t0, t0 + E), vcap(cap0, cap0 + E);
    if ((rc = upload(g, vsrc, &d.src)) || (rc = upload(g, vdst, &d.dst)) || (rc = upload(g, vt0, &d.t0)) ||
        (rc = upload(g, vcap, &d.cap0)) || (rc = upload(g, indptr, &d.indptr)) ||
        (rc = upload(g, indices, &d.indices)) || (rc = upload(g, csr_eid, &d.csr_eid)) ||
        (rc = upload(g, eid_of, &d.eid_of)) || (rc = upload(g, dem, &d.dem)) ||
        (rc = upload(g, origins, &d.origins)) || (rc = upload(g, nx_order, &d.nx_order)) ||
        (rc = upload(g, out_ptr, &d.out_ptr)) || (rc = upload(g, out_dst, &d.out_dst)) ||
        (rc = upload(g, out_eid, &d.out_eid)) || (rc = upload(g, in_ptr, &d.in_ptr)) ||
        (rc = upload(g, in_src, &d.in_src)) || (rc = upload(g, in_eid, &d.in_eid)) ||
        (rc = upload(g, blist, &d.blist)) || (rc = upload(g, blink, &d.blink)) ||
        (rc = upload(g, od_ptr, &d.od_ptr)) || (rc = upload(g, od_dst, &d.od_dst)) ||
        (rc = upload(g, od_dem, &d.od_dem)) || (rc = upload(g, b_origin, &d.b_origin)) ||
        (rc = upload(g, b_od_dst, &d.b_od_dst)) || (rc = upload(g, b_lsrc, &d.b_lsrc)) ||
        (rc = upload(g, b_indptr, &d.b_indptr)) || (rc = upload(g, b_indices, &d.b_indices)) ||
        (rc = upload(g, b_csr_eid, &d.b_csr_eid))) {
        trx_graph_destroy(g);
        return rc;
    }
    if (!small && trx::big_waves(d) <= 0) {
        int rc2 = fail(TRX_EUNSUP, "graph (N=%d, E=%d) does not fit the large-graph kernel's LDS budget", N, E);
        trx_graph_destroy(g);
        return rc2;
    }
    *out = g;
    return TRX_OK;
}

int trx_graph_destroy(trx_graph* g) {
    if (!g) return TRX_OK;
    for (void* p : g->allocs) (void)hipFree(p);
    delete g;
    return TRX_OK;
}

int trx_graph_info(const trx_graph* g, int32_t* num_nodes, int32_t* num_edges, int32_t* num_origins,
                   double* total_demand) {
    if (!g) return fail(TRX_EINVAL, "graph is NULL");
    if (num_nodes) *num_nodes = g->dg.N;
    if (num_edges) *num_edges = g->dg.E;
    if (num_origins) *num_origins = g->dg.Z;
    if (total_demand) *total_demand = g->dg.total_demand;
    return TRX_OK;
}

int64_t trx_workspace_bytes(const trx_graph* g, int32_t num_envs) {
    if (!g || num_envs < 0) return fail(TRX_EINVAL, "bad arguments");
    // small graphs: per-env work lives in LDS; the sparse kernel's rare exact-heap
    // replays use one FibLane per tree here
    if (g->dg.N <= trx::kSmallMaxNodes)
        return (int64_t)std::max<size_t>(256, trx::sparse_workspace_bytes(g->dg, num_envs));
    // large graphs: one exact-heap scratch slot per wave (rarely touched)
    return (int64_t)std::max<size_t>(256, trx::big_workspace_bytes(g->dg, num_envs));
}

int64_t trx_gp_state_bytes(const trx_graph* g, int32_t num_envs, int32_t keep_paths) {
    if (!g || num_envs < 0) return fail(TRX_EINVAL, "bad arguments");
    if (keep_paths < 1 || keep_paths > trx::kGpMaxPaths - 1)
        return fail(TRX_EUNSUP, "gp_keep_paths %d: this build supports 1..%d", keep_paths, trx::kGpMaxPaths - 1);
    if (g->dg.N > trx::kSmallMaxNodes || g->dg.E > 128)
        return fail(TRX_EUNSUP, "GP assignment supports N <= %d, E <= 128", trx::kSmallMaxNodes);
    return (int64_t)num_envs * (int64_t)trx::gp_layout(g->dg.P, keep_paths).total;
}

const char* trx_env_kernel_name(const trx_graph* g, const trx_params* p) {
    if (!g || check_params(p)) return "";
    return env_kernel_label(select_env_kernel(g->dg, *p));
}

int trx_assign(const trx_graph* g, const trx_params* p, int32_t B, trx_state* s, const uint8_t* env_mask, void* ws,
               void* stream) {
    return run(g, p, B, s, trx::kModeAssign, nullptr, nullptr, nullptr, nullptr, env_mask, ws, stream);
}

int trx_reset(const trx_graph* g, const trx_params* p, int32_t B, trx_state* s, const uint8_t* env_mask, void* ws,
              void* stream) {
    return run(g, p, B, s, trx::kModeReset, nullptr, nullptr, nullptr, nullptr, env_mask, ws, stream);
}

int trx_step(const trx_graph* g, const trx_params* p, int32_t B, trx_state* s, const int32_t* action,
             double* reward, uint8_t* done, uint8_t* valid, void* ws, void* stream) {
    if (!action || !reward || !done || !valid) return fail(TRX_EINVAL, "step output/action buffer is NULL");
    return run(g, p, B, s, trx::kModeStep, action, reward, done, valid, nullptr, ws, stream);
}

int trx_observe(const trx_graph* g, int32_t B, const trx_state* s, float* node_x, float* edge_x, float* mask,
                void* ws, void* stream) {
    (void)ws;
    int rc;
    if (!g) return fail(TRX_EINVAL, "graph is NULL");
    if ((rc = check_state(s, false))) return rc;
    if (!node_x || !edge_x) return fail(TRX_EINVAL, "observation buffers are NULL");
    if (B <= 0) return B == 0 ? TRX_OK : fail(TRX_EINVAL, "num_envs < 0");
    hipError_t e = hipSetDevice(g->device);
    if (e != hipSuccess) return fail(TRX_EHIP, "hipSetDevice: %s", hipGetErrorString(e));
    if (g->dg.N <= trx::kSmallMaxNodes)
        e = trx::launch_observe_kernel(g->dg, B, *s, node_x, edge_x, mask, static_cast<hipStream_t>(stream));
    else
        e = trx::launch_observe_big(g->dg, B, *s, node_x, edge_x, mask, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "observe launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_forward(int32_t num_nodes, int32_t heads, int32_t channels, const int32_t* rowptr, const int32_t* src,
                    const void* xh, int32_t xh_bf16, const float* a_src, const float* a_dst, const float* a_edge,
                    float negative_slope, const float* bias, float* out, float* alpha, void* stream) {
    if (num_nodes < 0 || heads <= 0 || heads > 8 || channels <= 0 || channels % 4 != 0 || heads * channels > 2048)
        return fail(TRX_EUNSUP, "gat: need 1<=heads<=8, channels%%4==0, heads*channels<=2048 (got %d x %d)", heads,
                    channels);
    if (channels < 256 && (256 % channels) != 0)
        return fail(TRX_EUNSUP, "gat: channels < 256 must divide 256 (got %d)", channels);
    if (channels > 256 && channels % 256 != 0) return fail(TRX_EUNSUP, "gat: channels > 256 must be a multiple of 256");
    if (num_nodes == 0) return TRX_OK;
    if (!rowptr || !src || !xh || !a_src || !a_dst || !a_edge || !out || !alpha)
        return fail(TRX_EINVAL, "gat_forward: NULL buffer");
    hipError_t e = trx::launch_gat_forward(num_nodes, heads, channels, rowptr, src, xh, xh_bf16, a_src, a_dst, a_edge,
                                           negative_slope, bias, out, alpha, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_forward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_backward(int32_t num_nodes, int32_t heads, int32_t channels, const int32_t* rowptr, const int32_t* src,
                     const int32_t* sptr, const int32_t* spos, const int32_t* sdst, const void* xh, int32_t xh_bf16,
                     const float* a_src, const float* a_dst, const float* a_edge, float negative_slope,
                     const float* alpha, const float* grad_out, void* grad_xh, float* grad_a_src, float* grad_a_dst,
                     float* grad_a_edge, void* stream) {
    if (num_nodes < 0 || heads <= 0 || heads > 8 || channels <= 0 || channels % 4 != 0 || heads * channels > 2048)
        return fail(TRX_EUNSUP, "gat: unsupported heads/channels");
    if (channels < 256 && (256 % channels) != 0)
        return fail(TRX_EUNSUP, "gat: channels < 256 must divide 256 (got %d)", channels);
    if (channels > 256 && channels % 256 != 0) return fail(TRX_EUNSUP, "gat: channels > 256 must be a multiple of 256");
    if (num_nodes == 0) return TRX_OK;
    if (!rowptr || !src || !sptr || !spos || !sdst || !xh || !alpha || !grad_out || !grad_xh || !grad_a_src ||
        !grad_a_dst || !grad_a_edge)
        return fail(TRX_EINVAL, "gat_backward: NULL buffer");
    hipError_t e = trx::launch_gat_backward(num_nodes, heads, channels, rowptr, src, sptr, spos, sdst, xh, xh_bf16,
                                            a_src, a_dst, a_edge, negative_slope, alpha, grad_out, grad_xh, grad_a_src,
                                            grad_a_dst, grad_a_edge, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per_update(double* tree, int64_t capacity, const int64_t* idx, const double* priority, int32_t n,
                   void* stream) {
    if (!tree || capacity <= 0 || n < 0 || (n > 0 && (!idx || !priority))) return fail(TRX_EINVAL, "per_update args");
    hipError_t e = trx::launch_per_update(tree, capacity, idx, priority, n, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per_update launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per_update_range(double* tree, int64_t capacity, int64_t lo, const double* priority, int32_t n,
                         void* stream) {
    if (!tree || !priority || capacity < 1 || n < 0 || lo < 0 || lo + n > capacity)
        return fail(TRX_EINVAL, "per_update_range: need 0 <= lo, lo + n <= capacity");
    hipError_t e = trx::launch_per_update_range(tree, capacity, lo, priority, n, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per_update_range launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per_add_range(double* tree, int64_t capacity, int64_t lo, int32_t n, double* max_priority, double eps,
                      double alpha, void* stream) {
    if (!tree || !max_priority || capacity < 1 || n < 0 || lo < 0 || lo + n > capacity)
        return fail(TRX_EINVAL, "per_add_range: need 0 <= lo, lo + n <= capacity");
    hipError_t e = trx::launch_per_add_range(tree, capacity, lo, n, max_priority, eps, alpha,
                                             static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per_add_range launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per_sample(const double* tree, int64_t capacity, const double* u, int32_t n, int64_t* out_idx,
                   double* out_priority, void* stream) {
    if (!tree || capacity <= 0 || n < 0 || (n > 0 && (!u || !out_idx || !out_priority)))
        return fail(TRX_EINVAL, "per_sample args");
    hipError_t e = trx::launch_per_sample(tree, capacity, u, n, out_idx, out_priority, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per_sample launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per32_add_range(float* tree, int64_t capacity, int64_t lo, int32_t n, double* max_priority, double eps,
                        double alpha, void* stream) {
    if (!tree || !max_priority || capacity < 1 || n < 0 || lo < 0 || lo + n > capacity)
        return fail(TRX_EINVAL, "per32_add_range: need 0 <= lo, lo + n <= capacity");
    hipError_t e = trx::launch_per32_add_range(tree, capacity, lo, n, max_priority, eps, alpha,
                                               static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per32_add_range launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per32_update(float* tree, int64_t capacity, const int64_t* idx, const double* td_error, int32_t n,
                     double* max_priority, double eps, double alpha, void* stream) {
    if (!tree || !max_priority || capacity < 1 || n < 0 || (n > 0 && (!idx || !td_error)))
        return fail(TRX_EINVAL, "per32_update args");
    hipError_t e = trx::launch_per32_update(tree, capacity, idx, td_error, n, max_priority, eps, alpha,
                                            static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per32_update launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per32_sample(const float* tree, int64_t capacity, const double* u, int32_t n, int64_t* out_idx,
                     float* out_priority, void* stream) {
    if (!tree || capacity < 1 || n < 0 || (n > 0 && (!u || !out_idx || !out_priority)))
        return fail(TRX_EINVAL, "per32_sample args");
    hipError_t e = trx::launch_per32_sample(tree, capacity, u, n, out_idx, out_priority,
                                            static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per32_sample launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_per32_sample_weighted(const float* tree, int64_t capacity, const double* u, int32_t n, const double* size,
                              double beta, int64_t* out_idx, float* out_priority, float* out_weight, void* stream) {
    if (!tree || capacity < 1 || n < 0 || (n > 0 && (!u || !size || !out_idx || !out_priority || !out_weight)))
        return fail(TRX_EINVAL, "per32_sample_weighted args");
    hipError_t e = trx::launch_per32_sample_weighted(tree, capacity, u, n, size, beta, out_idx, out_priority,
                                                     out_weight, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "per32_sample_weighted launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_layer0_infer(const trx_gat_layer0_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "gat_layer0_infer: NULL args");
    const int HC = a->heads * a->channels;
    if (a->num_graphs < 0) return fail(TRX_EINVAL, "gat_layer0_infer: num_graphs < 0");
    if (a->nodes_per_graph < 1 || a->nodes_per_graph > 32)
        return fail(TRX_EUNSUP, "gat_layer0_infer: nodes_per_graph must be 1..32 (got %d)", a->nodes_per_graph);
    if (a->heads < 1 || a->heads > 8 || a->channels % 4 != 0 || (HC != 256 && HC != 512 && HC != 1024))
        return fail(TRX_EUNSUP, "gat_layer0_infer: heads*channels must be 256, 512 or 1024 (got %d x %d)", a->heads,
                    a->channels);
    if (a->max_graph_edges < 1 || a->max_graph_edges > 256)
        return fail(TRX_EUNSUP, "gat_layer0_infer: max_graph_edges must be 1..256");
    if (!a->x0 || !a->w0 || !a->rowptr || !a->col || !a->a_edge || !a->bias || !a->ln_weight || !a->ln_bias ||
        !a->wp || !a->bp || !a->u || !a->stats)
        return fail(TRX_EINVAL, "gat_layer0_infer: NULL input or parameter buffer");
    if (a->a_edge_stride < a->a_edge_offset + a->heads || a->a_edge_offset < 0)
        return fail(TRX_EINVAL, "gat_layer0_infer: a_edge stride/offset");
    if (!a->out_f32 && !a->out_bf16) return fail(TRX_EINVAL, "gat_layer0_infer: no output");
    const uintptr_t al16 = (uintptr_t)a->w0 | (uintptr_t)a->wp | (uintptr_t)a->bias | (uintptr_t)a->ln_weight |
                           (uintptr_t)a->ln_bias | (uintptr_t)a->bp | (uintptr_t)a->out_f32;
    if ((al16 & 15) || ((uintptr_t)a->out_bf16 & 7))
        return fail(TRX_EINVAL, "gat_layer0_infer: parameter / output buffers must be 16-byte aligned");
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_gat_layer0(*a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_layer0_infer launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_mid_infer(const trx_gat_mid_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "gat_mid_infer: NULL args");
    const int HC = a->heads * a->channels;
    if (a->num_graphs < 0) return fail(TRX_EINVAL, "gat_mid_infer: num_graphs < 0");
    if (a->nodes_per_graph < 1 || a->nodes_per_graph > 32)
        return fail(TRX_EUNSUP, "gat_mid_infer: nodes_per_graph must be 1..32 (got %d)", a->nodes_per_graph);
    if (a->channels != 256 || a->heads < 1 || a->heads > 4)
        return fail(TRX_EUNSUP, "gat_mid_infer: channels must be 256 and heads 1..4 (got %d x %d)", a->heads,
                    a->channels);
    if (a->l0_heads < 1 || a->l0_heads > 8 || HC % a->l0_heads != 0 || (HC / a->l0_heads) % 4 != 0)
        return fail(TRX_EUNSUP, "gat_mid_infer: layer-0 heads must divide heads*channels into multiples of 4");
    if (a->max_graph_edges < 1 || a->max_graph_edges > 256)
        return fail(TRX_EUNSUP, "gat_mid_infer: max_graph_edges must be 1..256");
    if (!a->xh || !a->rowptr || !a->col || !a->a_edge || !a->att_src || !a->att_dst || !a->bias || !a->ln_weight ||
        !a->ln_bias || !a->desc || !a->l0_w0 || !a->l0_bias || !a->l0_ln_weight || !a->l0_ln_bias || !a->l0_wp ||
        !a->l0_bp)
        return fail(TRX_EINVAL, "gat_mid_infer: NULL input or parameter buffer");
    if (a->a_edge_stride < a->a_edge_offset + a->heads || a->a_edge_offset < 0)
        return fail(TRX_EINVAL, "gat_mid_infer: a_edge stride/offset");
    if (!a->out_f32 && !a->out_bf16) return fail(TRX_EINVAL, "gat_mid_infer: no output");
    const uintptr_t al16 = (uintptr_t)a->xh | (uintptr_t)a->att_src | (uintptr_t)a->att_dst | (uintptr_t)a->bias |
                           (uintptr_t)a->ln_weight | (uintptr_t)a->ln_bias | (uintptr_t)a->l0_w0 |
                           (uintptr_t)a->l0_bias | (uintptr_t)a->l0_ln_weight | (uintptr_t)a->l0_ln_bias |
                           (uintptr_t)a->l0_wp | (uintptr_t)a->l0_bp | (uintptr_t)a->out_f32;
    if ((al16 & 15) || ((uintptr_t)a->out_bf16 & 7))
        return fail(TRX_EINVAL, "gat_mid_infer: buffers must be 16-byte aligned");
    if (trx::gat_mid_smem(*a) > 160 * 1024) return fail(TRX_EUNSUP, "gat_mid_infer: LDS > 160 KB");
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_gat_mid(*a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_mid_infer launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_layer0_prepare(int32_t heads, int32_t channels, const float* w0, const float* att_src,
                           const float* att_dst, const float* bias, float* u, double* stats, void* stream) {
    if (heads < 1 || heads > 8 || channels < 1) return fail(TRX_EINVAL, "gat_layer0_prepare: heads 1..8, channels");
    if (!w0 || !att_src || !att_dst || !bias || !u || !stats)
        return fail(TRX_EINVAL, "gat_layer0_prepare: NULL buffer");
    hipError_t e = trx::launch_gat_layer0_prepare(heads, channels, w0, att_src, att_dst, bias, u, stats,
                                                  static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_layer0_prepare launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

// networks of one *_multi launch: same sizes, shapes and mode (their buffers differ)
static bool same_shape(const trx_gat_layer_args& x, const trx_gat_layer_args& y) {
    return x.num_graphs == y.num_graphs &&
           x.nodes_per_graph == y.nodes_per_graph &&
           x.heads == y.heads &&
           x.channels == y.channels &&
           x.max_graph_edges == y.max_graph_edges &&
           x.in_dim == y.in_dim &&
           x.exact == y.exact &&
           (x.pool != nullptr) == (y.pool != nullptr);
}

static int check_gat_layer_infer(const trx_gat_layer_args* a) {
    if (!a) return fail(TRX_EINVAL, "gat_layer_infer: NULL args");
    const int HC = a->heads * a->channels;
    if (a->num_graphs < 0) return fail(TRX_EINVAL, "gat_layer_infer: num_graphs < 0");
    if (a->nodes_per_graph < 1 || a->nodes_per_graph > 32)
        return fail(TRX_EUNSUP, "gat_layer_infer: nodes_per_graph must be 1..32 (got %d)", a->nodes_per_graph);
    if (a->heads < 1 || a->heads > 8 || a->channels % 4 != 0 || (HC != 256 && HC != 512 && HC != 1024))
        return fail(TRX_EUNSUP, "gat_layer_infer: heads*channels must be 256, 512 or 1024 (got %d x %d)", a->heads,
                    a->channels);
    if (!a->concat && a->heads != 1) return fail(TRX_EUNSUP, "gat_layer_infer: concat=False needs heads == 1");
    if (a->max_graph_edges < 1 || a->max_graph_edges > 256)
        return fail(TRX_EUNSUP, "gat_layer_infer: max_graph_edges must be 1..256");
    if (a->in_dim != 0 && a->in_dim != 4) return fail(TRX_EUNSUP, "gat_layer_infer: in_dim must be 0 or 4");
    if (a->channels > 256 || (a->channels < 64 ? 64 % a->channels : a->channels % 64) != 0 || a->channels % 8 != 0)
        return fail(TRX_EUNSUP, "gat_layer_infer: channels must be 8..256, dividing or divisible by 64");
    if (a->in_dim == 0 ? !a->xh : (!a->x0 || !a->w0)) return fail(TRX_EINVAL, "gat_layer_infer: NULL layer input");
    if (!a->rowptr || !a->col || !a->a_edge || !a->att_src || !a->att_dst || !a->bias || !a->ln_weight ||
        !a->ln_bias)
        return fail(TRX_EINVAL, "gat_layer_infer: NULL parameter buffer");
    if (a->a_edge_stride < a->a_edge_offset + a->heads || a->a_edge_offset < 0)
        return fail(TRX_EINVAL, "gat_layer_infer: a_edge stride/offset");
    if (a->residual == 1 ? !a->res : a->residual == 2 ? (!a->wp || !a->bp || a->in_dim == 0) : a->residual != 0)
        return fail(TRX_EINVAL, "gat_layer_infer: bad residual spec");
    if (a->activation != 0 && a->activation != 1) return fail(TRX_EINVAL, "gat_layer_infer: activation 0|1");
    if (!a->out_f32 && !a->out_bf16 && !a->pool) return fail(TRX_EINVAL, "gat_layer_infer: no output");
    if (trx::gat_layer_infer_smem(*a) > 160 * 1024) return fail(TRX_EUNSUP, "gat_layer_infer: LDS > 160 KB");
    return TRX_OK;
}

int trx_gat_layer_infer_multi(const trx_gat_layer_args* a, int32_t count, void* stream) {
    if (!a || count < 1 || count > TRX_MAX_NETS)
        return fail(TRX_EINVAL, "gat_layer_infer_multi: 1..%d networks", TRX_MAX_NETS);
    for (int k = 0; k < count; ++k) {
        const int rc = check_gat_layer_infer(a + k);
        if (rc != TRX_OK) return rc;
        const trx_gat_layer_args& b = a[k];
        if (!same_shape(b, *a))
            return fail(TRX_EINVAL, "gat_layer_infer_multi: network %d differs from network 0 in shape or mode", k);
    }
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_gat_layer_infer(a, count, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_layer_infer launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_layer_infer(const trx_gat_layer_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "gat_layer_infer: NULL args");
    return trx_gat_layer_infer_multi(a, 1, stream);
}

int trx_gat_tail_infer(const trx_gat_tail_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "gat_tail_infer: NULL args");
    if (a->num_graphs < 0) return fail(TRX_EINVAL, "gat_tail_infer: num_graphs < 0");
    if (a->channels != 256 || a->hidden != 256)
        return fail(TRX_EUNSUP, "gat_tail_infer: channels and hidden must be 256 (got %d, %d)", a->channels, a->hidden);
    if (a->in_dim < 128 || a->in_dim > 8192 || a->in_dim % 128 != 0)
        return fail(TRX_EUNSUP, "gat_tail_infer: in_dim must be a multiple of 128 in 128..8192 (got %d)", a->in_dim);
    if (a->nodes_per_graph < 1 || a->nodes_per_graph > 32)
        return fail(TRX_EUNSUP, "gat_tail_infer: nodes_per_graph must be 1..32 (got %d)", a->nodes_per_graph);
    if (a->edges_per_graph < 1 || a->edges_per_graph > 128)
        return fail(TRX_EUNSUP, "gat_tail_infer: edges_per_graph must be 1..128 (got %d)", a->edges_per_graph);
    if (a->max_graph_edges < 1 || a->max_graph_edges > 256)
        return fail(TRX_EUNSUP, "gat_tail_infer: max_graph_edges must be 1..256");
    if (a->edge_dim < 1 || a->edge_dim > 8) return fail(TRX_EUNSUP, "gat_tail_infer: edge_dim must be 1..8");
    if (!a->x || !a->w_lin || !a->rowptr || !a->col || !a->a_edge || !a->att_src || !a->att_dst || !a->bias ||
        !a->ln_weight || !a->ln_bias || !a->w_nodes || !a->w_ctx || !a->b1 || !a->src || !a->dst || !a->ea ||
        !a->we || !a->w2 || !a->b2 || !a->out)
        return fail(TRX_EINVAL, "gat_tail_infer: NULL buffer");
    if (a->softmax && !a->mask) return fail(TRX_EINVAL, "gat_tail_infer: softmax needs a mask");
    if (a->u && (!a->softmax || !a->action)) return fail(TRX_EINVAL, "gat_tail_infer: a draw needs softmax and action");
    if (a->a_edge_stride < a->a_edge_offset + 1 || a->a_edge_offset < 0)
        return fail(TRX_EINVAL, "gat_tail_infer: a_edge stride/offset");
    if (trx::gat_tail_smem(*a) > 160 * 1024) return fail(TRX_EUNSUP, "gat_tail_infer: LDS > 160 KB");
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_gat_tail_infer(*a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_tail_infer launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

// networks of one *_multi launch: same sizes, shapes and mode (their buffers differ)
static bool same_shape(const trx_edge_head_args& x, const trx_edge_head_args& y) {
    return x.num_graphs == y.num_graphs &&
           x.edges_per_graph == y.edges_per_graph &&
           x.nodes_per_graph == y.nodes_per_graph &&
           x.hidden == y.hidden &&
           x.edge_dim == y.edge_dim &&
           x.exact == y.exact &&
           x.softmax == y.softmax &&
           (x.u != nullptr) == (y.u != nullptr);
}

static int check_edge_head_infer(const trx_edge_head_args* a) {
    if (!a) return fail(TRX_EINVAL, "edge_head_infer: NULL args");
    if (a->num_graphs < 0 || a->edges_per_graph < 1 || a->edges_per_graph > 4096)
        return fail(TRX_EUNSUP, "edge_head_infer: edges_per_graph must be 1..4096");
    if (a->hidden < 1 || a->hidden > 512 || a->edge_dim < 1 || a->edge_dim > 8)
        return fail(TRX_EUNSUP, "edge_head_infer: hidden 1..512, edge_dim 1..8");
    if (a->nodes_per_graph < 1 || (int64_t)a->nodes_per_graph * a->hidden > 32768)
        return fail(TRX_EUNSUP, "edge_head_infer: nodes_per_graph must be 1..32768/hidden");
    if (a->hidden % 4) return fail(TRX_EUNSUP, "edge_head_infer: hidden must be a multiple of 4");
    if (((uintptr_t)a->c | (uintptr_t)a->w2 | (uintptr_t)a->we) & 15)
        return fail(TRX_EINVAL, "edge_head_infer: c, w2 and we must be 16-byte aligned (16-byte loads)");
    if (trx::edge_head_infer_smem(*a) > 160 * 1024)
        return fail(TRX_EUNSUP, "edge_head_infer: graph too large for LDS (nodes_per_graph, edges_per_graph)");
    if (!a->src || !a->dst || !a->p || !a->c || !a->ea || !a->we || !a->w2 || !a->b2 || !a->out || (a->softmax && !a->mask))
        return fail(TRX_EINVAL, "edge_head_infer: NULL buffer");
    if (a->u && (!a->softmax || !a->action)) return fail(TRX_EINVAL, "edge_head_infer: u needs softmax and action");
    return TRX_OK;
}

int trx_edge_head_infer_multi(const trx_edge_head_args* a, int32_t count, void* stream) {
    if (!a || count < 1 || count > TRX_MAX_NETS)
        return fail(TRX_EINVAL, "edge_head_infer_multi: 1..%d networks", TRX_MAX_NETS);
    for (int k = 0; k < count; ++k) {
        const int rc = check_edge_head_infer(a + k);
        if (rc != TRX_OK) return rc;
        const trx_edge_head_args& b = a[k];
        if (!same_shape(b, *a))
            return fail(TRX_EINVAL, "edge_head_infer_multi: network %d differs from network 0 in shape or mode", k);
    }
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_edge_head_infer(a, count, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "edge_head_infer launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_edge_head_infer(const trx_edge_head_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "edge_head_infer: NULL args");
    return trx_edge_head_infer_multi(a, 1, stream);
}

static int check_edge_head_backward(const trx_edge_head_args* a, const trx_edge_head_bwd_io* io) {
    if (!a || !io) return fail(TRX_EINVAL, "edge_head_backward: NULL args");
    if (a->num_graphs < 0 || a->edges_per_graph < 1 || a->edges_per_graph > 4096)
        return fail(TRX_EUNSUP, "edge_head_backward: edges_per_graph must be 1..4096");
    if (a->hidden < 1 || a->hidden > 256 || a->hidden % 4 || a->edge_dim < 1 || a->edge_dim > 8)
        return fail(TRX_EUNSUP, "edge_head_backward: hidden 4..256 (multiple of 4), edge_dim 1..8");
    if (a->nodes_per_graph < 1 || trx::edge_head_bwd_smem(*a) > 160 * 1024)
        return fail(TRX_EUNSUP, "edge_head_backward: graph too large for LDS (nodes_per_graph, edges_per_graph)");
    if (!a->src || !a->dst || !a->p || !a->c || !a->ea || !a->we || !a->w2 || !io->grad_logits || !io->grad_p ||
        !io->grad_c || !io->grad_w2_part || !io->grad_we_part || !io->grad_ea)
        return fail(TRX_EINVAL, "edge_head_backward: NULL buffer");
    return TRX_OK;
}

// the fields every network of one backward launch must share (the kernel reads
// network 0's for the launch shape; each block's buffers are its own): those of
// the forward's same_shape plus the presence of grad_z
static bool same_shape_bwd(const trx_edge_head_args& x, const trx_edge_head_bwd_io& xio, const trx_edge_head_args& y,
                           const trx_edge_head_bwd_io& yio) {
    return same_shape(x, y) && (xio.grad_z != nullptr) == (yio.grad_z != nullptr);
}

int trx_edge_head_backward_multi(const trx_edge_head_args* a, const trx_edge_head_bwd_io* io, int32_t count,
                                 void* stream) {
    if (!a || !io || count < 1 || count > TRX_MAX_NETS)
        return fail(TRX_EINVAL, "edge_head_backward_multi: 1..%d networks", TRX_MAX_NETS);
    trx::EdgeHeadBwdItem items[TRX_MAX_NETS];
    for (int k = 0; k < count; ++k) {
        const int rc = check_edge_head_backward(a + k, io + k);
        if (rc != TRX_OK) return rc;
        if (!same_shape_bwd(a[k], io[k], *a, *io))
            return fail(TRX_EINVAL, "edge_head_backward_multi: network %d differs from network 0 in shape or mode", k);
        items[k].a = a[k];
        items[k].io = io[k];
    }
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_edge_head_bwd(items, count, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "edge_head_backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_edge_head_backward(const trx_edge_head_args* a, const float* grad_logits, void* grad_p, float* grad_c,
                           void* grad_z, float* grad_w2_part, float* grad_we_part, float* grad_ea, void* stream) {
    const trx_edge_head_bwd_io io{grad_logits, grad_p, grad_c, grad_z, grad_w2_part, grad_we_part, grad_ea};
    return trx_edge_head_backward_multi(a, &io, 1, stream);
}

static bool same_heads(const trx_gat_prologue_args& x, const trx_gat_prologue_args& y) {
    for (int l = 0; l < x.num_layers && l < TRX_MAX_GAT_LAYERS; ++l)
        if (x.heads[l] != y.heads[l] || x.channels[l] != y.channels[l]) return false;
    return true;
}

// networks of one *_multi launch: same sizes, shapes and mode (their buffers differ)
static bool same_shape(const trx_gat_prologue_args& x, const trx_gat_prologue_args& y) {
    return x.num_graphs == y.num_graphs &&
           x.nodes_per_graph == y.nodes_per_graph &&
           x.edges_per_graph == y.edges_per_graph &&
           x.node_dim == y.node_dim &&
           x.edge_dim == y.edge_dim &&
           x.num_layers == y.num_layers &&
           x.exact == y.exact &&
           same_heads(x, y);
}

static int check_gat_prologue_infer(const trx_gat_prologue_args* a) {
    if (!a) return fail(TRX_EINVAL, "gat_prologue_infer: NULL args");
    if (a->num_graphs < 0) return fail(TRX_EINVAL, "gat_prologue_infer: num_graphs < 0");
    if (a->nodes_per_graph < 1 || a->nodes_per_graph > 64 || a->edges_per_graph < 0 || a->edges_per_graph > 1024)
        return fail(TRX_EUNSUP, "gat_prologue_infer: nodes_per_graph 1..64, edges_per_graph 0..1024");
    if (a->node_dim < 1 || a->node_dim > 8 || a->edge_dim < 1 || a->edge_dim > 8)
        return fail(TRX_EUNSUP, "gat_prologue_infer: node_dim and edge_dim must be 1..8");
    if (a->num_layers < 1 || a->num_layers > TRX_MAX_GAT_LAYERS)
        return fail(TRX_EUNSUP, "gat_prologue_infer: num_layers must be 1..%d", TRX_MAX_GAT_LAYERS);
    int A = 0;
    for (int l = 0; l < a->num_layers; ++l) {
        if (a->heads[l] < 1 || a->channels[l] < 1) return fail(TRX_EINVAL, "gat_prologue_infer: heads/channels < 1");
        if (!a->lin_edge_w[l] || !a->att_edge[l]) return fail(TRX_EINVAL, "gat_prologue_infer: NULL layer weights");
        A += a->heads[l];
    }
    if (A > 32) return fail(TRX_EUNSUP, "gat_prologue_infer: sum of heads must be <= 32");
    if (!a->node_x || !a->edge_x || !a->node_ln_w || !a->node_ln_b || !a->edge_ln_w || !a->edge_ln_b || !a->src ||
        !a->dst || !a->rowptr || !a->pos_src || !a->m_work || !a->x0 || !a->ea || !a->a_edge)
        return fail(TRX_EINVAL, "gat_prologue_infer: NULL buffer");
    return TRX_OK;
}

int trx_gat_prologue_infer_multi(const trx_gat_prologue_args* a, int32_t count, void* stream) {
    if (!a || count < 1 || count > TRX_MAX_NETS)
        return fail(TRX_EINVAL, "gat_prologue_infer_multi: 1..%d networks", TRX_MAX_NETS);
    for (int k = 0; k < count; ++k) {
        const int rc = check_gat_prologue_infer(a + k);
        if (rc != TRX_OK) return rc;
        const trx_gat_prologue_args& b = a[k];
        if (!same_shape(b, *a))
            return fail(TRX_EINVAL, "gat_prologue_infer_multi: network %d differs from network 0 in shape or mode", k);
    }
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_gat_prologue(a, count, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_prologue_infer launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_prologue_infer(const trx_gat_prologue_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "gat_prologue_infer: NULL args");
    return trx_gat_prologue_infer_multi(a, 1, stream);
}

int trx_layer_tail_forward(int32_t N, int32_t F, int32_t act, int32_t res_dtype, const float* out, const float* bias,
                           const float* ln_w, const float* ln_b, float eps, const void* res, float* y, float* stats,
                           void* stream) {
    if (N < 0 || F < 4 || F > 1024 || F % 4) return fail(TRX_EUNSUP, "layer_tail: F must be 4..1024, multiple of 4");
    if (act != 0 && act != 1) return fail(TRX_EINVAL, "layer_tail: act must be 0 (relu(h + res)) or 1 (elu(h))");
    if (res_dtype != 0 && res_dtype != 1) return fail(TRX_EUNSUP, "layer_tail: res dtype 0 (float32) or 1 (bfloat16)");
    if (!out || !bias || !ln_w || !ln_b || !y || !stats || (act == 0 && !res))
        return fail(TRX_EINVAL, "layer_tail: NULL buffer");
    if (N == 0) return TRX_OK;
    hipError_t e = trx::launch_layer_tail_fwd(N, F, act, res_dtype, out, bias, ln_w, ln_b, eps, res, y, stats,
                                              static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "layer_tail forward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int64_t trx_layer_tail_workspace_floats(int32_t N, int32_t F) {
    return N < 0 || F < 0 ? -1 : (int64_t)trx::layer_tail_blocks(N) * 3 * F;
}

int trx_layer_tail_backward(int32_t N, int32_t F, int32_t act, int32_t res_dtype, const float* grad_y,
                            const float* out, const float* bias, const float* ln_w, const float* y, const float* stats,
                            float* grad_out, void* grad_res, float* grads, float* workspace, void* stream) {
    if (N < 0 || F < 4 || F > 1024 || F % 4) return fail(TRX_EUNSUP, "layer_tail: F must be 4..1024, multiple of 4");
    if (act != 0 && act != 1) return fail(TRX_EINVAL, "layer_tail: act must be 0 (relu(h + res)) or 1 (elu(h))");
    if (res_dtype != 0 && res_dtype != 1) return fail(TRX_EUNSUP, "layer_tail: res dtype 0 (float32) or 1 (bfloat16)");
    if (!grad_y || !out || !bias || !ln_w || !y || !stats || !grad_out || !grads || !workspace ||
        (act == 0 && !grad_res))
        return fail(TRX_EINVAL, "layer_tail: NULL buffer");
    if (N == 0) return TRX_OK;
    hipError_t e = trx::launch_layer_tail_bwd(N, F, act, res_dtype, grad_y, out, bias, ln_w, y, stats, grad_out,
                                              grad_res, workspace, grads, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "layer_tail backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

static int att_dots_check(int32_t N, int32_t H, int32_t C, int32_t xh_dtype) {
    if (N < 0 || H < 1 || H > 8 || C < 4 || C % 4 || H * C > 1024)
        return fail(TRX_EUNSUP, "att_dots: need 1 <= heads <= 8, channels % 4 == 0, heads*channels <= 1024");
    if (xh_dtype != 0 && xh_dtype != 1) return fail(TRX_EUNSUP, "att_dots: xh dtype 0 (float32) or 1 (bfloat16)");
    return TRX_OK;
}

int trx_att_dots_forward(int32_t N, int32_t H, int32_t C, const void* xh, int32_t xh_dtype, const float* att_src,
                         const float* att_dst, float* a_src, float* a_dst, void* stream) {
    if (int rc = att_dots_check(N, H, C, xh_dtype)) return rc;
    if (!xh || !att_src || !att_dst || !a_src || !a_dst) return fail(TRX_EINVAL, "att_dots: NULL buffer");
    if (N == 0) return TRX_OK;
    hipError_t e = trx::launch_att_dots_fwd(N, H, C, xh, xh_dtype, att_src, att_dst, a_src, a_dst,
                                            static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "att_dots forward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int64_t trx_att_dots_workspace_floats(int32_t N, int32_t H, int32_t C) {
    return N < 0 || H < 0 || C < 0 ? -1 : (int64_t)trx::att_dots_blocks(N) * 2 * H * C;
}

int trx_att_dots_backward(int32_t N, int32_t H, int32_t C, const void* xh, int32_t xh_dtype, const float* att_src,
                          const float* att_dst, const float* grad_src, const float* grad_dst, void* grad_xh,
                          float* grad_att, float* workspace, void* stream) {
    if (int rc = att_dots_check(N, H, C, xh_dtype)) return rc;
    if (!xh || !att_src || !att_dst || !grad_src || !grad_dst || !grad_xh || !grad_att || !workspace)
        return fail(TRX_EINVAL, "att_dots: NULL buffer");
    if (N == 0) return TRX_OK;
    hipError_t e = trx::launch_att_dots_bwd(N, H, C, xh, xh_dtype, att_src, att_dst, grad_src, grad_dst, grad_xh,
                                            grad_att, workspace, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "att_dots backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_small_ln_forward(int32_t N, int32_t d, const float* x, const float* w, const float* b, float eps, float* y,
                         float* stats, void* stream) {
    if (N < 0 || d < 1 || d > 8) return fail(TRX_EUNSUP, "small_ln: row width must be 1..8 (got %d)", d);
    if (!x || !w || !b || !y || !stats) return fail(TRX_EINVAL, "small_ln: NULL buffer");
    if (N == 0) return TRX_OK;
    hipError_t e = trx::launch_small_ln_fwd(N, d, x, w, b, eps, y, stats, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "small_ln forward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int64_t trx_small_ln_workspace_floats(int32_t N, int32_t d) {
    return N < 0 || d < 0 ? -1 : (int64_t)trx::small_ln_blocks(N) * 2 * d;
}

int trx_small_ln_backward(int32_t N, int32_t d, const float* grad_y, const float* x, const float* w,
                          const float* stats, float* grad_x, float* grad_wb, float* workspace, void* stream) {
    if (N < 0 || d < 1 || d > 8) return fail(TRX_EUNSUP, "small_ln: row width must be 1..8 (got %d)", d);
    if (!grad_y || !x || !w || !stats || !grad_x || !grad_wb || !workspace)
        return fail(TRX_EINVAL, "small_ln: NULL buffer");
    if (N == 0) return TRX_OK;
    hipError_t e = trx::launch_small_ln_bwd(N, d, grad_y, x, w, stats, grad_x, grad_wb, workspace,
                                            static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "small_ln backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_graph_pool_forward(int32_t B, int32_t n, int32_t F, const float* x, float* out, float* ties, void* stream) {
    if (B < 0 || n < 1 || F < 1) return fail(TRX_EINVAL, "graph_pool: B >= 0, n >= 1, F >= 1");
    if (!x || !out || !ties) return fail(TRX_EINVAL, "graph_pool: NULL buffer");
    if (B == 0) return TRX_OK;
    hipError_t e = trx::launch_graph_pool_fwd(B, n, F, x, out, ties, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "graph_pool forward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_graph_pool_backward(int32_t B, int32_t n, int32_t F, const float* x, const float* out, const float* ties,
                            const float* grad_out, float* grad_x, void* stream) {
    if (B < 0 || n < 1 || F < 1) return fail(TRX_EINVAL, "graph_pool: B >= 0, n >= 1, F >= 1");
    if (!x || !out || !ties || !grad_out || !grad_x) return fail(TRX_EINVAL, "graph_pool: NULL buffer");
    if (B == 0) return TRX_OK;
    hipError_t e = trx::launch_graph_pool_bwd(B, n, F, x, out, ties, grad_out, grad_x, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "graph_pool backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_bf16_round(const trx_round_list* l, void* stream) {
    if (!l || l->count < 0 || l->count > TRX_MAX_ROUND) return fail(TRX_EINVAL, "bf16_round: count must be 0..%d", TRX_MAX_ROUND);
    for (int k = 0; k < l->count; ++k)
        if (!l->src[k] || !l->dst[k] || l->rows[k] < 0 || l->cols[k] < 0 || l->src_stride[k] < l->cols[k] ||
            l->out_bf16[k] < 0 || (l->out_bf16[k] > 3 && (l->out_bf16[k] < 16 || l->out_bf16[k] > 23)) ||
            (l->dst_stride[k] != 0 && l->dst_stride[k] < (l->out_bf16[k] >= 16 ? 3 : 1) * l->cols[k]))
            return fail(TRX_EINVAL, "bf16_round: bad entry %d", k);
    if (l->count == 0) return TRX_OK;
    hipError_t e = trx::launch_bf16_round(*l, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "bf16_round launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_episode_step(int32_t num_envs, const double* reward, const uint8_t* done, const double* tstt,
                     double reward_scale, int64_t max_steps, double* scaled, float* scaled_f32, float* done_f32,
                     double* ep_reward, double* ep_tstt_sum, double* ep_auc, double* ep_prev_tstt, int64_t* ep_len,
                     uint8_t* finished, void* stream) {
    if (num_envs < 0 || (num_envs > 0 && (!reward || !done || !tstt || !scaled || !scaled_f32 || !done_f32 ||
                                          !ep_reward || !ep_tstt_sum || !ep_auc || !ep_prev_tstt || !ep_len ||
                                          !finished)))
        return fail(TRX_EINVAL, "episode_step args");
    hipError_t e = trx::launch_episode_step(num_envs, reward, done, tstt, reward_scale, max_steps, scaled, scaled_f32,
                                            done_f32, ep_reward, ep_tstt_sum, ep_auc, ep_prev_tstt, ep_len, finished,
                                            static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "episode_step launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_multi_gather(const trx_copy_list* l, const int64_t* idx, int32_t nrows, void* stream) {
    if (!l || l->count < 0 || l->count > TRX_MAX_COPY || nrows < 0 || (nrows > 0 && !idx))
        return fail(TRX_EINVAL, "multi_gather: count must be 0..16, nrows >= 0, idx");
    for (int k = 0; k < l->count; ++k) {
        if (!l->src[k] || !l->dst[k] || l->bytes[k] < 0) return fail(TRX_EINVAL, "multi_gather: bad entry %d", k);
    }
    hipError_t e = trx::launch_multi_gather(*l, idx, nrows, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "multi_gather launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_multi_copy(const trx_copy_list* l, void* stream) {
    if (!l || l->count < 0 || l->count > TRX_MAX_COPY) return fail(TRX_EINVAL, "multi_copy: count must be 0..16");
    for (int k = 0; k < l->count; ++k)
        if (!l->src[k] || !l->dst[k] || l->bytes[k] < 0) return fail(TRX_EINVAL, "multi_copy: bad entry %d", k);
    if (l->count == 0) return TRX_OK;
    hipError_t e = trx::launch_multi_copy(*l, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "multi_copy launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int64_t trx_gat_layer_backward_part_floats(int32_t heads, int32_t channels, int32_t in_dim) {
    if (heads < 1 || channels < 1) return fail(TRX_EINVAL, "bad heads/channels");
    return (int64_t)heads * channels * (in_dim > 0 ? 14 : 5);
}

// networks of one *_multi launch: same sizes, shapes and mode (their buffers differ)
static bool same_shape(const trx_gat_layer_bwd_args& x, const trx_gat_layer_bwd_args& y) {
    return x.num_graphs == y.num_graphs &&
           x.nodes_per_graph == y.nodes_per_graph &&
           x.heads == y.heads &&
           x.channels == y.channels &&
           x.max_graph_edges == y.max_graph_edges &&
           x.in_dim == y.in_dim &&
           x.exact == y.exact &&
           x.activation == y.activation &&
           x.residual == y.residual &&
           (x.g_pool != nullptr) == (y.g_pool != nullptr);
}

static int check_gat_layer_backward(const trx_gat_layer_bwd_args* a) {
    if (!a) return fail(TRX_EINVAL, "gat_layer_backward: NULL args");
    const int HC = a->heads * a->channels;
    if (a->num_graphs < 0 || a->nodes_per_graph < 1 || a->nodes_per_graph > 32)
        return fail(TRX_EUNSUP, "gat_layer_backward: nodes_per_graph must be 1..32");
    if (a->heads < 1 || a->heads > 8 || a->channels % 4 || (HC != 256 && HC != 512 && HC != 1024) ||
        a->channels > 256 || (a->channels < 64 ? 64 % a->channels : a->channels % 64) != 0)
        return fail(TRX_EUNSUP, "gat_layer_backward: heads*channels 256/512/1024, channels dividing or divisible by 64");
    if (a->max_graph_edges < 1 || a->max_graph_edges > 256)
        return fail(TRX_EUNSUP, "gat_layer_backward: max_graph_edges must be 1..256");
    if (a->in_dim != 0 && a->in_dim != 4) return fail(TRX_EUNSUP, "gat_layer_backward: in_dim must be 0 or 4");
    if (a->activation != 0 && a->activation != 1) return fail(TRX_EINVAL, "gat_layer_backward: activation 0|1");
    if (a->residual < 0 || a->residual > 2 || (a->residual == 2) != (a->in_dim == 4 && a->wp != nullptr))
        return fail(TRX_EINVAL, "gat_layer_backward: residual 2 needs in_dim 4 and wp (and only then)");
    if (!a->rowptr || !a->col || !a->sptr || !a->spos || (a->in_dim ? (!a->x0 || !a->w0 || !a->g_x0) : !a->xh) ||
        !a->a_edge || !a->att_src || !a->att_dst || !a->ln_weight || !a->alpha || !a->asd || !a->v || !a->stats ||
        !a->y || !a->g_xh || !a->g_res || !a->g_a_edge || !a->part || (!a->gy && !a->gy_bf16 && !a->g_pool))
        return fail(TRX_EINVAL, "gat_layer_backward: NULL buffer");
    if (a->a_edge_offset < 0 || a->a_edge_stride < a->a_edge_offset + a->heads)
        return fail(TRX_EINVAL, "gat_layer_backward: a_edge stride/offset");
    if (trx::gat_layer_bwd_smem(*a) > 160 * 1024) return fail(TRX_EUNSUP, "gat_layer_backward: LDS > 160 KB");
    return TRX_OK;
}

int trx_gat_layer_backward_multi(const trx_gat_layer_bwd_args* a, int32_t count, void* stream) {
    if (!a || count < 1 || count > TRX_MAX_NETS)
        return fail(TRX_EINVAL, "gat_layer_backward_multi: 1..%d networks", TRX_MAX_NETS);
    for (int k = 0; k < count; ++k) {
        const int rc = check_gat_layer_backward(a + k);
        if (rc != TRX_OK) return rc;
        const trx_gat_layer_bwd_args& b = a[k];
        if (!same_shape(b, *a))
            return fail(TRX_EINVAL, "gat_layer_backward_multi: network %d differs from network 0 in shape or mode", k);
    }
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_gat_layer_bwd(a, count, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_layer_backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_layer_backward(const trx_gat_layer_bwd_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "gat_layer_backward: NULL args");
    return trx_gat_layer_backward_multi(a, 1, stream);
}

int trx_partial_sum(const float* part, int32_t rows, int32_t width, int64_t stride, float* out, void* stream) {
    if (!part || !out || rows < 0 || width < 0 || stride < width) return fail(TRX_EINVAL, "partial_sum args");
    if (width == 0) return TRX_OK;
    hipError_t e = trx::launch_partial_sum(part, rows, width, stride, out, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "partial_sum launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_partial_sum_multi(const trx_psum_list* l, void* stream) {
    if (!l || l->count < 0 || l->count > TRX_MAX_PSUM || l->rows < 0)
        return fail(TRX_EINVAL, "partial_sum_multi: count 0..%d, rows >= 0", TRX_MAX_PSUM);
    for (int e = 0; e < l->count; ++e)
        if (!l->part[e] || !l->out[e] || l->width[e] < 0 || l->stride[e] < l->width[e] || l->out_cols[e] < 0 ||
            (l->out_cols[e] > 0 && l->out_ld[e] < l->out_cols[e]))
            return fail(TRX_EINVAL, "partial_sum_multi: bad entry %d", e);
    if (l->count == 0 || l->rows == 0) return TRX_OK;
    hipError_t e = trx::launch_partial_sum_multi(*l, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "partial_sum_multi launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_edge_att_weights_backward(const trx_gat_prologue_args* a, const float* g_m, int32_t g_m_stride, float* out,
                                  void* stream) {
    if (!a || !g_m || !out) return fail(TRX_EINVAL, "edge_att_weights_backward: NULL argument");
    if (a->num_layers < 1 || a->num_layers > TRX_MAX_GAT_LAYERS || a->edge_dim < 1 || a->edge_dim > 8 ||
        g_m_stride < a->edge_dim)
        return fail(TRX_EUNSUP, "edge_att_weights_backward: layers 1..4, edge_dim 1..8, stride >= edge_dim");
    for (int l = 0; l < a->num_layers; ++l)
        if (a->heads[l] < 1 || a->channels[l] < 1 || !a->lin_edge_w[l] || !a->att_edge[l])
            return fail(TRX_EINVAL, "edge_att_weights_backward: layer %d", l);
    hipError_t e = trx::launch_edge_att_weights_bwd(*a, g_m, g_m_stride, out, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "edge_att_weights_backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

// networks of one *_multi launch: same sizes, shapes and mode (their buffers differ)
static bool same_shape(const trx_gat_prologue_bwd_args& x, const trx_gat_prologue_bwd_args& y) {
    return x.num_graphs == y.num_graphs &&
           x.nodes_per_graph == y.nodes_per_graph &&
           x.edges_per_graph == y.edges_per_graph &&
           x.node_dim == y.node_dim &&
           x.edge_dim == y.edge_dim &&
           x.A == y.A &&
           x.exact == y.exact;
}

static int check_gat_prologue_backward(const trx_gat_prologue_bwd_args* a) {
    if (!a) return fail(TRX_EINVAL, "gat_prologue_backward: NULL args");
    if (a->num_graphs < 0 || a->nodes_per_graph < 1 || a->nodes_per_graph > 64 || a->edges_per_graph < 0 ||
        a->edges_per_graph > 1024 || a->node_dim < 1 || a->node_dim > 8 || a->edge_dim < 1 || a->edge_dim > 8 ||
        a->A < 1 || a->A > 32)
        return fail(TRX_EUNSUP, "gat_prologue_backward: sizes (nodes <= 64, links <= 1024, dims <= 8, heads <= 32)");
    if (!a->node_x || !a->edge_x || !a->node_ln_w || !a->node_ln_b || !a->edge_ln_w || !a->edge_ln_b || !a->src ||
        !a->dst || !a->rowptr || !a->pos_src || !a->m_work || !a->g_a_edge || !a->g_x0 || !a->part)
        return fail(TRX_EINVAL, "gat_prologue_backward: NULL buffer");
    return TRX_OK;
}

int trx_gat_prologue_backward_multi(const trx_gat_prologue_bwd_args* a, int32_t count, void* stream) {
    if (!a || count < 1 || count > TRX_MAX_NETS)
        return fail(TRX_EINVAL, "gat_prologue_backward_multi: 1..%d networks", TRX_MAX_NETS);
    for (int k = 0; k < count; ++k) {
        const int rc = check_gat_prologue_backward(a + k);
        if (rc != TRX_OK) return rc;
        const trx_gat_prologue_bwd_args& b = a[k];
        if (!same_shape(b, *a))
            return fail(TRX_EINVAL, "gat_prologue_backward_multi: network %d differs from network 0 in shape or mode", k);
    }
    if (a->num_graphs == 0) return TRX_OK;
    hipError_t e = trx::launch_gat_prologue_bwd(a, count, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "gat_prologue_backward launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_gat_prologue_backward(const trx_gat_prologue_bwd_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "gat_prologue_backward: NULL args");
    return trx_gat_prologue_backward_multi(a, 1, stream);
}

int trx_sac_loss(const trx_sac_loss_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "sac_loss: NULL args");
    if (a->num_graphs < 1 || a->edges_per_graph < 1 || a->edges_per_graph > 256)
        return fail(TRX_EUNSUP, "sac_loss: need >= 1 graph and 1..256 links per graph");
    if (!a->next_probs || !a->qt1 || !a->qt2 || !a->reward || !a->done || !a->q1 || !a->q2 || !a->logits ||
        !a->mask || !a->action || !a->weights || !a->log_alpha || !a->g_q1 || !a->g_q2 || !a->g_logits ||
        !a->td_error || !a->part || !a->out || !a->g_log_alpha)
        return fail(TRX_EINVAL, "sac_loss: NULL buffer");
    hipError_t e = trx::launch_sac_loss(*a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "sac_loss launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_sac_adam(const trx_adam_args* a, void* stream) {
    if (!a) return fail(TRX_EINVAL, "sac_adam: NULL args");
    if (a->nseg < 1 || a->nblocks < 1) return fail(TRX_EINVAL, "sac_adam: empty segment / block table");
    if (!a->segs || !a->blocks || !a->g_base || !a->m || !a->v || !a->partial || !a->step || !a->scal)
        return fail(TRX_EINVAL, "sac_adam: NULL buffer");
    hipError_t e = trx::launch_sac_adam(*a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(TRX_EHIP, "sac_adam launch: %s", hipGetErrorString(e));
    return TRX_OK;
}

int trx_graph_patch_memsets(void* hip_graph, int32_t* n_patched) {
    if (!hip_graph) return fail(TRX_EINVAL, "graph_patch_memsets: NULL graph");
    int n = 0;
    hipError_t e = trx::patch_graph_memsets(static_cast<hipGraph_t>(hip_graph), &n);
    if (n_patched) *n_patched = n;
    if (e != hipSuccess) return fail(TRX_EHIP, "graph_patch_memsets: %s", hipGetErrorString(e));
    return TRX_OK;
}

}  // extern "C"

/*
 * trx_oracle.c -- CPU restatement of the reference's static traffic assignment.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker (and the timed
 * "port" CPU baseline in bench.py).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product path (libtrafficrl.so)
 * never links or calls it.
 *
 * Restates, statement by statement, /root/reference/src/env/repair_env.py:
 *   compute_travel_time (BPR)         667-677
 *   _all_or_nothing, scipy branch     481-503  + _path_edges_from_predecessors 707-722
 *   compute_flow_assignment (MSA/FW/CFW) 299-345
 *   compute_tstt                      724-735
 *   compute_reward_with_goal          244-291, is_goal_complete 293-294
 *   _all_or_nothing_torch (sp_backend="torch": float32 Floyd-Warshall, strict <,
 *     k ascending, next_hop walk)     520-573
 *   get_state (betweenness + features) 751-819, networkx 3.4 Brandes order
 * and scipy 1.15.3 scipy.sparse.csgraph.dijkstra (Fibonacci heap, float64
 * labels, strict-improvement predecessors, CSR rows sorted by column as
 * csr_matrix((w,(row,col))) produces them).  The heap is restated from
 * scipy/sparse/csgraph/_shortest_path.pyx (FibonacciHeap: insert_node,
 * decrease_val, link, remove_min); tools/gen_golden.py + tests pin it against
 * scipy's own predecessor matrices, ties included.
 *
 * Numerics pinned to the reference's numpy semantics:
 *   - every float32 op rounds to float32 (compile with -ffp-contract=off);
 *   - Python-float scalars (step, 1-step, alpha) are rounded to float32 before
 *     the array op (NumPy 2 weak-scalar rule, NEP 50);
 *   - vc**4 is float32(((double)vc^2)^2): the host-independent power
 *     (numpy's own float32 power is SVML on AVX-512 hosts, not correctly
 *     rounded; see tools/gen_golden.py "native" vs "crpow");
 *   - np.sum(float32) is numpy's pairwise_sum (8 accumulators, block 128);
 *   - shortest-path labels are float64 sums of float32 costs.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_NONE (-9999)

typedef struct {
    int N, E, P;
    const int32_t *src, *dst;     /* [E] 0-based, file order */
    const float *t0, *cap0;       /* [E] */
    const int32_t *od_o, *od_d;   /* [P] OD dict order (0-based) */
    const double *od_v;           /* [P] */
    /* derived (built by orc_graph_build) */
    int32_t *indptr, *indices, *csr_eid;  /* CSR sorted by (src, dst) */
    int32_t *eid_of;              /* [N*N] (u,v) -> edge id (last wins, like edge_id_map) */
    int32_t *org_ptr, *org_idx;   /* OD entries grouped by origin, dict order kept */
    double total_demand;
} orc_graph;

/* ---------------------------------------------------------------- graph */
int orc_graph_build(orc_graph* g) {
    int N = g->N, E = g->E, P = g->P;
    g->indptr = (int32_t*)calloc(N + 1, sizeof(int32_t));
    g->indices = (int32_t*)malloc(sizeof(int32_t) * (E > 0 ? E : 1));
    g->csr_eid = (int32_t*)malloc(sizeof(int32_t) * (E > 0 ? E : 1));
    g->eid_of = (int32_t*)malloc(sizeof(int32_t) * N * N);
    g->org_ptr = (int32_t*)calloc(N + 1, sizeof(int32_t));
    g->org_idx = (int32_t*)malloc(sizeof(int32_t) * (P > 0 ? P : 1));
    if (!g->indptr || !g->indices || !g->csr_eid || !g->eid_of || !g->org_ptr || !g->org_idx) return -1;
    for (int i = 0; i < N * N; i++) g->eid_of[i] = -1;
    for (int e = 0; e < E; e++) {
        if (g->src[e] < 0 || g->src[e] >= N || g->dst[e] < 0 || g->dst[e] >= N) return -2;
        if (g->eid_of[g->src[e] * N + g->dst[e]] >= 0) return -3; /* parallel links: csr would sum them */
        g->eid_of[g->src[e] * N + g->dst[e]] = e;
        g->indptr[g->src[e] + 1]++;
    }
    for (int u = 0; u < N; u++) g->indptr[u + 1] += g->indptr[u];
    /* rows sorted by column index (csr canonical format) */
    int pos = 0;
    for (int u = 0; u < N; u++)
        for (int v = 0; v < N; v++) {
            int e = g->eid_of[u * N + v];
            if (e >= 0) { g->indices[pos] = v; g->csr_eid[pos] = e; pos++; }
        }
    double tot = 0.0;
    for (int k = 0; k < P; k++) {
        g->org_ptr[g->od_o[k] + 1]++;
        tot += g->od_v[k];
    }
    for (int u = 0; u < N; u++) g->org_ptr[u + 1] += g->org_ptr[u];
    int* fill = (int*)calloc(N, sizeof(int));
    for (int k = 0; k < P; k++) {
        int o = g->od_o[k];
        g->org_idx[g->org_ptr[o] + fill[o]++] = k;
    }
    free(fill);
    g->total_demand = tot; /* float(np.sum(list(values))) -- integer demands: exact */
    return 0;
}

void orc_graph_free(orc_graph* g) {
    free(g->indptr); free(g->indices); free(g->csr_eid); free(g->eid_of);
    free(g->org_ptr); free(g->org_idx);
}

/* ------------------------------------------------------------------ BPR */
/* repair_env.py:667-677 */
void orc_bpr(int E, const float* flow, const float* cap, const float* t0, const float* damaged,
             float alpha, float beta, float* t) {
    const float cap_floor = (float)1e-6;
    for (int e = 0; e < E; e++) {
        float c = cap[e] > cap_floor ? cap[e] : cap_floor;       /* np.maximum(cap, 1e-6) */
        float vc = flow[e] / c;
        vc = vc < 0.0f ? 0.0f : (vc > 10.0f ? 10.0f : vc);      /* np.clip(., 0, 10) */
        float p;
        if (beta == 4.0f) {
            double v = (double)vc, v2 = v * v;
            p = (float)(v2 * v2);
        } else {  /* integer beta: left-to-right float64 product (same as the HIP kernel) */
            double v = (double)vc, acc = 1.0;
            for (int i = 0; i < (int)beta; i++) acc = acc * v;
            p = (float)acc;
        }
        float a = alpha * p;
        float s = 1.0f + a;
        float te = t0[e] * s;
        if (damaged[e] > 0.5f) te = 1e6f;
        t[e] = te;
    }
}

/* numpy pairwise_sum for float32 (numpy/_core/src/umath/loops_utils.h.src) */
static float pairwise_f32(const float* a, long n) {
    if (n < 8) {
        float r = 0.0f;
        for (long i = 0; i < n; i++) r += a[i];
        return r;
    } else if (n <= 128) {
        float r[8];
        long i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_f32(a, n2) + pairwise_f32(a + n2, n - n2);
    }
}

float orc_pairwise_sum_f32(const float* a, long n) { return pairwise_f32(a, n); }

/* repair_env.py:724-735 */
double orc_tstt(int E, const float* flow, const float* t, double unassigned, double total_demand,
                double penalty_coef, float* scratch) {
    for (int e = 0; e < E; e++) scratch[e] = flow[e] * t[e];
    double base = (double)pairwise_f32(scratch, E);
    double td = total_demand > 1.0 ? total_demand : 1.0;
    double att = base / td;
    double pen = 0.0;
    if (unassigned > 0) pen = penalty_coef * (unassigned / td);
    return att + pen;
}

/* ------------------------------------------------- scipy Fibonacci heap */
enum { NOT_IN_HEAP = 0, IN_HEAP = 1, SCANNED = 2 };
typedef struct fnode {
    int index, rank, state;
    double val;
    struct fnode *parent, *left, *right, *children;
} fnode;
typedef struct {
    fnode* min;
    fnode* roots[100];
} fheap;

static void fh_add_sibling(fnode* node, fnode* ns) {
    if (node->right) node->right->left = ns;
    ns->right = node->right;
    ns->left = node;
    node->right = ns;
    ns->parent = node->parent;
    if (ns->parent) ns->parent->rank += 1;
}
static void fh_add_child(fnode* node, fnode* c) {
    c->parent = node;
    if (node->children) {
        fh_add_sibling(node->children, c);
    } else {
        node->children = c;
        c->right = NULL;
        c->left = NULL;
        node->rank = 1;
    }
}
static void fh_remove(fnode* node) {
    if (node->parent) {
        node->parent->rank -= 1;
        if (node->parent->children == node) node->parent->children = node->right;
    }
    if (node->left) node->left->right = node->right;
    if (node->right) node->right->left = node->left;
    node->left = node->right = node->parent = NULL;
}
static void fh_insert(fheap* h, fnode* node) {
    if (h->min) {
        if (node->val < h->min->val) {
            node->left = NULL;
            node->right = h->min;
            h->min->left = node;
            h->min = node;
        } else {
            fh_add_sibling(h->min, node);
        }
    } else {
        h->min = node;
    }
}
static void fh_decrease(fheap* h, fnode* node, double nv) {
    node->val = nv;
    if (node->parent && node->parent->val >= nv) {
        fh_remove(node);
        fh_insert(h, node);
    } else if (h->min->val > node->val) {
        fh_remove(node);
        node->right = h->min;
        h->min->left = node;
        h->min = node;
    }
}
static void fh_link(fheap* h, fnode* node) {
    for (;;) {
        if (h->roots[node->rank] == NULL) {
            h->roots[node->rank] = node;
            return;
        }
        fnode* ln = h->roots[node->rank];
        h->roots[node->rank] = NULL;
        if (node->val < ln->val || node == h->min) {
            fh_remove(ln);
            fh_add_child(node, ln);
        } else {
            fh_remove(node);
            fh_add_child(ln, node);
            node = ln;
        }
    }
}
static fnode* fh_remove_min(fheap* h) {
    fnode* temp = h->min->children;
    while (temp) {
        fnode* tr = temp->right;
        fh_remove(temp);
        fh_add_sibling(h->min, temp);
        temp = tr;
    }
    fnode* out = h->min;
    temp = h->min->right;
    fh_remove(h->min);
    h->min = temp;
    if (!temp) return out;
    for (int i = 0; i < 100; i++) h->roots[i] = NULL;
    while (temp) {
        if (temp->val < h->min->val) h->min = temp;
        fnode* tr = temp->right;
        fh_link(h, temp);
        temp = tr;
    }
    temp = h->min;
    while (temp->left) temp = temp->left;
    if (h->min != temp) {
        fh_remove(h->min);
        h->min->right = temp;
        temp->left = h->min;
    }
    return out;
}

/* Single-source scipy dijkstra.  w_csr[k] = float64 cost of CSR slot k.
 * pred[v] = tail node or ORC_NONE; dist[v] = +inf if unreachable.
 * order (optional) receives the scan order, returns number scanned. */
int orc_sssp_scipy(const orc_graph* g, const double* w_csr, int source, double* dist, int32_t* pred,
                   int32_t* order, fnode* nodes) {
    int N = g->N, nscan = 0;
    for (int k = 0; k < N; k++) {
        nodes[k].index = k; nodes[k].rank = 0; nodes[k].state = NOT_IN_HEAP; nodes[k].val = 0.0;
        nodes[k].parent = nodes[k].left = nodes[k].right = nodes[k].children = NULL;
        dist[k] = INFINITY;
        pred[k] = ORC_NONE;
    }
    fheap h;
    h.min = NULL;
    dist[source] = 0.0;
    fh_insert(&h, &nodes[source]);
    while (h.min) {
        fnode* v = fh_remove_min(&h);
        v->state = SCANNED;
        if (order) order[nscan] = v->index;
        nscan++;
        for (int j = g->indptr[v->index]; j < g->indptr[v->index + 1]; j++) {
            int jc = g->indices[j];
            fnode* cur = &nodes[jc];
            if (cur->state != SCANNED) {
                double nv = v->val + w_csr[j];
                if (cur->state == NOT_IN_HEAP) {
                    cur->state = IN_HEAP;
                    cur->val = nv;
                    fh_insert(&h, cur);
                    pred[jc] = v->index;
                } else if (cur->val > nv) {
                    fh_decrease(&h, cur, nv);
                    pred[jc] = v->index;
                }
            }
        }
        dist[v->index] = v->val;
    }
    return nscan;
}

/* all-pairs scipy dijkstra for a weight vector t (edge order) */
void orc_all_pairs(const orc_graph* g, const float* t, double* dist_NN, int32_t* pred_NN) {
    int N = g->N, E = g->E;
    double* w = (double*)malloc(sizeof(double) * (E > 0 ? E : 1));
    fnode* nodes = (fnode*)malloc(sizeof(fnode) * N);
    for (int k = 0; k < E; k++) w[k] = (double)t[g->csr_eid[k]];
    for (int s = 0; s < N; s++) orc_sssp_scipy(g, w, s, dist_NN + (long)s * N, pred_NN + (long)s * N, NULL, nodes);
    free(w); free(nodes);
}

/* ------------------------------------------------------- all-or-nothing */
typedef struct {
    double* w;       /* [E] csr-ordered costs */
    double* dist;    /* [N] */
    int32_t* pred;   /* [N] */
    int32_t* path;   /* [N] */
    fnode* nodes;    /* [N] */
    float* d_fw;     /* [E] */
    float* d_prev;   /* [E] */
    float* dir;      /* [E] */
    float* aux;      /* [E] */
    float* t;        /* [E] */
    float* scratch;  /* [E] */
    float* fw_dist;  /* [N*N] torch-backend Floyd-Warshall */
    int32_t* fw_nh;  /* [N*N] */
    int sp;          /* ORC_SP_* */
} orc_ws;

static int ws_alloc(orc_ws* ws, int N, int E) {
    int EE = E > 0 ? E : 1;
    ws->w = (double*)malloc(sizeof(double) * EE);
    ws->dist = (double*)malloc(sizeof(double) * N);
    ws->pred = (int32_t*)malloc(sizeof(int32_t) * N);
    ws->path = (int32_t*)malloc(sizeof(int32_t) * (N + 1));
    ws->nodes = (fnode*)malloc(sizeof(fnode) * N);
    ws->d_fw = (float*)malloc(sizeof(float) * EE);
    ws->d_prev = (float*)malloc(sizeof(float) * EE);
    ws->dir = (float*)malloc(sizeof(float) * EE);
    ws->aux = (float*)malloc(sizeof(float) * EE);
    ws->t = (float*)malloc(sizeof(float) * EE);
    ws->scratch = (float*)malloc(sizeof(float) * EE);
    ws->fw_dist = (float*)malloc(sizeof(float) * N * N);
    ws->fw_nh = (int32_t*)malloc(sizeof(int32_t) * N * N);
    ws->sp = 0;
    return (ws->w && ws->dist && ws->pred && ws->path && ws->nodes && ws->d_fw && ws->d_prev && ws->dir &&
            ws->aux && ws->t && ws->scratch && ws->fw_dist && ws->fw_nh) ? 0 : -1;
}
static void ws_free(orc_ws* ws) {
    free(ws->w); free(ws->dist); free(ws->pred); free(ws->path); free(ws->nodes);
    free(ws->d_fw); free(ws->d_prev); free(ws->dir); free(ws->aux); free(ws->t); free(ws->scratch);
    free(ws->fw_dist); free(ws->fw_nh);
}

/* repair_env.py:481-503 (+ 707-722): returns unassigned demand */
static double aon(const orc_graph* g, const float* t, float* aux, orc_ws* ws) {
    int N = g->N, E = g->E;
    double unassigned = 0.0;
    for (int e = 0; e < E; e++) aux[e] = 0.0f;
    for (int k = 0; k < E; k++) ws->w[k] = (double)t[g->csr_eid[k]];
    for (int origin = 0; origin < N; origin++) {
        if (g->org_ptr[origin] == g->org_ptr[origin + 1]) continue;
        orc_sssp_scipy(g, ws->w, origin, ws->dist, ws->pred, NULL, ws->nodes);
        for (int q = g->org_ptr[origin]; q < g->org_ptr[origin + 1]; q++) {
            int k = g->org_idx[q];
            int dest = g->od_d[k];
            double demand = g->od_v[k];
            /* _path_edges_from_predecessors */
            if (dest == origin || ws->pred[dest] < 0) { unassigned += demand; continue; }
            int n = 0, cur = dest;
            while (cur != origin && cur != ORC_NONE) { ws->path[n++] = cur; cur = ws->pred[cur]; }
            if (cur != origin) { unassigned += demand; continue; }
            ws->path[n++] = origin;
            float dem32 = (float)demand;
            for (int i = n - 1; i > 0; i--) {
                int e = g->eid_of[ws->path[i] * N + ws->path[i - 1]];
                aux[e] = aux[e] + dem32;
            }
        }
    }
    return unassigned;
}

double orc_aon(const orc_graph* g, const float* t, float* aux) {
    orc_ws ws;
    if (ws_alloc(&ws, g->N, g->E)) return NAN;
    double u = aon(g, t, aux, &ws);
    ws_free(&ws);
    return u;
}

/* repair_env.py:520-573 (_all_or_nothing_torch): float32 all-pairs
 * Floyd-Warshall, dist init 1e12 with a zero diagonal, then dist[u][v] =
 * t[e] and next_hop[u][v] = v per link in file order; for k ascending
 * alt = dist[i][k] + dist[k][j] (float32), strict `alt < dist` takes alt and
 * next_hop[i][k].  Each OD pair (dict order, origin != dest) walks next_hop
 * from the origin for at most N hops; a pair that does not reach its
 * destination is unassigned (its partial path is dropped).  Returns
 * unassigned demand.  dist/nh: [N*N] scratch. */
static double aon_fw(const orc_graph* g, const float* t, float* aux, float* dist, int32_t* nh, int32_t* path) {
    int N = g->N, E = g->E;
    double unassigned = 0.0;
    for (int e = 0; e < E; e++) aux[e] = 0.0f;
    for (int i = 0; i < N * N; i++) { dist[i] = 1e12f; nh[i] = -1; }
    for (int i = 0; i < N; i++) dist[i * N + i] = 0.0f;
    for (int e = 0; e < E; e++) {
        dist[g->src[e] * N + g->dst[e]] = t[e];
        nh[g->src[e] * N + g->dst[e]] = g->dst[e];
    }
    for (int k = 0; k < N; k++) {
        const float* rowk = dist + (long)k * N;
        for (int i = 0; i < N; i++) {
            if (i == k) continue;  /* alt[k][j] = 0 + d[k][j] and alt[i][k] = d[i][k] + 0 never improve */
            const float dik = dist[(long)i * N + k];
            const int32_t nik = nh[(long)i * N + k];
            float* rowi = dist + (long)i * N;
            int32_t* nhi = nh + (long)i * N;
            for (int j = 0; j < N; j++) {
                float alt = dik + rowk[j];
                if (alt < rowi[j]) { rowi[j] = alt; nhi[j] = nik; }
            }
        }
    }
    for (int q = 0; q < g->P; q++) {
        int o = g->od_o[q], d = g->od_d[q];
        double demand = g->od_v[q];
        if (o == d) continue;
        int n = 0, cur = o, hops = 0, ok = 1;
        while (cur != d && cur != -1 && hops < N) {
            int nxt = nh[(long)cur * N + d];
            if (nxt < 0) { ok = 0; break; }
            path[n++] = g->eid_of[cur * N + nxt];
            cur = nxt;
            hops++;
        }
        if (!ok || cur != d) { unassigned += demand; continue; }
        float dem32 = (float)demand;
        for (int i = 0; i < n; i++) aux[path[i]] = aux[path[i]] + dem32;
    }
    return unassigned;
}

double orc_aon_fw(const orc_graph* g, const float* t, float* aux, int32_t* nh_out) {
    int N = g->N;
    float* dist = (float*)malloc(sizeof(float) * N * N);
    int32_t* nh = nh_out ? nh_out : (int32_t*)malloc(sizeof(int32_t) * N * N);
    int32_t* path = (int32_t*)malloc(sizeof(int32_t) * (N + 1));
    double u = aon_fw(g, t, aux, dist, nh, path);
    free(dist); free(path);
    if (!nh_out) free(nh);
    return u;
}

enum { ORC_MSA = 0, ORC_FW = 1, ORC_CFW = 2 };
enum { ORC_SP_SCIPY = 0, ORC_SP_TORCH = 1 };

/* repair_env.py:299-345.  flow: in = warm start, out = final flow.
 * t_out (optional) = BPR(final flow).  Returns tstt. */
static double assign_one(const orc_graph* g, int method, int iters, float alpha, float beta,
                         double penalty_coef, const float* cap, const float* damaged, float* flow,
                         float* t_out, double* unassigned_out, orc_ws* ws) {
    int E = g->E;
    float* t = ws->t;
    double unassigned = 0.0;
    int have_prev = 0;
    orc_bpr(E, flow, cap, g->t0, damaged, alpha, beta, t);
    for (int it = 0; it < iters; it++) {
        double un = ws->sp == ORC_SP_TORCH ? aon_fw(g, t, ws->aux, ws->fw_dist, ws->fw_nh, ws->path)
                                           : aon(g, t, ws->aux, ws);
        for (int e = 0; e < E; e++) ws->d_fw[e] = ws->aux[e] - flow[e];
        if (method == ORC_CFW) {
            float* dir = ws->dir;
            if (!have_prev) {
                for (int e = 0; e < E; e++) dir[e] = ws->d_fw[e];
            } else {
                /* np.dot(float32) is BLAS sdot in the reference (order is
                 * library-defined); accumulated in float64 here. */
                double num = 0.0, den = 0.0;
                for (int e = 0; e < E; e++) {
                    float df = ws->d_fw[e] - ws->d_prev[e];
                    num += (double)(ws->d_fw[e] * df);
                    den += (double)(ws->d_prev[e] * ws->d_prev[e]);
                }
                num = (double)(float)num;
                den = (double)(float)den + 1e-12;
                double b = num / den;
                if (b < 0.0) b = 0.0;
                float b32 = (float)b;
                for (int e = 0; e < E; e++) dir[e] = ws->d_fw[e] + b32 * ws->d_prev[e];
            }
            float step = (float)(2.0 / (it + 2.0));
            for (int e = 0; e < E; e++) {
                float f = flow[e] + step * dir[e];
                flow[e] = f > 0.0f ? f : 0.0f;
            }
            memcpy(ws->d_prev, dir, sizeof(float) * E);
            have_prev = 1;
        } else {
            double stepd = method == ORC_FW ? 2.0 / (it + 2.0) : 1.0 / (it + 1.0);
            float om = (float)(1 - stepd), s = (float)stepd;
            for (int e = 0; e < E; e++) {
                float a = om * flow[e];
                float b = s * ws->aux[e];
                flow[e] = a + b;
            }
        }
        for (int e = 0; e < E; e++)
            if (isnan(flow[e])) flow[e] = 0.0f; /* nan_to_num guard (338-340) */
        orc_bpr(E, flow, cap, g->t0, damaged, alpha, beta, t);
        unassigned = un;
    }
    if (t_out) memcpy(t_out, t, sizeof(float) * E);
    if (unassigned_out) *unassigned_out = unassigned;
    return orc_tstt(E, flow, t, unassigned, g->total_demand, penalty_coef, ws->scratch);
}

/* Batched assignment over B envs (row-major [B,E] arrays).  env_mask may be
 * NULL.  OpenMP over envs when nthreads > 1 (CPU baseline).  Returns 0. */
int orc_assign_batch(const orc_graph* g, int B, int method, int iters, float alpha, float beta,
                     double penalty_coef, const float* cap, const float* damaged, float* flow, float* t_out,
                     double* tstt, double* unassigned, const uint8_t* env_mask, int nthreads, int sp) {
    int E = g->E;
    int err = 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads) reduction(| : err)
#endif
    {
        orc_ws ws;
        if (ws_alloc(&ws, g->N, E)) {
            err = 1;
        } else {
            ws.sp = sp;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
            for (int b = 0; b < B; b++) {
                if (env_mask && !env_mask[b]) continue;
                double un = 0.0;
                double ts = assign_one(g, method, iters, alpha, beta, penalty_coef, cap + (long)b * E,
                                       damaged + (long)b * E, flow + (long)b * E,
                                       t_out ? t_out + (long)b * E : NULL, &un, &ws);
                if (tstt) tstt[b] = ts;
                if (unassigned) unassigned[b] = un;
            }
            ws_free(&ws);
        }
    }
    return err ? -1 : 0;
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---------------------------------------------------------------- reward */
/* repair_env.py:244-294.  mode: 0 delta, 1 log_delta, 2 neg_tstt,
 * 3 minimize_tstt, 4 rel_improve.  initial_tstt < 0 means None. */
double orc_reward(int mode, double prev, double curr, double initial_tstt, int complete, double alpha,
                  double beta, double gamma, double clip) {
    double delta, reward;
    double bonus = complete ? beta : 0.0;
    if (mode == 2) {
        delta = -curr;
    } else if (mode == 1) {
        double a = prev > 1.0 ? prev : 1.0, b = curr > 1.0 ? curr : 1.0;
        delta = log10(a) - log10(b);
    } else if (mode == 3 || mode == 4) {
        double base = initial_tstt >= 0 ? initial_tstt : prev;
        double bb = base > 1.0 ? base : 1.0;
        if (mode == 3) {
            reward = -alpha * (curr / bb);
        } else {
            double delta_pct = ((prev - curr) / bb) * 100.0;
            double ratio = curr / bb;
            reward = alpha * delta_pct - 1.0 * ratio;
        }
        reward = reward + bonus;
        if (clip > 0) reward = reward < -clip ? -clip : (reward > clip ? clip : reward);
        return reward;
    } else {
        delta = prev - curr;
    }
    reward = alpha * delta + bonus - gamma;
    if (clip > 0) reward = reward < -clip ? -clip : (reward > clip ? clip : reward);
    return reward;
}

/* ------------------------------------------------------------ get_state */
/* repair_env.py:751-819 for B envs (the timed CPU baseline's observation
 * leg; oracle.py's observation() is the pure-Python restatement it is
 * checked against).  Betweenness: networkx 3.4 betweenness_centrality on
 * G.edge_subgraph(active links), normalized, directed -- Brandes BFS
 * (_single_source_shortest_path_basic) and accumulation (_accumulate_basic)
 * with networkx's node order (first appearance in the link list) and
 * adjacency order (link insertion order), float64.  node_x [B,N,4],
 * edge_x [B,E,6], mask [B,E] (may be NULL). */
typedef struct {
    int32_t *order, *adj_ptr, *adj, *adj_e, *nodes, *D, *Q, *S, *P_ptr, *P_cnt, *P;
    double *sigma, *delta, *bc;
    uint8_t* on;
    float *tmp, *bw;
} orc_obs_ws;

static int obs_ws_alloc(orc_obs_ws* w, int N, int E) {
    int EE = E > 0 ? E : 1;
    w->order = (int32_t*)malloc(sizeof(int32_t) * N);
    w->adj_ptr = (int32_t*)calloc(N + 1, sizeof(int32_t));
    w->adj = (int32_t*)malloc(sizeof(int32_t) * EE);
    w->adj_e = (int32_t*)malloc(sizeof(int32_t) * EE);
    w->nodes = (int32_t*)malloc(sizeof(int32_t) * N);
    w->D = (int32_t*)malloc(sizeof(int32_t) * N);
    w->Q = (int32_t*)malloc(sizeof(int32_t) * N);
    w->S = (int32_t*)malloc(sizeof(int32_t) * N);
    w->P_ptr = (int32_t*)malloc(sizeof(int32_t) * (N + 1));
    w->P_cnt = (int32_t*)malloc(sizeof(int32_t) * N);
    w->P = (int32_t*)malloc(sizeof(int32_t) * EE);
    w->sigma = (double*)malloc(sizeof(double) * N);
    w->delta = (double*)malloc(sizeof(double) * N);
    w->bc = (double*)malloc(sizeof(double) * N);
    w->on = (uint8_t*)malloc(N);
    w->tmp = (float*)malloc(sizeof(float) * EE);
    w->bw = (float*)malloc(sizeof(float) * N);
    return (w->bw && w->order && w->adj_ptr && w->adj && w->adj_e && w->nodes && w->D && w->Q && w->S && w->P_ptr &&
            w->P_cnt && w->P && w->sigma && w->delta && w->bc && w->on && w->tmp) ? 0 : -1;
}
static void obs_ws_free(orc_obs_ws* w) {
    free(w->order); free(w->adj_ptr); free(w->adj); free(w->adj_e); free(w->nodes); free(w->D); free(w->Q);
    free(w->S); free(w->P_ptr); free(w->P_cnt); free(w->P); free(w->sigma); free(w->delta); free(w->bc);
    free(w->on); free(w->tmp); free(w->bw);
}

/* node order and adjacency of the reference's nx.DiGraph (repair_env.py:106-109) */
static void obs_topology(const orc_graph* g, orc_obs_ws* w) {
    int N = g->N, E = g->E, cnt = 0;
    memset(w->on, 0, N);
    for (int e = 0; e < E; e++) {
        int uv[2] = {g->src[e], g->dst[e]};
        for (int k = 0; k < 2; k++)
            if (!w->on[uv[k]]) { w->on[uv[k]] = 1; w->order[cnt++] = uv[k]; }
    }
    for (int i = cnt; i < N; i++) w->order[i] = -1;  /* isolated nodes are not in the nx graph */
    memset(w->adj_ptr, 0, sizeof(int32_t) * (N + 1));
    for (int e = 0; e < E; e++) w->adj_ptr[g->src[e] + 1]++;
    for (int u = 0; u < N; u++) w->adj_ptr[u + 1] += w->adj_ptr[u];
    int* fill = (int*)calloc(N, sizeof(int));
    for (int e = 0; e < E; e++) {
        int u = g->src[e], k = w->adj_ptr[u] + fill[u]++;
        w->adj[k] = g->dst[e];
        w->adj_e[k] = e;
    }
    free(fill);
    /* predecessor slots: at most the in-degree of each node */
    memset(w->P_ptr, 0, sizeof(int32_t) * (N + 1));
    for (int e = 0; e < E; e++) w->P_ptr[g->dst[e] + 1]++;
    for (int u = 0; u < N; u++) w->P_ptr[u + 1] += w->P_ptr[u];
}

static void obs_betweenness(const orc_graph* g, orc_obs_ws* w, const float* damaged, float* bw_out) {
    int N = g->N, n = 0;
    /* edge_subgraph nodes: graph order, incident to an active link */
    memset(w->on, 0, N);
    for (int e = 0; e < g->E; e++)
        if (damaged[e] == 0.0f) { w->on[g->src[e]] = 1; w->on[g->dst[e]] = 1; }
    for (int i = 0; i < N && w->order[i] >= 0; i++)
        if (w->on[w->order[i]]) w->nodes[n++] = w->order[i];
    for (int v = 0; v < N; v++) w->bc[v] = 0.0;
    for (int si = 0; si < n; si++) {
        int s = w->nodes[si];
        for (int v = 0; v < N; v++) { w->sigma[v] = 0.0; w->D[v] = -1; w->P_cnt[v] = 0; w->delta[v] = 0.0; }
        w->sigma[s] = 1.0;
        w->D[s] = 0;
        int qh = 0, qt = 0, ns = 0;
        w->Q[qt++] = s;
        while (qh < qt) {
            int v = w->Q[qh++];
            w->S[ns++] = v;
            int Dv = w->D[v];
            double sv = w->sigma[v];
            for (int k = w->adj_ptr[v]; k < w->adj_ptr[v + 1]; k++) {
                if (damaged[w->adj_e[k]] != 0.0f) continue;
                int x = w->adj[k];
                if (w->D[x] < 0) { w->Q[qt++] = x; w->D[x] = Dv + 1; }
                if (w->D[x] == Dv + 1) { w->sigma[x] += sv; w->P[w->P_ptr[x] + w->P_cnt[x]++] = v; }
            }
        }
        while (ns > 0) {
            int x = w->S[--ns];
            double coeff = (1.0 + w->delta[x]) / w->sigma[x];
            for (int k = 0; k < w->P_cnt[x]; k++) {
                int v = w->P[w->P_ptr[x] + k];
                w->delta[v] += w->sigma[v] * coeff;
            }
            if (x != s) w->bc[x] += w->delta[x];
        }
    }
    if (n > 2) {
        double scale = 1.0 / ((double)(n - 1) * (double)(n - 2));
        for (int i = 0; i < n; i++) w->bc[w->nodes[i]] *= scale;
    }
    for (int v = 0; v < N; v++) bw_out[v] = w->on[v] ? (float)w->bc[v] : 0.0f;
}

static void obs_one(const orc_graph* g, orc_obs_ws* w, const float* cap, const float* damaged, const float* goal,
                    const float* flow, double tstt, float* node_x, float* edge_x, float* mask) {
    int N = g->N, E = g->E;
    float* b = w->bw;
    obs_betweenness(g, w, damaged, b);
    float bmax = 0.0f;
    for (int v = 0; v < N; v++) bmax = b[v] > bmax ? b[v] : bmax;
    if (bmax > 0.0f)
        for (int v = 0; v < N; v++) b[v] = b[v] / bmax;
    /* goal_total / remaining: float(np.sum(float32)) -- integer-valued, exact */
    double goal_total = 0.0, remaining = 0.0;
    int n_und = 0;
    for (int e = 0; e < E; e++) {
        goal_total += goal[e];
        remaining += (double)(goal[e] * damaged[e]);
        if (damaged[e] == 0.0f) w->tmp[n_und++] = flow[e];
    }
    double rr = remaining / (goal_total > 1.0 ? goal_total : 1.0);
    double avg = n_und > 0 ? (double)(pairwise_f32(w->tmp, n_und) / (float)n_und) : 0.0;
    double dn = g->total_demand / (double)(E > 1 ? E : 1);
    double afn = avg / (dn > 1.0 ? dn : 1.0);
    double lt = log10(tstt > 1.0 ? tstt : 1.0);
    for (int v = 0; v < N; v++) {
        node_x[v * 4 + 0] = b[v];
        node_x[v * 4 + 1] = (float)rr;
        node_x[v * 4 + 2] = (float)afn;
        node_x[v * 4 + 3] = (float)lt;
    }
    float max_t0 = 0.0f, max_cap = 0.0f;
    for (int e = 0; e < E; e++) {
        max_t0 = g->t0[e] > max_t0 ? g->t0[e] : max_t0;
        max_cap = g->cap0[e] > max_cap ? g->cap0[e] : max_cap;
    }
    double lt0 = log10((double)max_t0 + 1.0), lcap = log10((double)max_cap + 1.0);
    for (int e = 0; e < E; e++) {
        float c = cap[e] > 1e-6f ? cap[e] : 1e-6f;
        float raw = flow[e] / c;
        float vc = damaged[e] > 0.0f ? 0.0f : raw;
        vc = log1pf(vc);
        vc = vc < 0.0f ? 0.0f : (vc > 10.0f ? 10.0f : vc);
        float* ex = edge_x + (long)e * 6;
        ex[0] = (float)((double)log10f(g->t0[e] + 1.0f) / lt0);
        ex[1] = (float)((double)log10f(cap[e] + 1.0f) / lcap);
        ex[2] = vc;
        ex[3] = damaged[e];
        ex[4] = goal[e];
        ex[5] = (float)e / (float)(E > 1 ? E - 1 : 1);
        if (mask) mask[e] = damaged[e];
    }
}

int orc_observe_batch(const orc_graph* g, int B, const float* cap, const float* damaged, const float* goal,
                      const float* flow, const double* tstt, float* node_x, float* edge_x, float* mask,
                      int nthreads) {
    int N = g->N, E = g->E, err = 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads) reduction(| : err)
#endif
    {
        orc_obs_ws w;
        if (obs_ws_alloc(&w, N, E)) {
            err = 1;
        } else {
            obs_topology(g, &w);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
            for (int b = 0; b < B; b++)
                obs_one(g, &w, cap + (long)b * E, damaged + (long)b * E, goal + (long)b * E, flow + (long)b * E,
                        tstt[b], node_x + (long)b * N * 4, edge_x + (long)b * E * 6, mask ? mask + (long)b * E : NULL);
            obs_ws_free(&w);
        }
    }
    return err ? -1 : 0;
}

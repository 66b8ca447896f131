// damage_host.hip -- RepairEnv.reset's damage draw for a whole env batch, on
// the host (no device code): src/env/repair_env.py:167-192.
//
// Per env the reference draws `rng.choice(E, count, replace=False)` from its own
// numpy Generator (PCG64, seeded default_rng(seed)) up to 50 times until the
// subgraph of the still-active links is strongly connected (networkx DiGraph:
// one arc per (u, v), carrying the LAST link id added for it, repair_env.py:
// 107-109), else takes a 51st draw unchecked.  That loop, in Python with a
// networkx check per draw, costs ~0.5 ms per env (2 s per 4096-env reset on
// Sioux Falls, ~7.5 draws per env).  Here the Generator is restated exactly so
// the masks AND the generator states after the call are numpy's own:
//   PCG64 (XSL-RR 128/64, state advanced before output), next_uint32 halves of
//   a 64-bit draw with numpy's one-word buffer, random_bounded_uint64 for
//   ranges below 2^32 = Lemire's bounded uint32 with rejection, choice without
//   replacement for E <= 10000 = Floyd's algorithm (hash-set semantics: a repeat
//   draw inserts j) followed by the Fisher-Yates shuffle of the picks.
// Strong connectivity: forward and backward reachability from one incident node
// over the active arcs (CSR built once per call).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "trafficrl.h"
#include "trx_internal.h"

namespace trx {
namespace {

typedef unsigned __int128 u128;

struct Pcg {
    u128 state, inc;
    uint32_t has32, u32;

    uint64_t next64() {
        const u128 mult = ((u128)2549297995355413924ULL << 64) | (u128)4865540595714422341ULL;
        state = state * mult + inc;
        const uint64_t x = (uint64_t)(state >> 64) ^ (uint64_t)state;
        const unsigned rot = (unsigned)(state >> 122);
        return (x >> rot) | (x << ((64 - rot) & 63));
    }
    uint32_t next32() {
        if (has32) {
            has32 = 0;
            return u32;
        }
        const uint64_t v = next64();
        has32 = 1;
        u32 = (uint32_t)(v >> 32);
        return (uint32_t)v;
    }
    // random_bounded_uint64(off = 0, rng, use_masked = false) for rng < 2^32 - 1
    uint64_t bounded(uint32_t rng) {
        if (rng == 0) return 0;
        const uint32_t ex = rng + 1;
        uint64_t m = (uint64_t)next32() * ex;
        uint32_t left = (uint32_t)m;
        if (left < ex) {
            const uint32_t thr = (UINT32_MAX - rng) % ex;
            while (left < thr) {
                m = (uint64_t)next32() * ex;
                left = (uint32_t)m;
            }
        }
        return m >> 32;
    }
};

// Generator.choice(pop, size, replace=False), pop <= 10000 (Floyd + shuffle)
void choice(Pcg& g, int pop, int size, int32_t* out, std::vector<uint8_t>& in_set) {
    std::fill(in_set.begin(), in_set.end(), 0);
    for (int j = pop - size; j < pop; ++j) {
        const int v = (int)g.bounded((uint32_t)j);
        const int pick = in_set[v] ? j : v;
        in_set[pick] = 1;
        out[j - pop + size] = pick;
    }
    for (int i = size - 1; i >= 1; --i) {
        const int j = (int)g.bounded((uint32_t)i);
        std::swap(out[i], out[j]);
    }
}

struct Csr {
    std::vector<int32_t> off, arc;   // arc = representative link id of an (u, v) arc
};

bool reach_all(const Csr& c, const int32_t* other, const uint8_t* dead, int N, int s0, const std::vector<uint8_t>& need,
               std::vector<uint8_t>& seen, std::vector<int32_t>& stack) {
    std::fill(seen.begin(), seen.end(), 0);
    int sp = 0, cnt = 1, total = 0;
    for (int v = 0; v < N; ++v) total += need[v];
    seen[s0] = 1;
    stack[sp++] = s0;
    while (sp) {
        const int x = stack[--sp];
        for (int k = c.off[x]; k < c.off[x + 1]; ++k) {
            const int e = c.arc[k];
            if (dead[e]) continue;
            const int y = other[e];
            if (!seen[y]) {
                seen[y] = 1;
                cnt += need[y];
                stack[sp++] = y;
            }
        }
    }
    return cnt == total;
}

}  // namespace
}  // namespace trx

extern "C" int trx_damage_sample(int32_t num_nodes, int32_t num_edges, const int32_t* src, const int32_t* dst,
                                 int32_t count, int32_t max_tries, int32_t num_envs, trx_pcg64* rngs, float* out_mask,
                                 int32_t nthreads) {
    using namespace trx;
    const int N = num_nodes, E = num_edges;
    if (N <= 0 || E <= 0 || E > 10000 || !src || !dst || count < 1 || count > E || max_tries < 0 || num_envs < 0 ||
        (num_envs > 0 && (!rngs || !out_mask)))
        return trx::set_error(TRX_EINVAL, "damage_sample: need 1 <= count <= E <= 10000, N > 0, buffers");
    for (int e = 0; e < E; ++e)
        if (src[e] < 0 || src[e] >= N || dst[e] < 0 || dst[e] >= N)
            return trx::set_error(TRX_EINVAL, "damage_sample: link %d endpoint out of range", e);
    // DiGraph arcs: the last link added for each (u, v) carries the arc's edge_id
    std::vector<uint8_t> is_rep(E, 1);
    {
        std::vector<std::pair<int64_t, int>> key(E);
        for (int e = 0; e < E; ++e) key[e] = {(int64_t)src[e] * N + dst[e], e};
        std::sort(key.begin(), key.end());
        for (int i = 0; i + 1 < E; ++i)
            if (key[i].first == key[i + 1].first) is_rep[key[i].second] = 0;
    }
    Csr fwd, bwd;
    fwd.off.assign(N + 1, 0);
    bwd.off.assign(N + 1, 0);
    for (int e = 0; e < E; ++e)
        if (is_rep[e]) {
            ++fwd.off[src[e] + 1];
            ++bwd.off[dst[e] + 1];
        }
    for (int v = 0; v < N; ++v) {
        fwd.off[v + 1] += fwd.off[v];
        bwd.off[v + 1] += bwd.off[v];
    }
    fwd.arc.resize(fwd.off[N]);
    bwd.arc.resize(bwd.off[N]);
    {
        std::vector<int32_t> pf(fwd.off.begin(), fwd.off.end() - 1), pb(bwd.off.begin(), bwd.off.end() - 1);
        for (int e = 0; e < E; ++e)
            if (is_rep[e]) {
                fwd.arc[pf[src[e]]++] = e;
                bwd.arc[pb[dst[e]]++] = e;
            }
    }
    auto work = [&](int b0, int b1) {
        std::vector<uint8_t> in_set(E), dead(E), need(N), seen(N);
        std::vector<int32_t> pick(count), stack(N);
        for (int b = b0; b < b1; ++b) {
            trx_pcg64& r = rngs[b];
            Pcg g{((u128)r.state_hi << 64) | r.state_lo, ((u128)r.inc_hi << 64) | r.inc_lo, r.has_uint32, r.uinteger};
            bool found = false;
            for (int t = 0; t < max_tries && !found; ++t) {
                choice(g, E, count, pick.data(), in_set);
                std::fill(dead.begin(), dead.end(), 0);
                for (int k = 0; k < count; ++k) dead[pick[k]] = 1;
                std::fill(need.begin(), need.end(), 0);
                int s0 = -1, any = 0;
                for (int e = 0; e < E; ++e)
                    if (is_rep[e] && !dead[e]) {
                        need[src[e]] = need[dst[e]] = 1;
                        any = 1;
                        if (s0 < 0) s0 = src[e];
                    }
                if (!any) continue;   // `if not active_edges: continue`
                found = reach_all(fwd, dst, dead.data(), N, s0, need, seen, stack) &&
                        reach_all(bwd, src, dead.data(), N, s0, need, seen, stack);
            }
            if (!found) choice(g, E, count, pick.data(), in_set);
            float* m = out_mask + (size_t)b * E;
            std::fill(m, m + E, 0.0f);
            for (int k = 0; k < count; ++k) m[pick[k]] = 1.0f;
            r.state_hi = (uint64_t)(g.state >> 64);
            r.state_lo = (uint64_t)g.state;
            r.has_uint32 = g.has32;
            r.uinteger = g.u32;
        }
    };
    int nt = nthreads > 0 ? nthreads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    nt = std::max(1, std::min(nt, (num_envs + 63) / 64));
    if (nt == 1) {
        work(0, num_envs);
    } else {
        std::vector<std::thread> th;
        const int per = (num_envs + nt - 1) / nt;
        for (int i = 0; i < nt; ++i) {
            const int b0 = i * per, b1 = std::min(num_envs, b0 + per);
            if (b0 < b1) th.emplace_back(work, b0, b1);
        }
        for (auto& t : th) t.join();
    }
    return TRX_OK;
}

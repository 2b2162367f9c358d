// Contraction hierarchy for the GPU one-to-all sweeps (GPHAST-style).
//
// The reference computes every CPD row with a Dijkstra search per source
// inside warthog's make_cpd_auto (README.md:82-95, [U]).  A Dijkstra per row is
// a priority-queue walk — latency-bound and serial — so the GPU build instead
// computes d(n, t) for a batch of targets t with two linear sweeps over a
// contraction hierarchy (Geisberger et al. CH; Delling et al. PHAST/GPHAST):
//   up-sweep   (rank ascending):  d(x) = [x==t ? 0 : INF] min_{x->v, rank v<rank x} w + d(v)
//   down-sweep (rank descending): d(n) = min(d(n), min_{n->x, rank x>rank n} w + d(x))
// which yields exact shortest distances (every shortest path has an up-down
// witness in the CH overlay).  Nodes are grouped into levels so that a level
// only reads levels already finished; each level is one GPU launch.
//
// Contraction is done in parallel rounds: each round contracts an independent
// set of locally-minimal-priority nodes, with witness searches that avoid every
// node contracted in the same round (so simultaneous removal preserves
// distances).  A witness search that hits its settle limit adds the shortcut
// (conservative, always correct).  The result is deterministic for any thread
// count: every adjacency list is kept sorted and merges are grouped by owner.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <numeric>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "cpd_internal.hpp"

namespace cpd {
namespace {

struct Adj {
    uint32_t v;
    uint32_t w;
};

struct Shortcut {
    uint32_t u, x, w;
};

inline uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Per-thread bounded Dijkstra scratch with O(1) reset via stamps.
struct Witness {
    std::vector<uint64_t> dist;
    std::vector<uint32_t> stamp;
    std::vector<uint32_t> tstamp;  // tstamp[v] == cur: v is a target of this search
    uint32_t cur = 0;
    std::vector<std::pair<uint64_t, uint32_t>> heap;
    std::vector<std::pair<uint64_t, uint32_t>> tgt;  // (via, node), via descending

    explicit Witness(uint32_t n) : dist(n), stamp(n, 0), tstamp(n, 0) {}

    void reset() {
        if (++cur == 0) {
            std::fill(stamp.begin(), stamp.end(), 0);
            std::fill(tstamp.begin(), tstamp.end(), 0);
            cur = 1;
        }
        heap.clear();
    }
    uint64_t get(uint32_t v) const { return stamp[v] == cur ? dist[v] : UINT64_MAX; }
    void set(uint32_t v, uint64_t d) {
        stamp[v] = cur;
        dist[v] = d;
    }
    // Dijkstra from `src` over `out`, never entering `skip` or nodes with
    // avoid[] set, for the targets in `tgt` (set by the caller: (via, node),
    // sorted by via descending).  Stops after `settle` settled nodes, or once
    // the frontier passes the largest via of the targets not yet settled —
    // every settled target's distance is final, and an unsettled one can no
    // longer come in at or under its via.  (Round 2 ran on to the largest via
    // of ALL targets; the witness decisions, get(x) <= via, are the same.)
    void run(const std::vector<std::vector<Adj>>& out, uint32_t src, uint32_t skip,
             const uint8_t* avoid, uint32_t settle) {
        reset();
        for (const auto& t : tgt) tstamp[t.second] = cur;
        set(src, 0);
        heap.push_back({0, src});
        auto cmp = [](const std::pair<uint64_t, uint32_t>& a,
                      const std::pair<uint64_t, uint32_t>& b) { return a.first > b.first; };
        uint32_t settled = 0;
        size_t open = 0;  // tgt[open..]: the targets not yet settled start here (via order)
        auto advance = [&] {
            while (open < tgt.size() && stamp[tgt[open].second] == cur &&
                   tstamp[tgt[open].second] != cur)
                ++open;
        };
        while (!heap.empty()) {
            std::pop_heap(heap.begin(), heap.end(), cmp);
            auto [d, v] = heap.back();
            heap.pop_back();
            if (d != get(v)) continue;
            if (open == tgt.size() || d > tgt[open].first || ++settled > settle) break;
            if (tstamp[v] == cur) {  // a target settles: its distance is final
                tstamp[v] = cur - 1;
                advance();
            }
            for (const Adj& a : out[v]) {
                if (a.v == skip || (avoid && avoid[a.v])) continue;
                uint64_t nd = d + a.w;
                if (nd < get(a.v)) {
                    set(a.v, nd);
                    heap.push_back({nd, a.v});
                    std::push_heap(heap.begin(), heap.end(), cmp);
                }
            }
        }
    }
};

struct Contractor {
    uint32_t n;
    std::vector<std::vector<Adj>> out, in;
    std::vector<uint8_t> done, sel;
    std::vector<int64_t> prio;
    std::vector<uint32_t> deleted, depth;
    uint32_t settle_contract, settle_sim;
    std::vector<Witness> scratch;

    // Shortcuts needed to contract v through its in-neighbour ins[i] (avoid =
    // same-round nodes, or nullptr).  If `outv` is null only counts them.
    uint32_t shortcuts_via(uint32_t v, size_t i, const uint8_t* avoid, uint32_t settle,
                           std::vector<Shortcut>* outv, Witness& ws) const {
        const Adj& a = in[v][i];
        const auto& outs = out[v];
        ws.tgt.clear();
        for (const Adj& b : outs)
            if (b.v != a.v) ws.tgt.push_back({(uint64_t)a.w + b.w, b.v});
        if (ws.tgt.empty()) return 0;
        std::sort(ws.tgt.begin(), ws.tgt.end(),
                  [](const std::pair<uint64_t, uint32_t>& x, const std::pair<uint64_t, uint32_t>& y) {
                      return x.first != y.first ? x.first > y.first : x.second < y.second;
                  });
        ws.run(out, a.v, v, avoid, settle);
        uint32_t count = 0;
        for (const Adj& b : outs) {
            if (b.v == a.v) continue;
            uint64_t via = (uint64_t)a.w + b.w;
            if (ws.get(b.v) <= via) continue;
            ++count;
            if (outv) {
                if (via >= 0xFFFFFFFFull) throw Error(CPD_E_RANGE, "shortcut weight >= 2^32-1");
                outv->push_back({a.v, b.v, (uint32_t)via});
            }
        }
        return count;
    }
    uint32_t shortcuts(uint32_t v, const uint8_t* avoid, uint32_t settle,
                       std::vector<Shortcut>* outv, Witness& ws) const {
        if (in[v].empty() || out[v].empty()) return 0;
        uint32_t count = 0;
        for (size_t i = 0; i < in[v].size(); ++i) count += shortcuts_via(v, i, avoid, settle, outv, ws);
        return count;
    }

    // priority = a*edge difference + b*contracted neighbours + c*depth; depth
    // bounds the sweep levels.  Round 3 (profiles/ch_prio_ab/): 8,2,12 —
    // 166 + 159 levels, 5.20M arcs, 343k rows/s on the 1M bench graph —
    // against round 2's 8,2,3 (189 + 194 levels, 5.09M arcs, 338k rows/s):
    // fewer latency-bound narrow levels outweigh 2% more arcs (8,2,20 / 8,2,30:
    // 343-345k / 345.6k, with the down-sweep's arcs and time growing).
    int64_t prio_ed = 8, prio_del = 2, prio_depth = 12;

    int64_t priority_of(uint32_t v, int64_t sc) const {
        int64_t ed = sc - (int64_t)in[v].size() - (int64_t)out[v].size();
        return prio_ed * ed + prio_del * (int64_t)deleted[v] + prio_depth * (int64_t)depth[v];
    }
    int64_t priority(uint32_t v, Witness& ws) const {
        return priority_of(v, shortcuts(v, nullptr, settle_sim, nullptr, ws));
    }

    // ids: the contraction works on internal ids (the DFS preorder: graph
    // neighbours get nearby ids, so a witness search's scratch and lists stay
    // in cache); orig[] maps back.  Every order that can change the result —
    // adjacency lists, tie-breaks, the contraction order inside a round — is
    // by ORIGINAL id, so the hierarchy is the one the node ids alone define.
    std::vector<uint32_t> orig;

    bool less_key(uint32_t a, uint32_t b) const {
        if (prio[a] != prio[b]) return prio[a] < prio[b];
        const uint32_t oa = orig[a], ob = orig[b];
        uint64_t ha = mix(oa), hb = mix(ob);
        if (ha != hb) return ha < hb;
        return oa < ob;
    }
};

// Insert (v, w) into a list kept sorted by original id (keep the lighter
// weight of a parallel arc).
void merge_into(std::vector<Adj>& lst, uint32_t v, uint32_t w, const uint32_t* orig) {
    const uint32_t ov = orig[v];
    auto it = std::lower_bound(lst.begin(), lst.end(), ov,
                               [orig](const Adj& a, uint32_t key) { return orig[a.v] < key; });
    if (it != lst.end() && it->v == v) {
        if (w < it->w) it->w = w;
    } else {
        lst.insert(it, Adj{v, w});
    }
}

}  // namespace

Hierarchy build_hierarchy(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                          const uint32_t* w, int threads, uint32_t settle_limit,
                          int verbose) {
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#else
    threads = 1;
#endif
    Contractor C;
    C.n = n;
    C.out.assign(n, {});
    C.in.assign(n, {});
    C.done.assign(n, 0);
    C.sel.assign(n, 0);
    C.prio.assign(n, 0);
    C.deleted.assign(n, 0);
    C.depth.assign(n, 0);
    C.settle_contract = settle_limit ? settle_limit : 400;
    C.settle_sim = std::max<uint32_t>(50, C.settle_contract / 4);
    if (const char* e = std::getenv("CPD_CH_PRIO")) {  // tuning knob: "ed,deleted,depth"
        long a, b, c;
        if (std::sscanf(e, "%ld,%ld,%ld", &a, &b, &c) == 3) {
            C.prio_ed = a;
            C.prio_del = b;
            C.prio_depth = c;
        }
    }

    // Internal ids (see Contractor::orig): lab[node] = DFS preorder position.
    std::vector<uint32_t> lab(n);
    dfs_preorder(n, row_ptr, dst, lab.data());
    C.orig.assign(n, 0);
    for (uint32_t v = 0; v < n; ++v) C.orig[lab[v]] = v;
    const uint32_t* orig = C.orig.data();
    // Overlay graph: no self loops, parallel edges reduced to the lightest;
    // lists sorted by original id.
    for (uint32_t v = 0; v < n; ++v)
        for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
            if (dst[e] != v) merge_into(C.out[lab[v]], lab[dst[e]], w[e], orig);
    for (uint32_t v = 0; v < n; ++v)  // tails in original order: in-lists come out sorted
        for (const Adj& a : C.out[lab[v]]) C.in[a.v].push_back({lab[v], a.w});

    C.scratch.reserve(threads);
    for (int t = 0; t < threads; ++t) C.scratch.emplace_back(n);

    Hierarchy H;
    H.rank.assign(n, 0);
    std::vector<std::vector<Adj>> up(n);              // recorded up arcs per node
    std::vector<std::tuple<uint32_t, uint32_t, uint32_t>> dn;  // (u, v, w)
    dn.reserve((size_t)row_ptr[n] * 2);

    std::vector<uint32_t> remaining(n);  // internal ids in ORIGINAL id order
    for (uint32_t v = 0; v < n; ++v) remaining[v] = lab[v];

    const double t_init = now_seconds();
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
#ifdef _OPENMP
        Witness& ws = C.scratch[omp_get_thread_num()];
#else
        Witness& ws = C.scratch[0];
#endif
        C.prio[i] = C.priority((uint32_t)i, ws);
    }

    uint32_t next_rank = 0, round = 0;
    std::vector<uint32_t> S, affected;
    std::vector<std::vector<Shortcut>> sc_local;
    std::vector<std::pair<uint32_t, uint32_t>> pairs;  // (node, in-neighbour index)
    std::vector<uint32_t> pair_sc;
    double t0 = now_seconds();
    double tph[5] = {0, 0, 0, 0, 0};  // pick, contract, remove, insert, priorities (verbose)
    double ta = t0;
    auto phase = [&](int k) {
        const double tb = now_seconds();
        tph[k] += tb - ta;
        ta = tb;
    };
    while (!remaining.empty()) {
        // 1. independent set of local priority minima (1-hop, both directions)
        S.clear();
        std::vector<uint8_t> pick(remaining.size(), 0);
#pragma omp parallel for schedule(static) num_threads(threads)
        for (int64_t i = 0; i < (int64_t)remaining.size(); ++i) {
            uint32_t v = remaining[i];
            bool ok = true;
            for (const Adj& a : C.out[v])
                if (!C.less_key(v, a.v)) { ok = false; break; }
            if (ok)
                for (const Adj& a : C.in[v])
                    if (!C.less_key(v, a.v)) { ok = false; break; }
            pick[i] = ok;
        }
        for (size_t i = 0; i < remaining.size(); ++i)
            if (pick[i]) S.push_back(remaining[i]);
        for (uint32_t v : S) C.sel[v] = 1;

        phase(0);
        // 2. shortcuts for every selected node, avoiding all selected nodes:
        // one task per (node, in-neighbour) witness search, so that the few
        // high-degree nodes of the late rounds still spread over every thread
        pairs.clear();
        for (uint32_t v : S)
            if (!C.out[v].empty())
                for (size_t i = 0; i < C.in[v].size(); ++i) pairs.push_back({v, (uint32_t)i});
        sc_local.assign(pairs.size(), {});
        std::exception_ptr err;  // an exception must not leave the parallel region
#pragma omp parallel for schedule(dynamic, 8) num_threads(threads)
        for (int64_t i = 0; i < (int64_t)pairs.size(); ++i) {
#ifdef _OPENMP
            Witness& ws = C.scratch[omp_get_thread_num()];
#else
            Witness& ws = C.scratch[0];
#endif
            try {
                C.shortcuts_via(pairs[i].first, pairs[i].second, C.sel.data(), C.settle_contract,
                                &sc_local[i], ws);
            } catch (...) {
#pragma omp critical(ch_err)
                if (!err) err = std::current_exception();
            }
        }
        if (err) std::rethrow_exception(err);

        phase(1);
        // 3. record hierarchy arcs, ranks
        for (uint32_t v : S) {
            const uint32_t ov = orig[v];
            H.rank[ov] = next_rank++;
            up[ov] = C.out[v];
            for (Adj& a : up[ov]) a.v = orig[a.v];
            for (const Adj& a : C.in[v]) dn.emplace_back(orig[a.v], ov, a.w);
        }

        // 4. remove S from the neighbours' lists; depth / deleted counters
        affected.clear();
        for (uint32_t v : S) {
            for (const Adj& a : C.out[v]) affected.push_back(a.v);
            for (const Adj& a : C.in[v]) affected.push_back(a.v);
        }
        std::sort(affected.begin(), affected.end());
        affected.erase(std::unique(affected.begin(), affected.end()), affected.end());
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
        for (int64_t i = 0; i < (int64_t)affected.size(); ++i) {
            uint32_t u = affected[i];
            uint32_t removed = 0, dep = C.depth[u];
            auto drop = [&](std::vector<Adj>& lst) {
                size_t k = 0;
                for (const Adj& a : lst) {
                    if (C.sel[a.v]) {
                        ++removed;
                        dep = std::max(dep, C.depth[a.v] + 1);
                    } else {
                        lst[k++] = a;
                    }
                }
                lst.resize(k);
            };
            drop(C.out[u]);
            drop(C.in[u]);
            C.deleted[u] += removed;
            C.depth[u] = dep;
        }
        for (uint32_t v : S) {
            C.done[v] = 1;
            std::vector<Adj>().swap(C.out[v]);
            std::vector<Adj>().swap(C.in[v]);
        }

        phase(2);
        // 5. insert shortcuts, grouped by owner list for determinism
        std::vector<Shortcut> all;
        for (auto& l : sc_local) all.insert(all.end(), l.begin(), l.end());
        auto by_u = [](const Shortcut& a, const Shortcut& b) {
            return a.u != b.u ? a.u < b.u : (a.x != b.x ? a.x < b.x : a.w < b.w);
        };
        auto by_x = [](const Shortcut& a, const Shortcut& b) {
            return a.x != b.x ? a.x < b.x : (a.u != b.u ? a.u < b.u : a.w < b.w);
        };
        std::sort(all.begin(), all.end(), by_u);
        std::vector<size_t> starts;
        for (size_t i = 0; i < all.size(); ++i)
            if (i == 0 || all[i].u != all[i - 1].u) starts.push_back(i);
        starts.push_back(all.size());
        int64_t ngroups = (int64_t)starts.size() - 1;
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
        for (int64_t g = 0; g < ngroups; ++g)
            for (size_t i = starts[g]; i < starts[g + 1]; ++i)
                merge_into(C.out[all[i].u], all[i].x, all[i].w, orig);
        std::sort(all.begin(), all.end(), by_x);
        starts.clear();
        for (size_t i = 0; i < all.size(); ++i)
            if (i == 0 || all[i].x != all[i - 1].x) starts.push_back(i);
        starts.push_back(all.size());
        ngroups = (int64_t)starts.size() - 1;
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
        for (int64_t g = 0; g < ngroups; ++g)
            for (size_t i = starts[g]; i < starts[g + 1]; ++i)
                merge_into(C.in[all[i].x], all[i].u, all[i].w, orig);
        // shortcut endpoints changed degree: their priority is stale too
        for (const Shortcut& s : all) {
            affected.push_back(s.u);
            affected.push_back(s.x);
        }
        std::sort(affected.begin(), affected.end());
        affected.erase(std::unique(affected.begin(), affected.end()), affected.end());

        for (uint32_t v : S) C.sel[v] = 0;

        phase(3);
        // 6. priorities of affected nodes (again one task per witness search),
        // then drop S from `remaining`
        pairs.clear();
        for (uint32_t u : affected)
            if (!C.done[u] && !C.out[u].empty())
                for (size_t i = 0; i < C.in[u].size(); ++i) pairs.push_back({u, (uint32_t)i});
        pair_sc.assign(pairs.size(), 0);
#pragma omp parallel for schedule(dynamic, 16) num_threads(threads)
        for (int64_t i = 0; i < (int64_t)pairs.size(); ++i) {
#ifdef _OPENMP
            Witness& ws = C.scratch[omp_get_thread_num()];
#else
            Witness& ws = C.scratch[0];
#endif
            pair_sc[i] = C.shortcuts_via(pairs[i].first, pairs[i].second, nullptr, C.settle_sim,
                                         nullptr, ws);
        }
        {
            size_t k = 0;
            for (uint32_t u : affected) {
                if (C.done[u]) continue;
                int64_t sc = 0;
                while (k < pairs.size() && pairs[k].first == u) sc += pair_sc[k++];
                C.prio[u] = C.priority_of(u, sc);
            }
        }
        size_t k = 0;
        for (uint32_t v : remaining)
            if (!C.done[v]) remaining[k++] = v;
        remaining.resize(k);
        phase(4);
        ++round;
        if (verbose && (round % 10 == 0 || remaining.empty()))
            std::fprintf(stderr, "[ch] round %u contracted %zu remaining %zu pairs %zu (%.1fs) prio %.2f\n",
                         round, S.size(), remaining.size(), pairs.size(), now_seconds() - t0, tph[4]);
    }
    C.scratch.clear();
    if (verbose)
        std::fprintf(stderr,
                     "[ch] initial priorities %.2fs; rounds: pick %.2f contract %.2f remove %.2f "
                     "insert %.2f priorities %.2f s\n",
                     t0 - t_init, tph[0], tph[1], tph[2], tph[3], tph[4]);

    // Hierarchy CSRs (node space, sorted by head for determinism).
    H.up_off.assign(n + 1, 0);
    for (uint32_t v = 0; v < n; ++v) H.up_off[v + 1] = H.up_off[v] + up[v].size();
    H.up_dst.resize(H.up_off[n]);
    H.up_w.resize(H.up_off[n]);
    for (uint32_t v = 0; v < n; ++v) {
        uint64_t p = H.up_off[v];
        for (const Adj& a : up[v]) {
            H.up_dst[p] = a.v;
            H.up_w[p] = a.w;
            ++p;
        }
        std::vector<Adj>().swap(up[v]);
    }
    std::sort(dn.begin(), dn.end());
    H.dn_off.assign(n + 1, 0);
    for (auto& t : dn) H.dn_off[std::get<0>(t) + 1]++;
    for (uint32_t v = 0; v < n; ++v) H.dn_off[v + 1] += H.dn_off[v];
    H.dn_dst.resize(dn.size());
    H.dn_w.resize(dn.size());
    for (size_t i = 0; i < dn.size(); ++i) {
        H.dn_dst[i] = std::get<1>(dn[i]);
        H.dn_w[i] = std::get<2>(dn[i]);
    }

    hierarchy_levels(H, n);
    if (verbose)
        std::fprintf(stderr,
                     "[ch] %u rounds, up arcs %llu, down arcs %llu, levels up %u down %u "
                     "(%.1fs)\n",
                     round, (unsigned long long)H.up_off[n],
                     (unsigned long long)H.dn_off[n], H.nlev_up, H.nlev_dn,
                     now_seconds() - t0);
    return H;
}

// Sweep levels of a finished hierarchy: level_up[x] = 1 + max level_up of
// x's down-arc heads (rank ascending), level_dn[v] = 1 + max level_dn of v's
// up-arc heads (rank descending).
void hierarchy_levels(Hierarchy& H, uint32_t n) {
    std::vector<uint32_t> by_rank(n);
    for (uint32_t v = 0; v < n; ++v) by_rank[H.rank[v]] = v;
    H.level_up.assign(n, 0);
    H.level_dn.assign(n, 0);
    uint32_t mu = 0, md = 0;
    for (uint32_t r = 0; r < n; ++r) {
        uint32_t x = by_rank[r], l = 0;
        for (uint64_t e = H.dn_off[x]; e < H.dn_off[x + 1]; ++e)
            l = std::max(l, H.level_up[H.dn_dst[e]] + 1);
        H.level_up[x] = l;
        mu = std::max(mu, l);
    }
    for (uint32_t r = n; r-- > 0;) {
        uint32_t v = by_rank[r], l = 0;
        for (uint64_t e = H.up_off[v]; e < H.up_off[v + 1]; ++e)
            l = std::max(l, H.level_dn[H.up_dst[e]] + 1);
        H.level_dn[v] = l;
        md = std::max(md, l);
    }
    H.nlev_up = mu + 1;
    H.nlev_dn = md + 1;
}

}  // namespace cpd

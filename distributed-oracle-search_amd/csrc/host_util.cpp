// Host utilities behind the C ABI: error channel, partitioner, DFS column
// order, CSR validation, distance bound, synthetic road graphs.
#include <sys/statvfs.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>
#include <queue>
#include <thread>

#include "cpd_internal.hpp"
#include "src_sha.h"

namespace cpd {

static thread_local std::string g_last_error = "no error";

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

double now_seconds() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

void check_csr(uint32_t n, uint32_t m, const uint32_t* row_ptr,
               const uint32_t* dst, const uint32_t* w) {
    CPD_REQUIRE(row_ptr && (m == 0 || (dst && w)), CPD_E_ARG, "null graph array");
    CPD_REQUIRE(n > 0, CPD_E_ARG, "graph has no nodes");
    CPD_REQUIRE(n < (1u << 28), CPD_E_RANGE,
                "N >= 2^28 does not fit the 28-bit run start column");
    CPD_REQUIRE(row_ptr[0] == 0 && row_ptr[n] == m, CPD_E_ARG,
                "row_ptr must start at 0 and end at m");
    for (uint32_t v = 0; v < n; ++v) {
        CPD_REQUIRE(row_ptr[v] <= row_ptr[v + 1], CPD_E_ARG,
                    "row_ptr not monotone");
        uint32_t deg = row_ptr[v + 1] - row_ptr[v];
        if (deg > CPD_MAX_DEGREE)
            throw Error(CPD_E_RANGE, "node " + std::to_string(v) + " has out-degree " +
                                         std::to_string(deg) +
                                         " > 15 (4-bit move field)");
    }
    for (uint32_t e = 0; e < m; ++e)
        CPD_REQUIRE(dst[e] < n, CPD_E_ARG, "edge head out of range");
}

// Iterative DFS preorder, warthog cpd::compute_dfs_preorder [U].
void dfs_preorder(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                  uint32_t* order) {
    const uint32_t UNSET = 0xFFFFFFFFu;
    std::fill(order, order + n, UNSET);
    std::vector<uint32_t> stack;
    stack.reserve(1024);
    uint32_t next = 0;
    for (uint32_t root = 0; root < n; ++root) {
        if (order[root] != UNSET) continue;
        stack.push_back(root);
        while (!stack.empty()) {
            uint32_t v = stack.back();
            stack.pop_back();
            if (order[v] != UNSET) continue;
            order[v] = next++;
            for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
                if (order[dst[e]] == UNSET) stack.push_back(dst[e]);
        }
    }
}

// Dijkstra (u64) from `src` over the CSR given; returns max finite distance
// and whether every node was reached.
static uint64_t eccentricity(uint32_t n, const uint64_t* off, const uint32_t* to,
                             const uint32_t* wt, uint32_t src, bool* all) {
    std::vector<uint64_t> d(n, UINT64_MAX);
    using QE = std::pair<uint64_t, uint32_t>;
    std::priority_queue<QE, std::vector<QE>, std::greater<QE>> pq;
    d[src] = 0;
    pq.push({0, src});
    uint64_t mx = 0;
    uint32_t settled = 0;
    while (!pq.empty()) {
        auto [dv, v] = pq.top();
        pq.pop();
        if (dv != d[v]) continue;
        ++settled;
        mx = std::max(mx, dv);
        for (uint64_t e = off[v]; e < off[v + 1]; ++e) {
            uint64_t nd = dv + wt[e];
            if (nd < d[to[e]]) {
                d[to[e]] = nd;
                pq.push({nd, to[e]});
            }
        }
    }
    *all = settled == n;
    return mx;
}

// Bound on every finite d(a,b): via a root r, d(a,b) <= d(a,r) + d(r,b) when the
// graph is strongly connected; otherwise the trivial (n-1) * w_max.
uint64_t distance_bound(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                        const uint32_t* w) {
    uint32_t m = row_ptr[n];
    uint64_t wmax = 0;
    for (uint32_t e = 0; e < m; ++e) wmax = std::max<uint64_t>(wmax, w[e]);
    uint64_t trivial = wmax * (uint64_t)(n - 1);
    if (m == 0) return 0;
    std::vector<uint64_t> off(n + 1);
    for (uint32_t v = 0; v <= n; ++v) off[v] = row_ptr[v];
    bool all_f = false, all_b = false;
    uint64_t ef = 0, eb = 0;
    // the forward search runs on its own thread beside the reversal + the
    // backward search
    std::thread fwd([&] { ef = eccentricity(n, off.data(), dst, w, 0, &all_f); });
    struct Join {
        std::thread& t;
        ~Join() {
            if (t.joinable()) t.join();
        }
    } join{fwd};
    // reverse graph
    std::vector<uint64_t> roff(n + 1, 0);
    std::vector<uint32_t> rto(m), rw(m);
    for (uint32_t e = 0; e < m; ++e) roff[dst[e] + 1]++;
    for (uint32_t v = 0; v < n; ++v) roff[v + 1] += roff[v];
    std::vector<uint64_t> pos(roff.begin(), roff.end() - 1);
    for (uint32_t v = 0; v < n; ++v)
        for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) {
            uint64_t p = pos[dst[e]]++;
            rto[p] = v;
            rw[p] = w[e];
        }
    eb = eccentricity(n, roff.data(), rto.data(), rw.data(), 0, &all_b);
    fwd.join();
    if (all_f && all_b) return std::min(trivial, ef + eb);
    return trivial;
}

// ---------------------------------------------------------------------------
// Synthetic grid-perturbed road graphs.  splitmix64 RNG so the
// output is identical on every host.
struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    uint32_t below(uint32_t k) { return (uint32_t)(((next() >> 32) * (uint64_t)k) >> 32); }
};

template <class T>
static void shuffle(std::vector<T>& v, Rng& r) {
    for (size_t i = v.size(); i > 1; --i) std::swap(v[i - 1], v[r.below((uint32_t)i)]);
}

struct SynthGraph {
    uint32_t n = 0;
    std::vector<uint32_t> row_ptr, dst, w;
    std::vector<int32_t> x, y;
};

static uint32_t uf_find(std::vector<uint32_t>& p, uint32_t a) {
    while (p[a] != a) {
        p[a] = p[p[a]];
        a = p[a];
    }
    return a;
}

// flags (CPD_SYNTH_*): SHUFFLE_IDS permutes node ids (else id = row-major
// lattice cell), ONE_WAY makes a fifth of the extra lattice edges one-way
// (else every edge is bidirectional), SHUFFLE_EDGES shuffles each node's
// out-edge order (else east, north, west, south).  The RNG stream is the same
// for every flag set, so the lattice, tree, extras and weights do not depend
// on the flags beyond what they switch.
static SynthGraph synth(uint32_t W, uint32_t H, double mean_outdeg, uint64_t seed,
                        uint32_t flags = CPD_SYNTH_SHUFFLED) {
    CPD_REQUIRE(W >= 2 && H >= 2, CPD_E_ARG, "lattice must be at least 2x2");
    CPD_REQUIRE((uint64_t)W * H < (1u << 28), CPD_E_RANGE, "lattice too large");
    CPD_REQUIRE(mean_outdeg >= 2.0 && mean_outdeg <= 4.0, CPD_E_ARG,
                "mean out-degree must be in [2, 4]");
    CPD_REQUIRE((flags & ~CPD_SYNTH_SHUFFLED) == 0, CPD_E_ARG, "unknown synth flags");
    Rng rng(seed);
    const uint32_t n = W * H;
    SynthGraph g;
    g.n = n;
    // node ids: random permutation, or the lattice cell itself
    std::vector<uint32_t> id(n);
    std::iota(id.begin(), id.end(), 0u);
    shuffle(id, rng);  // drawn either way (same RNG stream for every flag set)
    if (!(flags & CPD_SYNTH_SHUFFLE_IDS)) std::iota(id.begin(), id.end(), 0u);
    std::vector<int32_t> gx(n), gy(n);
    for (uint32_t j = 0; j < H; ++j)
        for (uint32_t i = 0; i < W; ++i) {
            uint32_t c = j * W + i;
            gx[c] = (int32_t)(i * 1000) + (int32_t)rng.below(601) - 300;
            gy[c] = (int32_t)(j * 1000) + (int32_t)rng.below(601) - 300;
        }
    // lattice edges (cell pairs)
    std::vector<std::pair<uint32_t, uint32_t>> lat;
    lat.reserve(2ull * n);
    for (uint32_t j = 0; j < H; ++j)
        for (uint32_t i = 0; i < W; ++i) {
            uint32_t c = j * W + i;
            if (i + 1 < W) lat.push_back({c, c + 1});
            if (j + 1 < H) lat.push_back({c, c + W});
        }
    shuffle(lat, rng);
    // random spanning tree (Kruskal over the shuffled lattice)
    std::vector<uint32_t> parent(n);
    std::iota(parent.begin(), parent.end(), 0u);
    std::vector<char> in_tree(lat.size(), 0);
    for (size_t k = 0; k < lat.size(); ++k) {
        uint32_t a = uf_find(parent, lat[k].first), b = uf_find(parent, lat[k].second);
        if (a != b) {
            parent[a] = b;
            in_tree[k] = 1;
        }
    }
    // directed arcs (cell space): tree edges both ways; extras until the target
    struct Arc { uint32_t a, b, wt; };
    std::vector<Arc> arcs;
    uint64_t target_arcs = (uint64_t)std::llround(mean_outdeg * n);
    arcs.reserve(target_arcs + 4);
    auto weight = [&](uint32_t a, uint32_t b, double speed) {
        double dx = gx[a] - gx[b], dy = gy[a] - gy[b];
        double asym = 1.0 + 0.15 * rng.uniform();
        double v = std::ceil(std::sqrt(dx * dx + dy * dy) * speed * asym / 10.0);
        return (uint32_t)std::min(65535.0, std::max(1.0, v));
    };
    for (size_t k = 0; k < lat.size(); ++k) {
        if (!in_tree[k]) continue;
        double speed = 0.6 + 0.8 * rng.uniform();
        arcs.push_back({lat[k].first, lat[k].second, weight(lat[k].first, lat[k].second, speed)});
        arcs.push_back({lat[k].second, lat[k].first, weight(lat[k].second, lat[k].first, speed)});
    }
    for (size_t k = 0; k < lat.size() && arcs.size() < target_arcs; ++k) {
        if (in_tree[k]) continue;
        double speed = 0.6 + 0.8 * rng.uniform();
        uint32_t a = lat[k].first, b = lat[k].second;
        const bool one_way = rng.uniform() < 0.2;
        const bool flip = one_way && rng.uniform() < 0.5;  // drawn under every flag set
        if (one_way && (flags & CPD_SYNTH_ONE_WAY)) {  // one-way street, random direction
            if (flip) std::swap(a, b);
            arcs.push_back({a, b, weight(a, b, speed)});
        } else {
            arcs.push_back({a, b, weight(a, b, speed)});
            arcs.push_back({b, a, weight(b, a, speed)});
        }
    }
    // CSR in node-id space; per-node out-edge order shuffled or by direction
    const uint32_t m = (uint32_t)arcs.size();
    if (!(flags & CPD_SYNTH_SHUFFLE_EDGES)) {
        // east, north, west, south (cell space): the k-th out-edge of every
        // node points the same way wherever that way has an edge
        auto dir = [W](const Arc& a) {
            return a.b == a.a + 1 ? 0 : a.b == a.a + W ? 1 : a.b + 1 == a.a ? 2 : 3;
        };
        std::stable_sort(arcs.begin(), arcs.end(), [&](const Arc& x, const Arc& y) {
            return x.a != y.a ? x.a < y.a : dir(x) < dir(y);
        });
    }
    g.row_ptr.assign(n + 1, 0);
    for (auto& a : arcs) g.row_ptr[id[a.a] + 1]++;
    for (uint32_t v = 0; v < n; ++v) g.row_ptr[v + 1] += g.row_ptr[v];
    g.dst.resize(m);
    g.w.resize(m);
    std::vector<uint32_t> pos(g.row_ptr.begin(), g.row_ptr.end() - 1);
    for (auto& a : arcs) {
        uint32_t p = pos[id[a.a]]++;
        g.dst[p] = id[a.b];
        g.w[p] = a.wt;
    }
    for (uint32_t v = 0; v < n; ++v) {
        uint32_t b = g.row_ptr[v], e = g.row_ptr[v + 1];
        for (uint32_t i = e - b; i > 1; --i) {
            uint32_t j = rng.below(i);
            if (!(flags & CPD_SYNTH_SHUFFLE_EDGES)) continue;  // drawn, not applied
            std::swap(g.dst[b + i - 1], g.dst[b + j]);
            std::swap(g.w[b + i - 1], g.w[b + j]);
        }
    }
    g.x.resize(n);
    g.y.resize(n);
    for (uint32_t c = 0; c < n; ++c) {
        g.x[id[c]] = gx[c];
        g.y[id[c]] = gy[c];
    }
    return g;
}

}  // namespace cpd

using namespace cpd;

extern "C" {

const char* cpd_last_error(void) { return g_last_error.c_str(); }

// CPD_SRC_SHA: sha256 (16 hex) of the sources this library was built from
// (Makefile PROV_SRCS; cpd.src_sha() recomputes it from a tree).
const char* cpd_version(void) { return "cpd-mi355x 0.3 gfx950 src:" CPD_SRC_SHA; }

int cpd_partition_nbuckets(uint32_t nodenum, int method, uint32_t key,
                           uint32_t* nbuckets) {
    return guarded([&] {
        CPD_REQUIRE(nbuckets && key > 0 && nodenum > 0, CPD_E_ARG,
                    "partition needs nodenum > 0 and partkey > 0");
        if (method == CPD_PART_MOD) {
            *nbuckets = std::min(key, nodenum);
        } else if (method == CPD_PART_DIV) {
            uint32_t chunk = (uint32_t)(((uint64_t)nodenum + key - 1) / key);
            *nbuckets = (nodenum + chunk - 1) / chunk;
        } else {
            throw Error(CPD_E_ARG, "partmethod must be div or mod");
        }
    });
}

int cpd_partition(uint32_t nodenum, uint32_t maxworker, int method, uint32_t key,
                  uint32_t node, uint32_t* wid, uint32_t* bid, uint32_t* bidx) {
    // No guarded(): this is called once per node by gen_distribute_conf.
    if (!wid || !bid || !bidx || key == 0 || maxworker == 0 || node >= nodenum)
        return fail(CPD_E_ARG, "partition: bad argument");
    uint32_t b, i;
    if (method == CPD_PART_MOD) {
        b = node % key;
        i = node / key;
    } else if (method == CPD_PART_DIV) {
        uint32_t chunk = (uint32_t)(((uint64_t)nodenum + key - 1) / key);
        b = node / chunk;
        i = node % chunk;
    } else {
        return fail(CPD_E_ARG, "partmethod must be div or mod");
    }
    *bid = b;
    *bidx = i;
    *wid = b % maxworker;
    return CPD_OK;
}

int cpd_bucket_bytes(uint32_t n, uint32_t bits, uint64_t nrows, uint32_t nbuckets,
                     uint32_t stripes, uint64_t* bytes) {
    return guarded([&] {
        CPD_REQUIRE(bytes && (bits == 1 || bits == 2 || bits == 4) && stripes >= 1, CPD_E_ARG,
                    "bucket bytes: bits must be 1, 2 or 4, stripes >= 1");
        // rows at ceil(n bits / 32) words, 8 B of target + count per row, a
        // header per bucket file (rounded to 4 KiB; DOSCPD02 pads its rows to
        // 4 KiB) and per part file a block of slack
        const uint64_t words = ((uint64_t)n * bits + 31u) / 32u;
        *bytes = nrows * (4ull * words + 8ull) + (uint64_t)nbuckets * (1ull + stripes) * 4096ull;
    });
}

int cpd_space_check(const char* dir, uint64_t bytes, uint64_t* avail) {
    return guarded([&] {
        CPD_REQUIRE(dir, CPD_E_ARG, "space check: null directory");
        struct statvfs sv {};
        if (::statvfs(dir, &sv) != 0)
            throw Error(CPD_E_IO, std::string("cannot stat the file system of ") + dir);
        const uint64_t have = (uint64_t)sv.f_bavail * (uint64_t)sv.f_frsize;
        if (avail) *avail = have;
        if (have < bytes)
            throw Error(CPD_E_IO, std::string(dir) + " has " + std::to_string(have >> 20) +
                                      " MiB free, the worker's bucket files need " +
                                      std::to_string((bytes + (1u << 20) - 1) >> 20) + " MiB");
    });
}

int cpd_dfs_preorder(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                     uint32_t* order) {
    return guarded([&] {
        CPD_REQUIRE(order && row_ptr && n > 0, CPD_E_ARG, "dfs: bad argument");
        CPD_REQUIRE(row_ptr[n] == 0 || dst, CPD_E_ARG, "dfs: null dst");
        dfs_preorder(n, row_ptr, dst, order);
    });
}

int cpd_synth_road_graph(uint32_t width, uint32_t height, double mean_outdeg,
                         uint64_t seed, uint32_t* n, uint32_t* m,
                         uint32_t* row_ptr, uint32_t* dst, uint32_t* w,
                         int32_t* x, int32_t* y) {
    return cpd_synth_road_graph_ex(width, height, mean_outdeg, seed, CPD_SYNTH_SHUFFLED, n, m,
                                   row_ptr, dst, w, x, y);
}

int cpd_synth_road_graph_ex(uint32_t width, uint32_t height, double mean_outdeg,
                            uint64_t seed, uint32_t flags, uint32_t* n, uint32_t* m,
                            uint32_t* row_ptr, uint32_t* dst, uint32_t* w,
                            int32_t* x, int32_t* y) {
    return guarded([&] {
        CPD_REQUIRE(n && m, CPD_E_ARG, "synth: n/m outputs required");
        SynthGraph g = synth(width, height, mean_outdeg, seed, flags);
        uint32_t gm = (uint32_t)g.dst.size();
        if (!row_ptr) {
            *n = g.n;
            *m = gm;
            return;
        }
        CPD_REQUIRE(*n == g.n && *m == gm, CPD_E_ARG,
                    "synth: buffer sizes do not match the size query");
        CPD_REQUIRE(dst && w, CPD_E_ARG, "synth: null output");
        std::memcpy(row_ptr, g.row_ptr.data(), (g.n + 1) * sizeof(uint32_t));
        std::memcpy(dst, g.dst.data(), gm * sizeof(uint32_t));
        std::memcpy(w, g.w.data(), gm * sizeof(uint32_t));
        if (x) std::memcpy(x, g.x.data(), g.n * sizeof(int32_t));
        if (y) std::memcpy(y, g.y.data(), g.n * sizeof(int32_t));
    });
}

int cpd_synth_congestion(uint32_t m, const uint32_t* w, double frac, double lo,
                         double hi, uint64_t seed, uint32_t* w_out) {
    return guarded([&] {
        CPD_REQUIRE(w && w_out, CPD_E_ARG, "congestion: null array");
        CPD_REQUIRE(frac >= 0 && frac <= 1 && lo >= 1.0 && hi >= lo, CPD_E_ARG,
                    "congestion: need 0<=frac<=1 and 1<=lo<=hi (weights only increase)");
        Rng rng(seed);
        for (uint32_t e = 0; e < m; ++e) {
            double pick = rng.uniform();
            double f = lo + (hi - lo) * rng.uniform();
            if (pick < frac) {
                double v = std::ceil((double)w[e] * f);
                w_out[e] = (uint32_t)std::min(4294967294.0, v);
            } else {
                w_out[e] = w[e];
            }
        }
    });
}

}  // extern "C"

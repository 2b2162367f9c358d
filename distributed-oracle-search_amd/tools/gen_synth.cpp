// bin/gen_synth — synthetic stand-ins for the reference's missing data blobs
// (melb-both.xy, melb-both.xy.diff, full.scen: .MISSING_LARGE_BLOBS:1-3),
// following SURVEY.md §8d:
//
//   gen_synth --width W --height H --seed S --out PREFIX [--outdeg 2.5]
//             [--diff-frac 0.1 --diff-lo 1 --diff-hi 3 --diff-seed 3]
//             [--queries Q --query-seed 2 [--sample K --sample-seed 5]]
//
// writes PREFIX.xy, PREFIX.xy.diff and (with --queries) PREFIX.scen, whose
// targets are uniform over all nodes or over a K-node sample.
#include <algorithm>
#include <cstdio>
#include <numeric>
#include <vector>

#include "cli.hpp"
#include "cpd_io.hpp"

struct SplitMix {
    uint64_t s;
    explicit SplitMix(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t k) { return (uint32_t)(((next() >> 32) * (uint64_t)k) >> 32); }
};

int main(int argc, char** argv) {
    cli::Args a(argc, argv);
    long long W = a.num("width", -1), H = a.num("height", W);
    std::string out = a.str("out");
    if (W < 2 || H < 2 || out.empty()) {
        std::fprintf(stderr, "usage: gen_synth --width W [--height H] --seed S --out PREFIX [--style shuffled|spec] ...\n");
        return 2;
    }
    uint64_t seed = (uint64_t)a.num("seed", 1);
    double outdeg = std::atof(a.str("outdeg", "2.5").c_str());
    // --style shuffled (default; round-1 graphs) | spec (SURVEY.md §8d as
    // written: row-major ids, bidirectional edges, E/N/W/S out-edge order)
    const std::string style = a.str("style", "shuffled");
    if (style != "shuffled" && style != "spec") {
        std::fprintf(stderr, "gen_synth: --style must be shuffled or spec\n");
        return 2;
    }
    const uint32_t flags = style == "spec" ? 0u : CPD_SYNTH_SHUFFLED;
    uint32_t n = 0, m = 0;
    cli::check(cpd_synth_road_graph_ex((uint32_t)W, (uint32_t)H, outdeg, seed, flags, &n, &m, nullptr,
                                       nullptr, nullptr, nullptr, nullptr),
               "synth");
    cpd::io::XYGraph g;
    g.n = n;
    g.m = m;
    g.row_ptr.resize(n + 1);
    g.dst.resize(m);
    g.w.resize(m);
    g.x.resize(n);
    g.y.resize(n);
    cli::check(cpd_synth_road_graph_ex((uint32_t)W, (uint32_t)H, outdeg, seed, flags, &n, &m,
                                       g.row_ptr.data(), g.dst.data(), g.w.data(), g.x.data(),
                                       g.y.data()),
               "synth");
    try {
        cpd::io::write_xy(out + ".xy", n, g.row_ptr.data(), g.dst.data(), g.w.data(), g.x.data(),
                          g.y.data());
        std::vector<uint32_t> wc(m);
        double frac = std::atof(a.str("diff-frac", "0.1").c_str());
        double lo = std::atof(a.str("diff-lo", "1.0").c_str());
        double hi = std::atof(a.str("diff-hi", "3.0").c_str());
        cli::check(cpd_synth_congestion(m, g.w.data(), frac, lo, hi, (uint64_t)a.num("diff-seed", 3),
                                        wc.data()),
                   "congestion");
        cpd::io::write_diff(out + ".xy.diff", g, wc);
        long long Q = a.num("queries", 0);
        if (Q > 0) {
            std::vector<uint32_t> pool;
            long long K = a.num("sample", 0);
            if (K > 0 && K < n) {
                std::vector<uint32_t> all(n);
                std::iota(all.begin(), all.end(), 0u);
                SplitMix r((uint64_t)a.num("sample-seed", 5));
                for (long long i = 0; i < K; ++i) std::swap(all[i], all[i + r.below((uint32_t)(n - i))]);
                pool.assign(all.begin(), all.begin() + K);
            }
            SplitMix r((uint64_t)a.num("query-seed", 2));
            cpd::io::Pairs q;
            q.reserve((size_t)Q);
            while ((long long)q.size() < Q) {
                uint32_t s = r.below(n);
                uint32_t t = pool.empty() ? r.below(n) : pool[r.below((uint32_t)pool.size())];
                if (s != t) q.push_back({s, t});
            }
            cpd::io::write_scen(out + ".scen", q);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "gen_synth: %s\n", e.what());
        return 1;
    }
    std::printf("gen_synth: %u nodes %u edges -> %s.xy\n", n, m, out.c_str());
    return 0;
}

// bin/make_cpd_auto — drop-in for warthog's make_cpd_auto (README.md:82-95),
// launched per worker by make_cpds.py:20-21:
//
//   make_cpd_auto --input X.xy --partmethod {div|mod} --partkey K
//                 --workerid I --maxworker W --outdir D
//                 [--partition M]      README.md:89 spelling of --partmethod
//                 [--device G]         default: I % (visible GPUs)
//                 [--batch B]          rows per GPU sweep (multiple of 1024)
//                 [--threads T]        host threads for the hierarchy build
//                 [--plan P | --no-plan-cache]
//
// Builds the CPD rows of every target this worker owns under the
// distribution_controller partition, on the GPU, and writes one file per
// owned bucket into D (README.md:92-93 "one or more CPDs ... auto-generated
// names").  The launcher is fire-and-forget (tmux, make_cpds.py:21), so timing
// is printed here.
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "cli.hpp"
#include "cpd_io.hpp"

using cpd::io::CpdBucket;

static double now() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

static std::string dir_of(const std::string& p) {
    size_t s = p.find_last_of('/');
    return s == std::string::npos ? "." : p.substr(0, s);
}

int main(int argc, char** argv) {
    cli::Args a(argc, argv);
    std::string input = a.str("input");
    std::string method = a.str_any({"partmethod", "partition"});
    long long key = a.num("partkey", -1), wid = a.num("workerid", -1), W = a.num("maxworker", -1);
    if (input.empty() || method.empty() || key <= 0 || wid < 0 || W <= 0 || wid >= W) {
        std::fprintf(stderr,
                     "usage: make_cpd_auto --input X.xy --partmethod {div|mod} --partkey K "
                     "--workerid I --maxworker W [--outdir D] [--device G] [--batch B] "
                     "[--threads T] [--plan P | --no-plan-cache]\n");
        return 2;
    }
    int mcode = cli::method_code(method);
    std::string outdir = a.str("outdir", dir_of(input));
    ::mkdir(outdir.c_str(), 0755);
    double t_start = now();
    try {
        cpd::io::XYGraph g = cpd::io::read_xy(input);
        uint64_t fp = cpd::io::graph_fingerprint(g.n, g.row_ptr.data(), g.dst.data(), g.w.data());
        double t_read = now() - t_start;

        // host preprocessing (column order + hierarchy), cached per graph
        char fph[32];
        std::snprintf(fph, sizeof fph, "%016llx", (unsigned long long)fp);
        std::string plan_path = a.str("plan", outdir + "/" + cpd::io::xy_stem(input) + "." + fph + ".plan");
        bool use_cache = !a.has("no-plan-cache");
        cpd_plan* plan = nullptr;
        double t0 = now();
        if (use_cache && cpd_plan_load(plan_path.c_str(), &plan) == CPD_OK) {
            std::printf("make_cpd_auto: loaded plan %s\n", plan_path.c_str());
        } else {
            cpd_plan_opts o{};
            o.threads = (int)a.num("threads", 0);
            o.verbose = a.has("verbose");
            cli::check(cpd_plan_create(g.row_ptr.data(), g.dst.data(), g.w.data(), g.n, g.m, &o, &plan),
                       "plan");
            if (use_cache) cli::check(cpd_plan_save(plan, plan_path.c_str()), "plan save");
        }
        double t_plan = now() - t0;
        cpd_plan_info info{};
        cli::check(cpd_plan_info_get(plan, &info), "plan info");
        std::vector<uint32_t> order(g.n);
        cli::check(cpd_plan_order(plan, order.data()), "order");

        // owned buckets
        uint32_t nb = 0;
        cli::check(cpd_partition_nbuckets(g.n, mcode, (uint32_t)key, &nb), "buckets");
        std::vector<uint32_t> owned;
        for (uint32_t b = 0; b < nb; ++b)
            if (b % (uint32_t)W == (uint32_t)wid) owned.push_back(b);
        uint32_t chunk = (uint32_t)(((uint64_t)g.n + key - 1) / key);
        auto bucket_nodes = [&](uint32_t b) {
            std::vector<uint32_t> v;
            if (mcode == CPD_PART_MOD) {
                for (uint64_t x = b; x < g.n; x += (uint64_t)key) v.push_back((uint32_t)x);
            } else {
                for (uint64_t x = (uint64_t)b * chunk; x < std::min<uint64_t>(g.n, (uint64_t)(b + 1) * chunk); ++x)
                    v.push_back((uint32_t)x);
            }
            return v;
        };

        int ndev = 0;
        cli::check(cpd_device_count(&ndev), "device count");
        if (ndev == 0) {
            std::fprintf(stderr, "make_cpd_auto: no GPU visible (this build has no CPU path)\n");
            return 1;
        }
        int device = (int)a.num("device", wid % ndev);
        cpd_graph* dg = nullptr;
        cli::check(cpd_graph_create(plan, device, &dg), "graph upload");
        cli::check(cpd_graph_set_batch(dg, (uint32_t)a.num("batch", 0)), "batch");
        uint32_t B = 0;
        cli::check(cpd_graph_get_batch(dg, &B), "batch");

        cpd::io::write_order(cpd::io::order_path(outdir, input), fp, order);

        double t_build = 0, t_io = 0;
        uint64_t rows_done = 0, runs_done = 0;
        cpd_rows* rows = nullptr;
        size_t i = 0;
        while (i < owned.size()) {
            // gather buckets until at least 4 sweeps' worth of rows
            std::vector<uint32_t> group, targets;
            std::vector<size_t> first;
            while (i < owned.size() && targets.size() < 4ull * B) {
                auto v = bucket_nodes(owned[i]);
                group.push_back(owned[i]);
                first.push_back(targets.size());
                targets.insert(targets.end(), v.begin(), v.end());
                ++i;
            }
            first.push_back(targets.size());
            double tb = now();
            cli::check(cpd_build_rows(dg, targets.data(), (uint32_t)targets.size(), rows, &rows), "build");
            uint32_t nr = 0;
            uint64_t tot = 0;
            cli::check(cpd_rows_count(rows, &nr, &tot), "rows");
            std::vector<uint64_t> off(nr + 1);
            std::vector<uint32_t> runs(tot);
            cli::check(cpd_rows_export(rows, off.data(), runs.data()), "export");
            t_build += now() - tb;
            double ti = now();
            for (size_t k = 0; k < group.size(); ++k) {
                CpdBucket b;
                b.n = g.n;
                b.bid = group[k];
                b.method = (uint32_t)mcode;
                b.key = (uint32_t)key;
                b.maxworker = (uint32_t)W;
                b.fingerprint = fp;
                b.targets.assign(targets.begin() + first[k], targets.begin() + first[k + 1]);
                uint64_t base = off[first[k]];
                for (size_t r = first[k]; r <= first[k + 1]; ++r) b.offsets.push_back(off[r] - base);
                b.runs.assign(runs.begin() + base, runs.begin() + off[first[k + 1]]);
                cpd::io::write_bucket(cpd::io::bucket_path(outdir, input, method, (uint32_t)key, group[k]), b);
            }
            t_io += now() - ti;
            rows_done += nr;
            runs_done += tot;
        }
        if (rows) cpd_rows_free(rows);
        cpd_graph_free(dg);
        cpd_plan_free(plan);
        double rate = t_build > 0 ? rows_done / t_build : 0.0;
        std::printf(
            "make_cpd_auto: worker %lld/%lld device %d: %llu rows in %zu buckets, %llu runs "
            "(%.1f per row); read %.3fs plan %.3fs (hierarchy %llu arcs, %u+%u levels) "
            "build %.3fs = %.1f rows/s, %.3f GTEPS; write %.3fs; total %.3fs\n",
            wid, W, device, (unsigned long long)rows_done, owned.size(),
            (unsigned long long)runs_done, rows_done ? (double)runs_done / rows_done : 0.0, t_read,
            t_plan, (unsigned long long)(info.ch_up_arcs + info.ch_dn_arcs), info.levels_up,
            info.levels_dn, t_build, rate, rate * g.m / 1e9, t_io, now() - t_start);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "make_cpd_auto: %s\n", e.what());
        return 1;
    }
    return 0;
}

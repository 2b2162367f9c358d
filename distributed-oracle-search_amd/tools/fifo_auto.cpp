// bin/fifo_auto — drop-in for warthog's resident query server with
// `--alg table-search` (make_fifos.py:20-21, README.md:107-111):
//
//   fifo_auto --input X.xy DIFF --partmethod {div|mod} --partkey K
//             --workerid I --maxworker W --outdir D --alg {table-search|cpd-search}
//             [--partition M] [--device G] [--fifo PATH] [--once]
//             [--index auto|rle|dense] [--read-threads T] [--parse-threads P]
//             [--verbose]  (per request on stderr: read+parse / prepare / compute)
//
// Creates its request FIFO, streams the CPD buckets this worker owns onto its
// GPU (as move tables at the graph's packed width when they are smaller
// than the runs, the runs then never held whole in HBM or host memory;
// compact-file pieces read by T threads, default 8), then serves requests on
// /tmp/worker{I}.fifo (process_query.py:86).  A request is what
// process_query.send_remote pipes in (process_query.py:66-79,89):
//     {worker JSON config}\n<query file> <answer fifo> <diff file>\n
// read until the writer closes.  The query file holds "{n}\n" + n "s t" lines
// (process_query.py:93-96).  The answer is ONE line of 10 comma-separated
// values on the answer FIFO (process_query.py:199-208):
//     n_expanded,n_inserted,n_touched,n_updated,n_surplus,plen,finished,
//     t_receive,t_astar,t_search
// For table-search: n_expanded = plen = moves walked, finished = queries that
// reached t, the A*-only fields 0.  For --alg cpd-search (cpd_query_search,
// driven by the request's hscale / fscale / time / itrs / k_moves, the
// library's workspace policy): the five search counters, plen of the paths
// found, finished.  Times in ns for both: t_receive = query file read and
// parse + upload and target sort on the GPU, t_search = the algorithm's
// device time (the walk kernel; the search passes + any table rebuild),
// t_astar = the search passes alone (0 for table-search).  With "debug":
// true in the config, per-query
// results are written to <query file>.res ("s t cost moves finished").
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <future>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "cli.hpp"
#include "cpd_io.hpp"

static double now() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

static volatile sig_atomic_t g_stop = 0;
static void on_signal(int) { g_stop = 1; }

// Value of a top-level key in the worker config (json.dumps output), as text.
static std::string json_field(const std::string& js, const std::string& key) {
    std::string pat = "\"" + key + "\"";
    size_t p = js.find(pat);
    if (p == std::string::npos) return "";
    p = js.find(':', p + pat.size());
    if (p == std::string::npos) return "";
    ++p;
    while (p < js.size() && js[p] == ' ') ++p;
    size_t e = p;
    while (e < js.size() && js[e] != ',' && js[e] != '}') ++e;
    std::string v = js.substr(p, e - p);
    while (!v.empty() && v.back() == ' ') v.pop_back();
    return v;
}

static std::string read_all(const std::string& path) {
    int fd = -1;
    while ((fd = ::open(path.c_str(), O_RDONLY)) < 0) {
        if (errno != EINTR || g_stop) return "";
    }
    std::string s;
    char buf[4096];
    for (;;) {
        ssize_t k = ::read(fd, buf, sizeof buf);
        if (k > 0) s.append(buf, (size_t)k);
        else if (k == 0) break;
        else if (errno != EINTR) break;
    }
    ::close(fd);
    return s;
}

static bool write_answer(const std::string& path, const std::string& line) {
    // process_query.send_remote mkfifo's the answer before writing the request
    // (process_query.py:72-73); tolerate a late mkfifo for up to 10 s
    for (int i = 0; i < 1000; ++i) {
        struct stat st;
        if (::stat(path.c_str(), &st) == 0) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    int fd = ::open(path.c_str(), O_WRONLY);
    if (fd < 0) return false;
    std::string out = line + "\n";
    const char* p = out.data();
    size_t left = out.size();
    while (left) {
        ssize_t k = ::write(fd, p, left);
        if (k < 0) {
            if (errno == EINTR) continue;
            ::close(fd);
            return false;
        }
        p += k;
        left -= (size_t)k;
    }
    ::close(fd);
    return true;
}

int main(int argc, char** argv) {
    cli::Args a(argc, argv);
    const auto& inputs = a.list("input");
    std::string method = a.str_any({"partmethod", "partition"});
    long long key = a.num("partkey", -1), wid = a.num("workerid", -1), W = a.num("maxworker", -1);
    std::string alg = a.str("alg", "table-search");
    if (inputs.empty() || method.empty() || key <= 0 || wid < 0 || W <= 0 || wid >= W) {
        std::fprintf(stderr,
                     "usage: fifo_auto --input X.xy [DIFF] --partmethod {div|mod} --partkey K "
                     "--workerid I --maxworker W --outdir D --alg table-search|cpd-search\n");
        return 2;
    }
    // table-search (make_fifos.py:20) or the CPD-heuristic search
    // (cpd_query_search; args.py:29-57)
    const bool search = alg == "cpd-search" || alg == "cpd_search";
    if (alg != "table-search" && !search) {
        std::fprintf(stderr, "fifo_auto: --alg must be table-search or cpd-search (got '%s')\n",
                     alg.c_str());
        return 2;
    }
    int mcode = cli::method_code(method);
    std::string xy = inputs[0];
    std::string outdir = a.str("outdir", ".");
    std::string fifo = a.str("fifo", "/tmp/worker" + std::to_string(wid) + ".fifo");
    bool once = a.has("once");
    // threads parsing a request's query file (a 1M-query file is ~14 MB)
    const int parse_threads = (int)a.num("parse-threads", 16);
    const bool verbose = a.has("verbose");
    signal(SIGINT, on_signal);
    signal(SIGTERM, on_signal);
    signal(SIGPIPE, SIG_IGN);

    // The request FIFO exists before the (possibly long) index load: a request
    // sent meanwhile blocks in its writer's open() until the loop below reads
    // it, instead of `cat <<CONF > fifo` creating a regular file there.  A
    // non-FIFO left at the path (such a file from an earlier run) is replaced.
    {
        struct stat st;
        if (::lstat(fifo.c_str(), &st) == 0 && !S_ISFIFO(st.st_mode)) ::unlink(fifo.c_str());
        if (::mkfifo(fifo.c_str(), 0666) != 0 && errno != EEXIST) {
            std::fprintf(stderr, "fifo_auto: mkfifo %s: %s\n", fifo.c_str(), std::strerror(errno));
            return 1;
        }
        if (::lstat(fifo.c_str(), &st) != 0 || !S_ISFIFO(st.st_mode)) {
            std::fprintf(stderr, "fifo_auto: %s is not a FIFO\n", fifo.c_str());
            return 1;
        }
    }

    cpd_index* ix = nullptr;
    cpd_graph* dg = nullptr;
    cpd_plan* plan = nullptr;
    cpd::io::XYGraph g;
    std::map<std::string, std::vector<uint32_t>> diff_cache;
    std::string active_diff = "-";
    int device = -1;
    bool arena = false;
    try {
        double t0 = now();
        // This worker's buckets, headers first (targets, run counts or
        // offsets): DOSCPD02/03 (compact move tables, what make_cpd_auto
        // writes by default) or DOSCPD01 (run words).  The node count comes
        // from the order file make_cpd_auto wrote beside them; the graph's
        // fingerprint is checked once the .xy is read.
        const uint32_t n0 = cpd::io::read_order_n(cpd::io::order_path(outdir, xy));
        uint32_t nb = 0;
        cli::check(cpd_partition_nbuckets(n0, mcode, (uint32_t)key, &nb), "buckets");
        std::vector<std::string> paths;
        std::vector<int> formats;
        std::vector<cpd::io::CpdBucket> heads;
        std::vector<cpd::io::MoveBucket> mheads;
        std::vector<uint32_t> targets;
        uint64_t total_runs = 0, compact_bytes = 0;
        uint32_t move_bits = 0;  // the compact rows' width (0: some bucket holds run words)
        bool all_compact = true;
        for (uint32_t b = 0; b < nb; ++b) {
            if (b % (uint32_t)W != (uint32_t)wid) continue;
            paths.push_back(cpd::io::bucket_path(outdir, xy, method, (uint32_t)key, b));
            formats.push_back(cpd::io::bucket_format(paths.back()));
            if (formats.back() == 1) {
                heads.push_back(cpd::io::read_bucket_head(paths.back()));
                mheads.emplace_back();
                const auto& bk = heads.back();
                targets.insert(targets.end(), bk.targets.begin(), bk.targets.end());
                total_runs += bk.offsets.back();
                all_compact = false;
            } else {
                mheads.push_back(cpd::io::read_move_bucket_head(paths.back()));
                heads.emplace_back();
                const auto& bk = mheads.back();
                if (bk.n != n0) throw std::runtime_error("bucket " + std::to_string(b) + " has another node count");
                targets.insert(targets.end(), bk.targets.begin(), bk.targets.end());
                total_runs += bk.total_runs;
                compact_bytes += 4ull * bk.words * bk.targets.size();
                move_bits = bk.bits;
            }
        }
        // The device side starts now, on a thread, beside the host reads
        // (VERDICT r04 item 7): the first HIP call and, for compact buckets,
        // the dense index's HBM committed as an arena (nrows x n padded to
        // 2048 columns x bits / 8 bytes: committing fresh HBM costs about a
        // second per 30 GB) that cpd_index_create_empty then carves.
        int ndev = 0;
        double t_dev = 0.0;
        int dev_rc = CPD_OK;
        std::string dev_err;
        std::thread dev_thr([&] {
            const double td = now();
            dev_rc = cpd_device_count(&ndev);
            if (dev_rc == CPD_OK && ndev > 0) {
                device = (int)a.num("device", wid % ndev);
                if (all_compact && !targets.empty() && move_bits) {
                    const uint64_t npad = (n0 + 2047ull) / 2048ull * 2048ull;
                    const uint64_t bytes = (uint64_t)targets.size() * (npad * move_bits / 32ull) * 4ull;
                    // only for an index that will be dense (--index rle keeps
                    // runs; auto takes tables when the runs weigh more — the
                    // index's own test): an unused arena would hold HBM the
                    // search workspace is sized from
                    const std::string im0 = a.str("index", "auto");
                    const bool dense = im0 == "dense" || (im0 != "rle" && 4ull * total_runs > bytes);
                    if (dense) arena = cpd_device_arena(device, bytes + (1ull << 20), 0) == CPD_OK;
                }
            }
            if (dev_rc != CPD_OK) dev_err = cpd_last_error();
            t_dev = now() - td;
        });
        struct Join {
            std::thread& t;
            ~Join() {
                if (t.joinable()) t.join();
            }
        } join{dev_thr};
        g = cpd::io::read_xy(xy);
        uint64_t fp = cpd::io::graph_fingerprint(g.n, g.row_ptr.data(), g.dst.data(), g.w.data());
        if (inputs.size() > 1) diff_cache[inputs[1]] = cpd::io::read_diff(inputs[1], g);
        cpd_plan_opts o{};
        o.no_hierarchy = 1;  // queries need the CSR + column order only
        cli::check(cpd_plan_create(g.row_ptr.data(), g.dst.data(), g.w.data(), g.n, g.m, &o, &plan),
                   "plan");
        std::vector<uint32_t> order(g.n);
        cli::check(cpd_plan_order(plan, order.data()), "order");
        std::vector<uint32_t> stored = cpd::io::read_order(cpd::io::order_path(outdir, xy), fp);
        if (stored != order) throw std::runtime_error("stored column order differs from this build's");
        for (size_t k = 0; k < paths.size(); ++k) {
            const bool rle = formats[k] == 1;
            const uint64_t bfp = rle ? heads[k].fingerprint : mheads[k].fingerprint;
            const uint32_t bkey = rle ? heads[k].key : mheads[k].key;
            const uint32_t bmethod = rle ? heads[k].method : mheads[k].method;
            if (bfp != fp || bkey != (uint32_t)key || bmethod != (uint32_t)mcode)
                throw std::runtime_error(paths[k] + " was built for another graph/partition");
        }
        const double t_graph0 = now();
        dev_thr.join();
        const double t_devwait = now() - t_graph0;
        if (dev_rc != CPD_OK) throw std::runtime_error("device: " + dev_err);
        if (ndev == 0) throw std::runtime_error("no GPU visible (this build has no CPU path)");
        cli::check(cpd_graph_create(plan, device, &dg), "graph upload");
        // then the rows, streamed in pieces of <= kPiece words (a longer row
        // alone): a dense index never holds the worker's runs in HBM or RAM
        const std::string im = a.str("index", "auto");
        const int imode = im == "rle" ? CPD_INDEX_RLE : im == "dense" ? CPD_INDEX_DENSE : CPD_INDEX_AUTO;
        cli::check(cpd_index_create_empty(dg, targets.data(), (uint32_t)targets.size(), imode,
                                          total_runs, &ix),
                   "index");
        const double t_rows0 = now();
        constexpr uint64_t kPiece = 64ull << 20;  // 256 MB
        std::vector<uint32_t> buf;
        std::vector<uint64_t> rel;
        // compact buckets: pieces read into two page-locked buffers by a
        // reader thread while the previous piece is appended (uploaded)
        uint32_t* pin[2] = {nullptr, nullptr};
        uint64_t pin_bytes = 0;
        const int read_threads = (int)a.num("read-threads", 8);
        for (size_t k = 0; k < paths.size(); ++k) {
            if (formats[k] == 2) {
                const auto& mh = mheads[k];
                const uint32_t nr = (uint32_t)mh.targets.size();
                if (!nr) continue;
                const uint32_t per = (uint32_t)std::min<uint64_t>(nr, std::max<uint64_t>(1, kPiece / mh.words));
                if (4ull * mh.words * per > pin_bytes) {  // grown for this bucket's pieces
                    for (auto& p : pin) {
                        cpd_host_free(p);
                        void* q = nullptr;
                        cli::check(cpd_host_alloc(4ull * mh.words * per, &q), "pinned buffer");
                        p = static_cast<uint32_t*>(q);
                    }
                    pin_bytes = 4ull * mh.words * per;
                }
                auto read = [&, k, per, nr](uint32_t r0, int slot) {
                    cpd::io::read_move_bucket_rows(paths[k], mheads[k], r0, std::min(per, nr - r0), pin[slot],
                                                   read_threads);
                };
                std::future<void> rd = std::async(std::launch::async, read, 0u, 0);
                for (uint32_t r0 = 0, i = 0; r0 < nr; r0 += per, ++i) {
                    rd.get();  // piece i is in pin[i & 1] (a read error is rethrown here)
                    if (r0 + per < nr) rd = std::async(std::launch::async, read, r0 + per, (int)((i + 1) & 1u));
                    const int rc = cpd_index_append_moves(ix, std::min(per, nr - r0), mh.bits, pin[i & 1u]);
                    if (rc != CPD_OK) {
                        if (rd.valid()) rd.wait();
                        cli::check(rc, "index rows");
                    }
                }
                continue;
            }
            const auto& off = heads[k].offsets;
            const uint32_t nr = (uint32_t)heads[k].targets.size();
            for (uint32_t r0 = 0; r0 < nr;) {
                uint32_t r1 = r0 + 1;
                while (r1 < nr && off[r1 + 1] - off[r0] <= kPiece) ++r1;
                buf.resize(off[r1] - off[r0]);
                cpd::io::read_bucket_runs(paths[k], heads[k], off[r0], buf.size(), buf.data());
                rel.resize(r1 - r0 + 1);
                for (uint32_t i = r0; i <= r1; ++i) rel[i - r0] = off[i] - off[r0];
                cli::check(cpd_index_append_rows(ix, r1 - r0, rel.data(), buf.data()), "index rows");
                r0 = r1;
            }
        }
        for (auto p : pin) cpd_host_free(p);
        const double t_rows = now() - t_rows0;
        int mode = 0;
        cli::check(cpd_index_get_mode(ix, &mode), "index mode");
        // one machine-readable line (bench.py's full-build leg reads it)
        std::printf("fifo_auto-json: {\"worker\": %lld, \"rows\": %zu, \"runs\": %llu, "
                    "\"index\": \"%s\", \"compact_bytes\": %llu, \"read_plan_s\": %.3f, "
                    "\"device_s\": %.3f, \"device_wait_s\": %.3f, \"arena\": %s, "
                    "\"graph_s\": %.3f, \"rows_s\": %.3f, \"ready_s\": %.3f}\n",
                    wid, targets.size(), (unsigned long long)total_runs,
                    mode == CPD_INDEX_DENSE ? "dense" : "rle", (unsigned long long)compact_bytes,
                    t_graph0 - t0, t_dev, t_devwait, arena ? "true" : "false",
                    t_rows0 - t_graph0, t_rows, now() - t0);
        std::printf("fifo_auto: worker %lld: %zu rows, %llu runs (%s index) on device %d, ready in "
                    "%.3fs; listening on %s\n",
                    wid, targets.size(), (unsigned long long)total_runs,
                    mode == CPD_INDEX_DENSE ? "dense" : "rle", device, now() - t0, fifo.c_str());
        std::fflush(stdout);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "fifo_auto: %s\n", e.what());
        ::unlink(fifo.c_str());
        return 1;
    }

    while (!g_stop) {
        std::string msg = read_all(fifo);
        if (g_stop) break;
        if (msg.empty()) continue;
        size_t nl = msg.find('\n');
        std::string conf = msg.substr(0, nl);
        if (conf == "quit" || conf == "exit") break;
        std::string rest = nl == std::string::npos ? "" : msg.substr(nl + 1);
        char qfile[4096] = {0}, answer[4096] = {0}, dname[4096] = {0};
        int got = std::sscanf(rest.c_str(), "%4095s %4095s %4095s", qfile, answer, dname);
        if (got < 2) {
            std::fprintf(stderr, "fifo_auto: malformed request: %s\n", msg.c_str());
            continue;
        }
        std::string diff = got >= 3 ? dname : "-";
        int k_moves = -1;
        std::string km = json_field(conf, "k_moves");
        if (!km.empty()) k_moves = std::atoi(km.c_str());
        bool debug = json_field(conf, "debug") == "true";
        // cpd-search knobs (process_query.py:149-160): hscale, fscale, time
        // (ns; args.get_time_ns may send a float), itrs; wall-clock time
        // limit; the workspace (first-pass columns per lane, escalation,
        // share of HBM) is the library's policy (capacity 0), the one the
        // bench measures
        cpd_search_opts so{1.0, 0.0, k_moves, -1, 0, 0, 0, CPD_SEARCH_AUTO, 0.0, 0};
        if (!json_field(conf, "hscale").empty()) so.hscale = std::atof(json_field(conf, "hscale").c_str());
        if (!json_field(conf, "fscale").empty()) so.fscale = std::atof(json_field(conf, "fscale").c_str());
        if (!json_field(conf, "itrs").empty()) so.itrs = std::atoll(json_field(conf, "itrs").c_str());
        if (!json_field(conf, "time").empty()) {
            const double tn = std::atof(json_field(conf, "time").c_str());
            so.time_ns = tn > 0 ? (uint64_t)tn : 0;
        }
        std::string line = "0,0,0,0,0,0,0,0,0,0";
        try {
            double t0 = now();
            // kept across requests: their pages stay mapped
            static std::vector<uint32_t> s, t;
            cpd::io::read_query_file(qfile, parse_threads, s, t);
            const double t_read = now() - t0;
            if (diff != active_diff) {
                if (diff == "-" ) {
                    cli::check(cpd_index_set_weights(ix, nullptr), "weights");
                } else {
                    auto it = diff_cache.find(diff);
                    if (it == diff_cache.end())
                        it = diff_cache.emplace(diff, cpd::io::read_diff(diff, g)).first;
                    cli::check(cpd_index_set_weights(ix, it->second.data()), "weights");
                }
                active_diff = diff;
            }
            const size_t nq = s.size();
            int rc = cpd_query_prepare(ix, s.data(), t.data(), (uint32_t)nq);
            if (rc != CPD_OK) throw std::runtime_error(cpd_last_error());
            double t_receive = now() - t0;
            cpd_query_stats st{};
            cpd_search_stats ss{};
            if (search) {
                rc = cpd_query_search(ix, &so, &ss);
                if (rc != CPD_OK) throw std::runtime_error(cpd_last_error());
                if (ss.overflow)
                    std::fprintf(stderr, "fifo_auto: %llu searches exceeded the workspace and stopped unfinished\n",
                                 (unsigned long long)ss.overflow);
            } else {
                rc = cpd_query_run(ix, k_moves, &st);
                if (rc != CPD_OK) throw std::runtime_error(cpd_last_error());
            }
            if (debug) {
                std::vector<uint64_t> cost(nq);
                std::vector<uint32_t> hops(nq);
                std::vector<uint8_t> fin(nq);
                cli::check(cpd_query_fetch(ix, cost.data(), hops.data(), fin.data()), "fetch");
                std::string res = std::string(qfile) + ".res";
                if (std::FILE* f = std::fopen(res.c_str(), "w")) {
                    for (size_t i = 0; i < nq; ++i)
                        std::fprintf(f, "%u %u %llu %u %u\n", s[i], t[i], (unsigned long long)cost[i],
                                     hops[i], fin[i] == 1 ? 1u : 0u);
                    std::fclose(f);
                }
            }
            // t_receive = query file read + parse + upload and sort on the
            // GPU; t_search = the algorithm's device time (table-search: the
            // walk kernel; cpd-search: the search passes + any table rebuild
            // for new weights), the same meaning for both; t_astar = the A*
            // passes alone (0 for table-search)
            char buf[512];
            if (search)
                std::snprintf(buf, sizeof buf, "%llu,%llu,%llu,%llu,%llu,%llu,%llu,%lld,%lld,%lld",
                              (unsigned long long)ss.expanded, (unsigned long long)ss.inserted,
                              (unsigned long long)ss.touched, (unsigned long long)ss.updated,
                              (unsigned long long)ss.surplus, (unsigned long long)ss.plen,
                              (unsigned long long)ss.finished, (long long)(t_receive * 1e9),
                              (long long)(ss.kernel_ms * 1e6),
                              (long long)((ss.kernel_ms + ss.tables_ms) * 1e6));
            else
                std::snprintf(buf, sizeof buf, "%llu,0,0,0,0,%llu,%llu,%lld,0,%lld",
                              (unsigned long long)st.hops, (unsigned long long)st.hops,
                              (unsigned long long)st.finished, (long long)(t_receive * 1e9),
                              (long long)(st.kernel_ms * 1e6));
            line = buf;
            if (verbose)  // the receive phase split (stderr: nothing reads stdout by then)
                std::fprintf(stderr, "fifo_auto-req: {\"queries\": %zu, \"read_parse_s\": %.6f, "
                             "\"prepare_s\": %.6f, \"compute_s\": %.6f}\n", nq, t_read,
                             t_receive - t_read, search ? ss.kernel_ms * 1e-3 : st.kernel_ms * 1e-3);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "fifo_auto: request failed: %s\n", e.what());
        }
        if (!write_answer(answer, line))
            std::fprintf(stderr, "fifo_auto: cannot write answer to %s\n", answer);
        if (once) break;
    }
    cpd_index_free(ix);
    cpd_graph_free(dg);
    cpd_plan_free(plan);
    if (arena) cpd_device_arena_release(device);
    return 0;
}

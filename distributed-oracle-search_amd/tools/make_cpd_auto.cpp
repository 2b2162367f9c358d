// bin/make_cpd_auto — drop-in for warthog's make_cpd_auto (README.md:82-95),
// launched per worker by make_cpds.py:20-21:
//
//   make_cpd_auto --input X.xy --partmethod {div|mod} --partkey K
//                 --workerid I --maxworker W --outdir D
//                 [--partition M]      README.md:89 spelling of --partmethod
//                 [--device G]         default: I % (visible GPUs)
//                 [--batch B]          rows per GPU sweep (multiple of 1024);
//                                      0 (default) = what fits in HBM, at most
//                                      2048 rows when files are written (the
//                                      disk bounds the worker) and
//                                      28672 with --discard (CPD_BATCH_MAX
//                                      overrides), with or without the arena
//                 [--no-arena]         allocate the batch buffers at graph setup
//                                      instead of committing them on a host
//                                      thread beside the plan (default)
//                 [--arena-touch]      also write the arena once while committing
//                 [--threads T]        host threads for the hierarchy build (--ch-host)
//                 [--ch-host]          contract the hierarchy on host threads, not the GPU
//                 [--plan P | --no-plan-cache]
//                 [--write-threads T]  host threads copying + writing rows (16)
//                 [--no-pipeline]      build, then export, then write, per group
//                 [--plan-only]        build / load the cached plan and exit
//                 [--targets-from S]   only rows of targets of scenario S (q s t)
//                 [--format moves|rle] bucket file layout: moves (default) =
//                                      the rows as move tables of 1/2/4 bits
//                                      per column (by max out-degree, n*bits/8
//                                      bytes per row); rle = DOSCPD01, the run
//                                      words (4 B per run)
//                 [--stripes K]        moves: the rows striped over K part
//                                      files per bucket (DOSCPD03, default 16:
//                                      writes to one file serialise on its
//                                      inode); 1 = one DOSCPD02 file
//                 [--discard]          null sink: every row is still built and
//                                      copied out of HBM (D2H), but no file is
//                                      written (times the build + export path
//                                      without the disk)
//
// The plan (column order + hierarchy) is cached in D per graph; workers that
// start together share it through cpd_plan_cache (one builds, the rest wait).
//
// Builds the CPD rows of every target this worker owns under the
// distribution_controller partition, on the GPU, and writes one file per
// owned bucket into D (README.md:92-93 "one or more CPDs ... auto-generated
// names").  The launcher is fire-and-forget (tmux, make_cpds.py:21), so timing
// is printed here.
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
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

static void ok(int rc, const char* what) {
    if (rc != CPD_OK)
        throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " + cpd_last_error());
}

// Overlapped bucket writer ("overlap D2H of RLE rows with
// the next batch's SSSP, plus parallel bucket-file writes").  Rows are built
// one sweep batch (B rows) per block, in bucket order, alternating between two
// cpd_rows.  While the GPU builds block k+1, a pool of host threads copies
// block k out of HBM in pieces (cpd_rows_export_range: each thread on its own
// stream) and writes each piece straight to its final position in its bucket
// file (BucketFile), so no bucket is ever held whole in host memory.  A
// bucket's .tmp is renamed once its last block is written.  The files are
// byte-identical to the sequential path (--no-pipeline).
// Destinations of the D2H copies: page-locked (cpd_host_alloc), one per
// writer thread, grown on demand.
struct PinnedBuf {
    uint32_t* p = nullptr;
    uint64_t cap = 0;
    uint32_t* get(uint64_t n) {
        if (n > cap) {
            cpd_host_free(p);
            p = nullptr;
            cap = 0;
            void* q = nullptr;
            ok(cpd_host_alloc(std::max<uint64_t>(n, 1) * sizeof(uint32_t), &q), "pinned buffer");
            p = static_cast<uint32_t*>(q);
            cap = n;
        }
        return p;
    }
    ~PinnedBuf() { cpd_host_free(p); }
};

class Pipeline {
public:
    Pipeline(cpd_graph* g, uint32_t B, int threads, bool discard, bool moves, uint32_t stripes)
        : g_(g), B_(B), discard_(discard), moves_(moves), stripes_(stripes) {
        for (int i = 0; i < std::max(1, threads); ++i) pool_.emplace_back([this] { worker(); });
    }
    ~Pipeline() {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : pool_) t.join();
        for (cpd_rows* r : rows_)
            if (r) cpd_rows_free(r);
    }

    void run(const std::vector<uint32_t>& targets, const std::vector<uint64_t>& first,
             const std::vector<CpdBucket>& heads, const std::vector<std::string>& paths) {
        using cpd::io::BucketFile;
        using cpd::io::MoveBucketFile;
        const size_t N = targets.size(), nb = heads.size();
        std::vector<std::unique_ptr<BucketFile>> files(nb);
        std::vector<std::unique_ptr<MoveBucketFile>> mfiles(nb);
        std::vector<uint64_t> bruns(nb, 0);  // runs of the bucket's rows scheduled so far
        std::vector<size_t> to_close;        // buckets finished by the block in flight
        auto open_bucket = [&](size_t k) {
            if (discard_) return;
            if (moves_)
                mfiles[k] = std::make_unique<MoveBucketFile>(paths[k], move_head(heads[k]), stripes_);
            else files[k] = std::make_unique<BucketFile>(paths[k], heads[k]);
        };
        auto close_bucket = [&](size_t k) {
            if (files[k]) files[k]->close(bruns[k]);
            if (mfiles[k]) mfiles[k]->close(bruns[k]);
            files[k].reset();
            mfiles[k].reset();
        };
        for (size_t k = 0; k < nb; ++k)
            if (first[k] == first[k + 1] && !discard_) {  // empty bucket: header (+ one offset)
                open_bucket(k);
                if (files[k]) {
                    const uint64_t zero = 0;
                    files[k]->write_offsets(0, &zero, 1);
                }
                close_bucket(k);
            }
        uint32_t words = 0;  // compact row width
        size_t kb = 0;
        for (size_t b0 = 0, blk = 0; b0 < N; b0 += B_, ++blk) {
            const uint32_t cnt = (uint32_t)std::min<size_t>(B_, N - b0);
            cpd_rows*& r = rows_[blk & 1];
            const double tb = now();
            if (b0 + cnt < N)  // the next block's up-sweep starts beside this block's first moves
                ok(cpd_graph_hint_next(g_, targets.data() + b0 + cnt,
                                       (uint32_t)std::min<size_t>(B_, N - b0 - cnt)),
                   "hint");
            ok(cpd_build_rows(g_, targets.data() + b0, cnt, r, &r), "build");
            t_build += now() - tb;
            auto offs = std::make_shared<std::vector<uint64_t>>(cnt + 1);
            ok(cpd_rows_export_range(r, 0, cnt, offs->data(), nullptr), "export offsets");
            if (!words) ok(cpd_rows_move_words(r, &words), "move words");
            // block k-1 written (it read the other cpd_rows): close what it finished
            const double tw = now();
            drain();
            t_wait += now() - tw;
            for (size_t k : to_close) close_bucket(k);
            to_close.clear();
            cpd_rows* rr = r;
            for (size_t i = b0; i < b0 + cnt;) {
                while (first[kb + 1] <= i) ++kb;
                if (!files[kb] && !mfiles[kb]) open_bucket(kb);
                const size_t seg_end = std::min<size_t>(first[kb + 1], b0 + cnt);
                const uint32_t r0 = (uint32_t)(i - b0), r1 = (uint32_t)(seg_end - b0);
                const uint32_t brow0 = (uint32_t)(i - first[kb]);
                const uint64_t base = bruns[kb];
                const bool last = seg_end == first[kb + 1];
                if (moves_)
                    schedule_moves(rr, mfiles[kb].get(), offs, r0, r1, brow0, words);
                else
                    schedule_runs(rr, files[kb].get(), offs, r0, r1, brow0, base, last);
                bruns[kb] += (*offs)[r1] - (*offs)[r0];
                if (last) to_close.push_back(kb);
                i = seg_end;
            }
            runs += offs->back();
        }
        const double tw = now();
        drain();
        t_wait += now() - tw;
        for (size_t k : to_close) close_bucket(k);
    }

    double t_build = 0, t_wait = 0;
    uint64_t runs = 0;
    // D2H copies: summed copy time over writer threads, bytes, first start /
    // last end (their wall span); file writes: summed time over threads
    double x_sum = 0, x_first = 0, x_last = 0, w_sum = 0;
    uint64_t x_bytes = 0;

private:
    cpd::io::MoveBucket move_head(const CpdBucket& h) const {
        cpd::io::MoveBucket m;
        m.n = h.n;
        m.bid = h.bid;
        m.method = h.method;
        m.key = h.key;
        m.maxworker = h.maxworker;
        uint32_t bits = 4;
        ok(cpd_graph_move_bits(g_, &bits), "move bits");
        m.bits = bits;
        m.words = (uint32_t)(((uint64_t)h.n * bits + 31u) / 32u);
        m.fingerprint = h.fingerprint;
        m.targets = h.targets;
        return m;
    }

    // DOSCPD01: bucket-relative offsets (the end offset with the last rows),
    // then the run words in pieces of <= kPieceRuns
    void schedule_runs(cpd_rows* rr, cpd::io::BucketFile* f,
                       const std::shared_ptr<std::vector<uint64_t>>& offs, uint32_t r0, uint32_t r1,
                       uint32_t brow0, uint64_t base, bool last) {
        if (f) submit([=] {
            std::vector<uint64_t> o;
            for (uint32_t u = r0; u < r1 + (last ? 1u : 0u); ++u)
                o.push_back(base + (*offs)[u] - (*offs)[r0]);
            f->write_offsets(brow0, o.data(), (uint32_t)o.size());
        });
        for (uint32_t p0 = r0; p0 < r1;) {
            uint32_t p1 = p0 + 1;
            while (p1 < r1 && (*offs)[p1 + 1] - (*offs)[p0] <= kPieceRuns) ++p1;
            const uint64_t run0 = base + (*offs)[p0] - (*offs)[r0];
            submit([=] {
                thread_local PinnedBuf buf;
                const uint64_t nr = (*offs)[p1] - (*offs)[p0];
                uint32_t* dst = buf.get(nr);
                const double te = now();
                ok(cpd_rows_export_range(rr, p0, p1 - p0, nullptr, dst), "export");
                const double tx = now();
                note_export(te, tx, nr * sizeof(uint32_t));
                if (f) {
                    f->write_runs(run0, dst, nr);
                    note_write(now() - tx);
                }
            });
            p0 = p1;
        }
    }

    // DOSCPD02: the rows' run counts, then the move tables in pieces of
    // <= kPieceRuns words
    void schedule_moves(cpd_rows* rr, cpd::io::MoveBucketFile* f,
                        const std::shared_ptr<std::vector<uint64_t>>& offs, uint32_t r0,
                        uint32_t r1, uint32_t brow0, uint32_t words) {
        if (f) submit([=] {
            std::vector<uint32_t> c(r1 - r0);
            for (uint32_t u = r0; u < r1; ++u) c[u - r0] = (uint32_t)((*offs)[u + 1] - (*offs)[u]);
            f->write_counts(brow0, c.data(), r1 - r0);
        });
        // pieces of <= kPieceRuns words, and at least one per writer thread
        // in a block so the whole pool copies and writes it
        const uint64_t fair = (B_ + pool_.size() - 1) / pool_.size();
        const uint32_t per = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kPieceRuns / words, fair));
        for (uint32_t p0 = r0; p0 < r1; p0 += per) {
            const uint32_t p1 = std::min(r1, p0 + per);
            submit([=] {
                thread_local PinnedBuf buf;
                const uint64_t nw = (uint64_t)words * (p1 - p0);
                uint32_t* dst = buf.get(nw);
                const double te = now();
                ok(cpd_rows_export_moves(rr, p0, p1 - p0, dst), "export moves");
                const double tx = now();
                note_export(te, tx, nw * sizeof(uint32_t));
                if (f) {
                    f->write_rows(brow0 + (p0 - r0), dst, p1 - p0);
                    note_write(now() - tx);
                }
            });
        }
    }

    void note_export(double t0, double t1, uint64_t bytes) {
        std::lock_guard<std::mutex> l(xmu_);
        x_sum += t1 - t0;
        x_bytes += bytes;
        if (x_first == 0 || t0 < x_first) x_first = t0;
        x_last = std::max(x_last, t1);
    }
    void note_write(double dt) {
        std::lock_guard<std::mutex> l(xmu_);
        w_sum += dt;
    }
    std::mutex xmu_;

    static constexpr uint64_t kPieceRuns = 64ull << 20;  // 256 MB of runs / words per copy+write

    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> l(mu_);
            q_.push_back(std::move(f));
            ++pending_;
        }
        cv_.notify_one();
    }
    void drain() {  // wait for every submitted job; rethrow the first failure
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [this] { return pending_ == 0; });
        if (err_) std::rethrow_exception(err_);
    }
    void worker() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            std::exception_ptr e;
            try {
                f();
            } catch (...) {
                e = std::current_exception();
            }
            std::lock_guard<std::mutex> l(mu_);
            if (e && !err_) err_ = e;
            if (--pending_ == 0) done_.notify_all();
        }
    }

    cpd_graph* g_;
    uint32_t B_;
    bool discard_, moves_;
    uint32_t stripes_;
    cpd_rows* rows_[2] = {nullptr, nullptr};
    std::vector<std::thread> pool_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::deque<std::function<void()>> q_;
    size_t pending_ = 0;
    bool stop_ = false;
    std::exception_ptr err_;
};

int main(int argc, char** argv) {
    cli::Args a(argc, argv);
    std::string input = a.str("input");
    std::string method = a.str_any({"partmethod", "partition"});
    long long key = a.num("partkey", -1), wid = a.num("workerid", -1), W = a.num("maxworker", -1);
    if (input.empty() || method.empty() || key <= 0 || wid < 0 || W <= 0 || wid >= W) {
        std::fprintf(stderr,
                     "usage: make_cpd_auto --input X.xy --partmethod {div|mod} --partkey K "
                     "--workerid I --maxworker W [--outdir D] [--device G] [--batch B] "
                     "[--threads T] [--plan P | --no-plan-cache] [--write-threads T] "
                     "[--no-pipeline] [--plan-only] [--targets-from SCEN] [--discard] "
                     "[--hbm-reserve GIB] [--format moves|rle] [--stripes K]\n");
        return 2;
    }
    int mcode = cli::method_code(method);
    const std::string format = a.str("format", "moves");
    if (format != "moves" && format != "rle") {
        std::fprintf(stderr, "make_cpd_auto: --format must be moves or rle\n");
        return 2;
    }
    const bool moves = format == "moves";
    // compact buckets striped over part files (DOSCPD03; 1 = one DOSCPD02 file)
    const long long stripes_arg = a.num("stripes", 16);
    if (stripes_arg < 1 || stripes_arg > 4096) {  // what the reader accepts
        std::fprintf(stderr, "make_cpd_auto: --stripes must be in [1, 4096]\n");
        return 2;
    }
    const uint32_t stripes = (uint32_t)stripes_arg;
    // the automatic batch's cap, the same with or without the arena: writing
    // files, the sink bounds the worker (the GPU builds rows ~30x faster than
    // a disk takes them), so a batch past 2048 rows only adds HBM
    // to commit beside the plan; --discard keeps the build-bound cap
    const uint32_t batch_cap = [&] {
        const char* bm = std::getenv("CPD_BATCH_MAX");
        const double dflt = a.has("discard") ? 28.0 : 2.0;
        const double k = bm && *bm ? std::max(1.0, std::min(32.0, std::floor(std::atof(bm) / 1024))) : dflt;
        return (uint32_t)k * 1024u;
    }();
    std::string outdir = a.str("outdir", dir_of(input));
    ::mkdir(outdir.c_str(), 0755);
    double t_start = now();
    try {
        cpd::io::XYGraph g = cpd::io::read_xy(input);
        uint64_t fp = cpd::io::graph_fingerprint(g.n, g.row_ptr.data(), g.dst.data(), g.w.data());
        double t_read = now() - t_start;

        // owned buckets
        uint32_t nb = 0;
        cli::check(cpd_partition_nbuckets(g.n, mcode, (uint32_t)key, &nb), "buckets");
        std::vector<uint32_t> owned;
        for (uint32_t b = 0; b < nb; ++b)
            if (b % (uint32_t)W == (uint32_t)wid) owned.push_back(b);
        uint32_t chunk = (uint32_t)(((uint64_t)g.n + key - 1) / key);
        // --targets-from SCEN: only the rows some query of the scenario needs
        // (its "q s t" targets; process_query.py:56-57 routes by t), so a
        // partial CPD for a known workload stays small on disk
        std::vector<char> wanted;
        if (a.has("targets-from")) {
            wanted.assign(g.n, 0);
            for (const auto& q : cpd::io::read_scen(a.str("targets-from"))) {
                if (q.second >= g.n) throw std::runtime_error("scenario target out of range");
                wanted[q.second] = 1;
            }
        }
        auto bucket_nodes = [&](uint32_t b) {
            std::vector<uint32_t> v;
            auto keep = [&](uint64_t x) {
                if (wanted.empty() || wanted[x]) v.push_back((uint32_t)x);
            };
            if (mcode == CPD_PART_MOD) {
                for (uint64_t x = b; x < g.n; x += (uint64_t)key) keep(x);
            } else {
                for (uint64_t x = (uint64_t)b * chunk; x < std::min<uint64_t>(g.n, (uint64_t)(b + 1) * chunk); ++x)
                    keep(x);
            }
            return v;
        };

        // Disk preflight: every owned row's bucket files must fit --outdir
        // before the plan and the GPU work start (eight `div 8` workers of the
        // 1M graph write 250 GB at once; a full disk would otherwise surface
        // as a write error minutes in).  The rle layout's size depends on the
        // runs, unknown before the build: not checked.
        if (moves && !a.has("discard") && !a.has("plan-only")) {
            uint64_t nrows = 0;
            for (uint32_t b : owned) nrows += bucket_nodes(b).size();
            uint32_t maxdeg = 1;
            for (uint32_t v = 0; v < g.n; ++v) maxdeg = std::max(maxdeg, g.row_ptr[v + 1] - g.row_ptr[v]);
            const uint32_t bits = maxdeg <= 2 ? 1u : maxdeg <= 4 ? 2u : 4u;
            uint64_t need = 0, have = 0;
            cli::check(cpd_bucket_bytes(g.n, bits, nrows, (uint32_t)owned.size(), stripes, &need),
                       "bucket bytes");
            if (cpd_space_check(outdir.c_str(), need, &have) != CPD_OK) {
                std::fprintf(stderr, "make_cpd_auto: %s\n", cpd_last_error());
                return 3;
            }
        }

        // host preprocessing (column order + hierarchy), cached per graph
        char fph[32];
        std::snprintf(fph, sizeof fph, "%016llx", (unsigned long long)fp);
        std::string plan_path = a.str("plan", outdir + "/" + cpd::io::xy_stem(input) + "." + fph + ".plan");
        bool use_cache = !a.has("no-plan-cache");
        cpd_plan* plan = nullptr;
        bool plan_loaded = false;
        double t0 = now();
        int ndev = 0;
        cli::check(cpd_device_count(&ndev), "device count");
        const int device = ndev ? (int)a.num("device", wid % ndev) : -1;
        cpd_plan_opts o{};
        o.threads = (int)a.num("threads", 0);
        o.verbose = a.has("verbose");
        // the hierarchy is contracted on this worker's GPU (the same hierarchy
        // as the host build's, in a fraction of its time); --ch-host: threads
        o.ch_gpu = ndev > 0 && !a.has("ch-host");
        o.ch_device = std::max(device, 0);
        // The build's HBM (batch buffers and two move-table row sets) is
        // committed on a host thread while the plan is contracted or loaded
        // (cpd_device_arena): committing 100-200 GB takes seconds.  --batch
        // 0 (default): what fits in 85% of the free HBM above --hbm-reserve
        // and a margin for the GPU contraction; --no-arena: the library
        // allocates at cpd_graph_set_batch, as before.
        const double hbm_reserve = a.real("hbm-reserve", 0.0) * (double)(1ull << 30);
        uint32_t batch = (uint32_t)a.num("batch", 0);
        const bool use_arena = ndev > 0 && !a.has("plan-only") && !a.has("no-arena");
        uint64_t arena_bytes = 0;
        double t_arena = 0.0, t_arena_wait = 0.0;
        int arena_rc = CPD_OK;
        std::string arena_err;
        std::thread arena_thr;
        struct JoinGuard {
            std::thread& t;
            ~JoinGuard() {
                if (t.joinable()) t.join();
            }
        } arena_guard{arena_thr};
        if (use_arena) {
            uint32_t maxdeg = 1;
            for (uint32_t v = 0; v < g.n; ++v) maxdeg = std::max(maxdeg, g.row_ptr[v + 1] - g.row_ptr[v]);
            if (batch == 0) {
                uint64_t fr = 0, tot = 0, per1k = 0;
                cli::check(cpd_device_mem_info(device, &fr, &tot), "device memory");
                cli::check(cpd_batch_bytes(g.n, maxdeg, 1024, &per1k), "batch bytes");
                const double margin = 24.0 * (double)(1ull << 30);  // the contraction's working set
                const double avail = (double)fr - hbm_reserve - margin;
                const double fit = avail > 0 ? 0.85 * avail / (double)per1k : 0.0;
                if (fit < 1.0)
                    throw std::runtime_error("HBM reserve leaves too little for a 1024-row batch");
                batch = (uint32_t)std::min((double)(batch_cap / 1024u), std::floor(fit)) * 1024u;
            }
            cli::check(cpd_batch_bytes(g.n, maxdeg, batch, &arena_bytes), "batch bytes");
            arena_thr = std::thread([&] {
                const double ta = now();
                arena_rc = cpd_device_arena(device, arena_bytes, a.has("arena-touch") ? 1 : 0);
                if (arena_rc != CPD_OK) arena_err = cpd_last_error();
                t_arena = now() - ta;
            });
        }
        if (use_cache) {
            // workers started together (make_cpds.py:58-60) share one cache:
            // one builds, the others wait for it and load its plan
            int status = 0;
            cli::check(cpd_plan_cache(plan_path.c_str(), g.row_ptr.data(), g.dst.data(), g.w.data(),
                                      g.n, g.m, &o, &plan, &status),
                       "plan");
            plan_loaded = status == 0;
            std::printf("make_cpd_auto: %s plan %s\n",
                        status == 0 ? "loaded" : status == 1 ? "built and cached" : "built (cache not written)",
                        plan_path.c_str());
        } else {
            cli::check(cpd_plan_create(g.row_ptr.data(), g.dst.data(), g.w.data(), g.n, g.m, &o, &plan),
                       "plan");
        }
        double t_plan = now() - t0;
        if (arena_thr.joinable()) {
            const double tw = now();
            arena_thr.join();
            t_arena_wait = now() - tw;
            if (arena_rc != CPD_OK)  // the library allocates at set_batch instead
                std::fprintf(stderr, "make_cpd_auto: HBM arena not committed (%s)\n", arena_err.c_str());
        }
        if (a.has("plan-only")) {  // warm the cache (host only, no GPU needed)
            std::printf("make_cpd_auto: plan ready in %.3fs\n", t_plan);
            cpd_plan_free(plan);
            return 0;
        }
        cpd_plan_info info{};
        cli::check(cpd_plan_info_get(plan, &info), "plan info");
        std::vector<uint32_t> order(g.n);
        cli::check(cpd_plan_order(plan, order.data()), "order");

        if (ndev == 0) {
            std::fprintf(stderr, "make_cpd_auto: no GPU visible (this build has no CPU path)\n");
            return 1;
        }
        cpd_graph* dg = nullptr;
        const double t_g0 = now();
        cli::check(cpd_graph_create(plan, device, &dg), "graph upload");
        const double t_graph = now() - t_g0;
        // --hbm-reserve GIB: HBM the auto batch leaves to what shares this GPU
        // (a fifo_auto serving beside the build)
        if (a.has("hbm-reserve"))
            cli::check(cpd_graph_set_hbm_reserve(dg, (uint64_t)(a.real("hbm-reserve", 0.0) * (1ull << 30))),
                       "hbm reserve");
        if (batch == 0) {  // --no-arena: what fits in 85% of the free HBM, capped as above
            uint32_t maxdeg = 1;
            for (uint32_t v = 0; v < g.n; ++v) maxdeg = std::max(maxdeg, g.row_ptr[v + 1] - g.row_ptr[v]);
            uint64_t fr = 0, tot = 0, per1k = 0;
            cli::check(cpd_device_mem_info(device, &fr, &tot), "device memory");
            cli::check(cpd_batch_bytes(g.n, maxdeg, 1024, &per1k), "batch bytes");
            const double fit = std::floor(0.85 * std::max(0.0, (double)fr - hbm_reserve) / (double)per1k);
            if (fit >= 1.0) batch = (uint32_t)std::min((double)(batch_cap / 1024u), fit) * 1024u;
        }
        cli::check(cpd_graph_set_batch(dg, batch), "batch");
        const double t_batch = now() - t_g0 - t_graph;
        // the .xy coordinates order each batch's lanes (compact target groups)
        if (g.x.size() == g.n && g.y.size() == g.n)
            cli::check(cpd_graph_set_coords(dg, g.x.data(), g.y.data()), "coordinates");
        uint32_t B = 0;
        cli::check(cpd_graph_get_batch(dg, &B), "batch");

        cpd::io::write_order(cpd::io::order_path(outdir, input), fp, order);

        double t_build = 0, t_io = 0;
        uint64_t rows_done = 0, runs_done = 0;
        double x_sum = 0, x_span = 0, w_sum = 0;
        uint64_t x_bytes = 0;
        const bool discard = a.has("discard");
        if (discard && a.has("no-pipeline"))
            throw std::runtime_error("--discard needs the pipelined writer");
        const double t_rows0 = now();
        const double t_setup = t_rows0 - t_g0;
        cpd_rows* rows = nullptr;
        if (a.has("no-pipeline")) {
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
                uint32_t nr = 0, words = 0, bits = 4;
                uint64_t tot = 0;
                cli::check(cpd_rows_count(rows, &nr, &tot), "rows");
                cli::check(cpd_rows_move_words(rows, &words), "move words");
                cli::check(cpd_rows_move_bits(rows, &bits), "move bits");
                std::vector<uint64_t> off(nr + 1);
                std::vector<uint32_t> runs(moves ? 0 : tot), mv(moves ? (size_t)nr * words : 0);
                if (moves) {
                    cli::check(cpd_rows_export_range(rows, 0, nr, off.data(), nullptr), "offsets");
                    cli::check(cpd_rows_export_moves(rows, 0, nr, mv.data()), "export moves");
                } else {
                    cli::check(cpd_rows_export(rows, off.data(), runs.data()), "export");
                }
                t_build += now() - tb;
                double ti = now();
                for (size_t k = 0; k < group.size(); ++k) {
                    const std::string path =
                        cpd::io::bucket_path(outdir, input, method, (uint32_t)key, group[k]);
                    if (moves) {
                        cpd::io::MoveBucket b;
                        b.n = g.n;
                        b.bid = group[k];
                        b.method = (uint32_t)mcode;
                        b.key = (uint32_t)key;
                        b.maxworker = (uint32_t)W;
                        b.words = words;
                        b.bits = bits;
                        b.fingerprint = fp;
                        b.targets.assign(targets.begin() + first[k], targets.begin() + first[k + 1]);
                        const uint32_t nb = (uint32_t)b.targets.size();
                        std::vector<uint32_t> c(nb);
                        for (uint32_t r = 0; r < nb; ++r)
                            c[r] = (uint32_t)(off[first[k] + r + 1] - off[first[k] + r]);
                        cpd::io::MoveBucketFile f(path, b, stripes);
                        f.write_counts(0, c.data(), nb);
                        f.write_rows(0, mv.data() + first[k] * (size_t)words, nb);
                        f.close(off[first[k + 1]] - off[first[k]]);
                        continue;
                    }
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
                    cpd::io::write_bucket(path, b);
                }
                t_io += now() - ti;
                rows_done += nr;
                runs_done += tot;
            }
        } else {
            Pipeline pl(dg, B, (int)a.num("write-threads", 16), discard, moves, stripes);
            std::vector<uint32_t> targets;
            std::vector<CpdBucket> heads(owned.size());
            std::vector<uint64_t> first(owned.size() + 1, 0);
            for (size_t k = 0; k < owned.size(); ++k) {
                CpdBucket& b = heads[k];
                b.n = g.n;
                b.bid = owned[k];
                b.method = (uint32_t)mcode;
                b.key = (uint32_t)key;
                b.maxworker = (uint32_t)W;
                b.fingerprint = fp;
                b.targets = bucket_nodes(owned[k]);
                first[k] = targets.size();
                targets.insert(targets.end(), b.targets.begin(), b.targets.end());
                b.targets.shrink_to_fit();
            }
            first[owned.size()] = targets.size();
            std::vector<std::string> paths(owned.size());
            for (size_t k = 0; k < owned.size(); ++k)
                paths[k] = cpd::io::bucket_path(outdir, input, method, (uint32_t)key, owned[k]);
            pl.run(targets, first, heads, paths);
            t_build = pl.t_build;
            t_io = pl.t_wait;
            rows_done = targets.size();
            runs_done = pl.runs;
            x_sum = pl.x_sum;
            x_bytes = pl.x_bytes;
            x_span = pl.x_last > pl.x_first ? pl.x_last - pl.x_first : 0.0;
            w_sum = pl.w_sum;
        }
        const double t_rows = now() - t_rows0;
        const double t_f0 = now();
        if (rows) cpd_rows_free(rows);
        cpd_graph_free(dg);
        cpd_plan_free(plan);
        if (use_arena) cli::check(cpd_device_arena_release(device), "arena release");
        const double t_free = now() - t_f0;
        double rate = t_build > 0 ? rows_done / t_build : 0.0;
        std::printf(
            "make_cpd_auto: worker %lld/%lld device %d: %llu rows in %zu buckets, %llu runs "
            "(%.1f per row); read %.3fs plan %.3fs (hierarchy %llu arcs, %u+%u levels) "
            "build %.3fs = %.1f rows/s, %.3f GTEPS; write %.3fs%s; total %.3fs\n",
            wid, W, device, (unsigned long long)rows_done, owned.size(),
            (unsigned long long)runs_done, rows_done ? (double)runs_done / rows_done : 0.0, t_read,
            t_plan, (unsigned long long)(info.ch_up_arcs + info.ch_dn_arcs), info.levels_up,
            info.levels_dn, t_build, rate, rate * g.m / 1e9, t_io,
            a.has("no-pipeline") ? "" : " (not hidden behind the build)", now() - t_start);
        // one machine-readable line (bench.py's full-build leg reads it):
        // rows_s = every owned row built and exported (and written, unless
        // --discard); export = the D2H copies (summed over writer threads,
        // and their wall span); wait = time the build loop stalled on them
        std::printf(
            "make_cpd_auto-json: {\"worker\": %lld, \"maxworker\": %lld, \"rows\": %llu, "
            "\"runs\": %llu, \"batch\": %u, \"discard\": %s, \"read_s\": %.3f, \"plan_s\": %.3f, "
            "\"plan_cached\": %s, \"graph_s\": %.3f, \"batch_alloc_s\": %.3f, \"setup_s\": %.3f, "
            "\"rows_s\": %.3f, \"build_calls_s\": %.3f, \"wait_s\": %.3f, \"free_s\": %.3f, "
            "\"export_bytes\": %llu, \"export_thread_s\": %.3f, \"export_span_s\": %.3f, "
            "\"write_thread_s\": %.3f, \"format\": \"%s\", \"arena_GB\": %.2f, "
            "\"arena_s\": %.3f, \"arena_wait_s\": %.3f, \"total_s\": %.3f}\n",
            wid, W, (unsigned long long)rows_done, (unsigned long long)runs_done, B,
            discard ? "true" : "false", t_read, t_plan, plan_loaded ? "true" : "false", t_graph,
            t_batch, t_setup, t_rows, t_build, t_io, t_free, (unsigned long long)x_bytes, x_sum, x_span,
            w_sum, format.c_str(), arena_rc == CPD_OK ? arena_bytes / 1e9 : 0.0, t_arena,
            t_arena_wait, now() - t_start);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "make_cpd_auto: %s\n", e.what());
        return 1;
    }
    return 0;
}

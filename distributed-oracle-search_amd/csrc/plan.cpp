// cpd_plan: the once-per-graph host preprocessing (column order + hierarchy).
#include <errno.h>
#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <fstream>
#include <exception>
#include <memory>
#include <thread>

#include "cpd_internal.hpp"

using namespace cpd;

namespace {

const char kPlanMagic[8] = {'D', 'O', 'S', 'P', 'L', 'A', 'N', '1'};

// A loaded hierarchy must be self-consistent before anything indexes by it:
// empty (a query-only plan) or rank / levels of n entries, up / down CSR with
// n + 1 monotone offsets ending at their arc counts, heads < n, levels below
// their level counts.
void check_hierarchy(const cpd_plan& p) {
    const Hierarchy& H = p.ch;
    const size_t n = p.n;
    if (H.rank.empty()) {
        CPD_REQUIRE(H.up_off.empty() && H.dn_off.empty() && H.level_up.empty() &&
                        H.level_dn.empty(),
                    CPD_E_IO, "plan file: partial hierarchy");
        return;
    }
    CPD_REQUIRE(H.rank.size() == n && H.level_up.size() == n && H.level_dn.size() == n,
                CPD_E_IO, "plan file: hierarchy arrays of the wrong size");
    auto csr = [&](const std::vector<uint64_t>& off, const std::vector<uint32_t>& to,
                   const std::vector<uint32_t>& wt) {
        CPD_REQUIRE(off.size() == n + 1 && off[0] == 0 && off[n] == to.size() &&
                        to.size() == wt.size(),
                    CPD_E_IO, "plan file: hierarchy arcs inconsistent");
        for (size_t v = 0; v < n; ++v)
            CPD_REQUIRE(off[v] <= off[v + 1], CPD_E_IO, "plan file: arc offsets not monotone");
        for (uint32_t x : to) CPD_REQUIRE(x < n, CPD_E_IO, "plan file: arc head out of range");
    };
    csr(H.up_off, H.up_dst, H.up_w);
    csr(H.dn_off, H.dn_dst, H.dn_w);
    for (size_t v = 0; v < n; ++v)
        CPD_REQUIRE(H.level_up[v] < H.nlev_up && H.level_dn[v] < H.nlev_dn, CPD_E_IO,
                    "plan file: level out of range");
}

template <class T>
void put_vec(std::ofstream& f, const std::vector<T>& v) {
    uint64_t k = v.size();
    f.write(reinterpret_cast<const char*>(&k), sizeof k);
    if (k) f.write(reinterpret_cast<const char*>(v.data()), k * sizeof(T));
}

template <class T>
void get_vec(std::ifstream& f, std::vector<T>& v) {
    uint64_t k = 0;
    f.read(reinterpret_cast<char*>(&k), sizeof k);
    CPD_REQUIRE(f && k < (1ull << 40), CPD_E_IO, "plan file truncated");
    v.resize(k);
    if (k) f.read(reinterpret_cast<char*>(v.data()), k * sizeof(T));
    CPD_REQUIRE(f, CPD_E_IO, "plan file truncated");
}

}  // namespace

extern "C" {

int cpd_plan_create(const uint32_t* row_ptr, const uint32_t* dst, const uint32_t* w,
                    uint32_t n, uint32_t m, const cpd_plan_opts* opts, cpd_plan** out) {
    return guarded([&] {
        CPD_REQUIRE(out, CPD_E_ARG, "plan: null output");
        *out = nullptr;
        check_csr(n, m, row_ptr, dst, w);
        auto p = std::make_unique<cpd_plan>();
        p->n = n;
        p->m = m;
        p->row_ptr.assign(row_ptr, row_ptr + n + 1);
        p->dst.assign(dst, dst + m);
        p->w.assign(w, w + m);
        int threads = opts ? opts->threads : 0;
        uint32_t settle = opts ? opts->witness_settle : 0;
        int verbose = opts ? opts->verbose : 0;
        // the column order and the distance bound (a DFS and two Dijkstras,
        // host-serial) run beside the hierarchy build, which needs neither
        std::exception_ptr side_err;
        std::thread side([&] {
            try {
                p->order.resize(n);
                dfs_preorder(n, row_ptr, dst, p->order.data());
                p->inv.resize(n);
                for (uint32_t v = 0; v < n; ++v) p->inv[p->order[v]] = v;
                p->dist_bound = distance_bound(n, row_ptr, dst, w);
            } catch (...) {
                side_err = std::current_exception();
            }
        });
        struct Join {
            std::thread& t;
            ~Join() {
                if (t.joinable()) t.join();
            }
        } join{side};
        std::exception_ptr ch_err;
        if (!(opts && opts->no_hierarchy)) {
            double t0 = now_seconds();
            try {
                if (opts && opts->ch_gpu) {
                    try {
                        p->ch = build_hierarchy_gpu(n, row_ptr, dst, w, opts->ch_device, settle,
                                                    verbose);
                    } catch (const Error& e) {
                        // the GPU contraction ran out of device memory or
                        // failed at run time: the host build gives the same
                        // hierarchy.  No device at all stays an
                        // error (ch_gpu asks for the GPU).
                        const bool no_device =
                            std::string(e.what()).find("no GPU visible") != std::string::npos;
                        if (!(e.code == CPD_E_OOM || (e.code == CPD_E_HIP && !no_device))) throw;
                        std::fprintf(stderr, "[cpd] GPU contraction failed (%s); contracting on "
                                             "host threads\n", e.what());
                        p->ch = build_hierarchy(n, row_ptr, dst, w, threads, settle, verbose);
                    }
                } else {
                    p->ch = build_hierarchy(n, row_ptr, dst, w, threads, settle, verbose);
                }
            } catch (...) {
                ch_err = std::current_exception();
            }
            p->ch_seconds = now_seconds() - t0;
        }
        side.join();
        // the graph's own errors first (as when they were checked before the
        // hierarchy): a distance range the u32 path cannot hold also makes
        // the contraction fail on a shortcut weight
        if (side_err) std::rethrow_exception(side_err);
        CPD_REQUIRE(p->dist_bound < 0xFFFFFFFFull, CPD_E_RANGE,
                    "graph distances may reach 2^32-1; the u32 distance path "
                    "cannot represent them");
        if (ch_err) std::rethrow_exception(ch_err);
        *out = p.release();
    });
}

int cpd_plan_info_get(const cpd_plan* p, cpd_plan_info* info) {
    return guarded([&] {
        CPD_REQUIRE(p && info, CPD_E_ARG, "plan info: null argument");
        info->n = p->n;
        info->m = p->m;
        CPD_REQUIRE(p->ch.up_off.empty() || p->ch.up_off.size() == (size_t)p->n + 1, CPD_E_ARG,
                    "plan hierarchy inconsistent");
        info->ch_up_arcs = p->ch.up_off.empty() ? 0 : p->ch.up_off[p->n];
        info->ch_dn_arcs = p->ch.dn_off.empty() ? 0 : p->ch.dn_off[p->n];
        info->levels_up = p->ch.nlev_up;
        info->levels_dn = p->ch.nlev_dn;
        info->dist_bound = p->dist_bound;
        info->ch_seconds = p->ch_seconds;
    });
}

int cpd_plan_order(const cpd_plan* p, uint32_t* order) {
    return guarded([&] {
        CPD_REQUIRE(p && order, CPD_E_ARG, "plan order: null argument");
        std::memcpy(order, p->order.data(), p->n * sizeof(uint32_t));
    });
}

int cpd_plan_export_ch(const cpd_plan* p, uint32_t* rank, uint64_t* up_off,
                       uint32_t* up_dst, uint32_t* up_w, uint64_t* dn_off,
                       uint32_t* dn_dst, uint32_t* dn_w, uint32_t* level_up,
                       uint32_t* level_dn) {
    return guarded([&] {
        CPD_REQUIRE(p, CPD_E_ARG, "plan export: null plan");
        CPD_REQUIRE(!p->ch.rank.empty(), CPD_E_ARG, "plan has no hierarchy");
        const Hierarchy& H = p->ch;
        auto cp = [](auto* dstp, const auto& v) {
            if (dstp && !v.empty()) std::memcpy(dstp, v.data(), v.size() * sizeof(v[0]));
        };
        cp(rank, H.rank);
        cp(up_off, H.up_off);
        cp(up_dst, H.up_dst);
        cp(up_w, H.up_w);
        cp(dn_off, H.dn_off);
        cp(dn_dst, H.dn_dst);
        cp(dn_w, H.dn_w);
        cp(level_up, H.level_up);
        cp(level_dn, H.level_dn);
    });
}

int cpd_plan_save(const cpd_plan* p, const char* path) {
    return guarded([&] {
        CPD_REQUIRE(p && path, CPD_E_ARG, "plan save: null argument");
        // a name of this process and call alone: concurrent savers (workers
        // started together, make_cpds.py:58-60) never truncate each other
        static std::atomic<unsigned> seq{0};
        std::string tmp = std::string(path) + ".tmp." + std::to_string(::getpid()) + "." +
                          std::to_string(seq++);
        struct Unlink {  // the temporary never outlives a failed save
            const std::string& f;
            bool armed = true;
            ~Unlink() {
                if (armed) ::unlink(f.c_str());
            }
        } cleanup{tmp};
        {
            std::ofstream f(tmp, std::ios::binary);
            CPD_REQUIRE(f, CPD_E_IO, std::string("cannot write ") + tmp);
            f.write(kPlanMagic, 8);
            uint32_t hdr[4] = {p->n, p->m, p->ch.nlev_up, p->ch.nlev_dn};
            f.write(reinterpret_cast<const char*>(hdr), sizeof hdr);
            f.write(reinterpret_cast<const char*>(&p->dist_bound), 8);
            f.write(reinterpret_cast<const char*>(&p->ch_seconds), 8);
            put_vec(f, p->row_ptr);
            put_vec(f, p->dst);
            put_vec(f, p->w);
            put_vec(f, p->order);
            const Hierarchy& H = p->ch;
            put_vec(f, H.rank);
            put_vec(f, H.up_off);
            put_vec(f, H.up_dst);
            put_vec(f, H.up_w);
            put_vec(f, H.dn_off);
            put_vec(f, H.dn_dst);
            put_vec(f, H.dn_w);
            put_vec(f, H.level_up);
            put_vec(f, H.level_dn);
            f.flush();
            CPD_REQUIRE(f, CPD_E_IO, "plan write failed");
        }
        CPD_REQUIRE(std::rename(tmp.c_str(), path) == 0, CPD_E_IO, "plan rename failed");
        cleanup.armed = false;
    });
}

int cpd_plan_load(const char* path, cpd_plan** out) {
    return guarded([&] {
        CPD_REQUIRE(path && out, CPD_E_ARG, "plan load: null argument");
        *out = nullptr;
        std::ifstream f(path, std::ios::binary);
        CPD_REQUIRE(f, CPD_E_IO, std::string("cannot open ") + path);
        char magic[8];
        f.read(magic, 8);
        CPD_REQUIRE(f && std::memcmp(magic, kPlanMagic, 8) == 0, CPD_E_IO,
                    "not a plan file");
        auto p = std::make_unique<cpd_plan>();
        uint32_t hdr[4];
        f.read(reinterpret_cast<char*>(hdr), sizeof hdr);
        f.read(reinterpret_cast<char*>(&p->dist_bound), 8);
        f.read(reinterpret_cast<char*>(&p->ch_seconds), 8);
        p->n = hdr[0];
        p->m = hdr[1];
        p->ch.nlev_up = hdr[2];
        p->ch.nlev_dn = hdr[3];
        get_vec(f, p->row_ptr);
        get_vec(f, p->dst);
        get_vec(f, p->w);
        get_vec(f, p->order);
        Hierarchy& H = p->ch;
        get_vec(f, H.rank);
        get_vec(f, H.up_off);
        get_vec(f, H.up_dst);
        get_vec(f, H.up_w);
        get_vec(f, H.dn_off);
        get_vec(f, H.dn_dst);
        get_vec(f, H.dn_w);
        get_vec(f, H.level_up);
        get_vec(f, H.level_dn);
        CPD_REQUIRE(p->row_ptr.size() == (size_t)p->n + 1 && p->order.size() == p->n &&
                        p->dst.size() == p->m && p->w.size() == p->m,
                    CPD_E_IO, "plan file inconsistent");
        check_csr(p->n, p->m, p->row_ptr.data(), p->dst.data(), p->w.data());
        // the column order must be a permutation (inv[] and every GPU array
        // are indexed by it)
        p->inv.assign(p->n, 0xFFFFFFFFu);
        for (uint32_t v = 0; v < p->n; ++v) {
            CPD_REQUIRE(p->order[v] < p->n && p->inv[p->order[v]] == 0xFFFFFFFFu, CPD_E_IO,
                        "plan file: column order is not a permutation");
            p->inv[p->order[v]] = v;
        }
        check_hierarchy(*p);
        *out = p.release();
    });
}

int cpd_plan_cache(const char* path, const uint32_t* row_ptr, const uint32_t* dst,
                   const uint32_t* w, uint32_t n, uint32_t m, const cpd_plan_opts* opts,
                   cpd_plan** out, int* status) {
    return guarded([&] {
        CPD_REQUIRE(path && out, CPD_E_ARG, "plan cache: null argument");
        *out = nullptr;
        check_csr(n, m, row_ptr, dst, w);
        // one builder per cache file: the others block here until it has
        // saved, then load its plan
        const std::string lock = std::string(path) + ".lock";
        const int fd = ::open(lock.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
        if (fd >= 0)
            while (::flock(fd, LOCK_EX) != 0 && errno == EINTR) {
            }
        struct Unlock {
            int fd;
            ~Unlock() {
                if (fd >= 0) ::close(fd);  // releases the flock
            }
        } unlock{fd};
        cpd_plan* p = nullptr;
        if (cpd_plan_load(path, &p) == CPD_OK) {
            const bool same = p->n == n && p->m == m &&
                              std::equal(p->row_ptr.begin(), p->row_ptr.end(), row_ptr) &&
                              std::equal(p->dst.begin(), p->dst.end(), dst) &&
                              std::equal(p->w.begin(), p->w.end(), w) &&
                              (p->ch.rank.empty() == (opts && opts->no_hierarchy));
            if (same) {
                *out = p;
                if (status) *status = 0;
                return;
            }
            cpd_plan_free(p);  // built for another graph: rebuild over it
        }
        int rc = cpd_plan_create(row_ptr, dst, w, n, m, opts, &p);
        if (rc != CPD_OK) throw Error(rc, cpd_last_error());
        rc = cpd_plan_save(p, path);
        if (status) *status = rc == CPD_OK ? 1 : 2;
        *out = p;
    });
}

void cpd_plan_free(cpd_plan* p) { delete p; }

}  // extern "C"

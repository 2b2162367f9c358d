// File formats on the drop-in boundary — see cpd_io.hpp.
#include "cpd_io.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <thread>

#include "cpd_internal.hpp"

namespace cpd {
namespace io {
namespace {

std::string slurp(const std::string& path) {
    std::FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw Error(CPD_E_IO, "cannot open " + path);
    std::string s;
    char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, k);
    std::fclose(f);
    return s;
}

// Minimal tokenizer over one line.
struct Line {
    const char* p;
    const char* e;
    bool word(std::string& out) {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
        if (p >= e) return false;
        const char* b = p;
        while (p < e && *p != ' ' && *p != '\t' && *p != '\r') ++p;
        out.assign(b, p);
        return true;
    }
    bool i64(int64_t& v) {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
        if (p >= e) return false;
        bool neg = false;
        if (*p == '-' || *p == '+') neg = *p++ == '-';
        if (p >= e || *p < '0' || *p > '9') return false;
        int64_t r = 0;
        while (p < e && *p >= '0' && *p <= '9') r = r * 10 + (*p++ - '0');
        v = neg ? -r : r;
        return true;
    }
};

template <class F>
void for_lines(const std::string& s, F&& f) {
    size_t i = 0, lineno = 0;
    while (i < s.size()) {
        size_t j = s.find('\n', i);
        if (j == std::string::npos) j = s.size();
        f(Line{s.data() + i, s.data() + j}, lineno++);
        i = j + 1;
    }
}

uint32_t to_u32(int64_t v, const std::string& what) {
    if (v < 0 || v > 0xFFFFFFFFll) throw Error(CPD_E_IO, what + " out of range");
    return (uint32_t)v;
}

const char kBucketMagic[8] = {'D', 'O', 'S', 'C', 'P', 'D', '0', '1'};
const char kOrderMagic[8] = {'D', 'O', 'S', 'O', 'R', 'D', '0', '1'};
const char kMoveBucketMagic[8] = {'D', 'O', 'S', 'C', 'P', 'D', '0', '2'};
const char kMoveStripedMagic[8] = {'D', 'O', 'S', 'C', 'P', 'D', '0', '3'};

}  // namespace

XYGraph read_xy(const std::string& path) {
    std::string s = slurp(path);
    XYGraph g;
    int64_t hn = -1, hm = -1;
    struct E { uint32_t a, b, w; };
    std::vector<E> edges;
    std::vector<std::pair<uint32_t, std::pair<int32_t, int32_t>>> verts;
    for_lines(s, [&](Line ln, size_t lineno) {
        std::string tag;
        Line probe = ln;
        if (!probe.word(tag)) return;
        if (tag == "nodes") {
            int64_t n, m;
            std::string et;
            if (!probe.i64(n) || !probe.word(et) || et != "edges" || !probe.i64(m))
                throw Error(CPD_E_IO, path + ": bad header line " + std::to_string(lineno + 1));
            hn = n;
            hm = m;
            edges.reserve((size_t)m);
        } else if (tag == "v") {
            int64_t id, x, y;
            if (!probe.i64(id) || !probe.i64(x) || !probe.i64(y))
                throw Error(CPD_E_IO, path + ": bad v line " + std::to_string(lineno + 1));
            verts.push_back({to_u32(id, "node id"), {(int32_t)x, (int32_t)y}});
        } else if (tag == "e") {
            int64_t a, b, w;
            if (!probe.i64(a) || !probe.i64(b) || !probe.i64(w))
                throw Error(CPD_E_IO, path + ": bad e line " + std::to_string(lineno + 1));
            edges.push_back({to_u32(a, "edge tail"), to_u32(b, "edge head"), to_u32(w, "edge cost")});
        }
        // anything else (comments) is ignored
    });
    if (hn < 0) throw Error(CPD_E_IO, path + ": missing 'nodes N edges M' header");
    if (hm != (int64_t)edges.size())
        throw Error(CPD_E_IO, path + ": header says " + std::to_string(hm) + " edges, file has " +
                                  std::to_string(edges.size()));
    g.n = (uint32_t)hn;
    g.m = (uint32_t)edges.size();
    g.x.assign(g.n, 0);
    g.y.assign(g.n, 0);
    for (auto& v : verts) {
        if (v.first >= g.n) throw Error(CPD_E_IO, path + ": vertex id out of range");
        g.x[v.first] = v.second.first;
        g.y[v.first] = v.second.second;
    }
    g.row_ptr.assign(g.n + 1, 0);
    for (auto& e : edges) {
        if (e.a >= g.n || e.b >= g.n) throw Error(CPD_E_IO, path + ": edge endpoint out of range");
        g.row_ptr[e.a + 1]++;
    }
    for (uint32_t v = 0; v < g.n; ++v) g.row_ptr[v + 1] += g.row_ptr[v];
    g.dst.resize(g.m);
    g.w.resize(g.m);
    std::vector<uint32_t> pos(g.row_ptr.begin(), g.row_ptr.end() - 1);
    for (auto& e : edges) {  // stable: file order within a node
        uint32_t p = pos[e.a]++;
        g.dst[p] = e.b;
        g.w[p] = e.w;
    }
    return g;
}

void write_xy(const std::string& path, uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
              const uint32_t* w, const int32_t* x, const int32_t* y) {
    std::vector<char> buf(1 << 20);  // outlives the FILE (closed by guard first)
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw Error(CPD_E_IO, "cannot write " + path);
    std::unique_ptr<std::FILE, int (*)(std::FILE*)> guard(f, std::fclose);
    std::setvbuf(f, buf.data(), _IOFBF, buf.size());
    std::fprintf(f, "c cpd-mi355x xy graph\nc nodes are 0-based; edges grouped by tail in out-edge order\nc\n");
    std::fprintf(f, "nodes %u edges %u\n", n, row_ptr[n]);
    for (uint32_t v = 0; v < n; ++v)
        std::fprintf(f, "v %u %d %d\n", v, x ? x[v] : 0, y ? y[v] : 0);
    for (uint32_t v = 0; v < n; ++v)
        for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
            std::fprintf(f, "e %u %u %u\n", v, dst[e], w[e]);
    if (std::ferror(f)) throw Error(CPD_E_IO, "write failed: " + path);
}

std::vector<uint32_t> read_diff(const std::string& path, const XYGraph& g) {
    std::vector<uint32_t> w = g.w;
    if (path.empty() || path == "-") return w;
    std::string s = slurp(path);
    for_lines(s, [&](Line ln, size_t lineno) {
        Line probe = ln;
        std::string tag;
        Line save = probe;
        if (!probe.word(tag)) return;
        Line nums = (tag == "e") ? probe : save;
        if (tag != "e" && !(tag[0] >= '0' && tag[0] <= '9')) return;  // comment / header
        int64_t a, b, c;
        if (!nums.i64(a) || !nums.i64(b) || !nums.i64(c))
            throw Error(CPD_E_IO, path + ": bad diff line " + std::to_string(lineno + 1));
        uint32_t ua = to_u32(a, "diff tail"), ub = to_u32(b, "diff head");
        if (ua >= g.n || ub >= g.n) throw Error(CPD_E_IO, path + ": diff node out of range");
        bool found = false;
        for (uint32_t e = g.row_ptr[ua]; e < g.row_ptr[ua + 1]; ++e)
            if (g.dst[e] == ub) {
                w[e] = to_u32(c, "diff cost");
                found = true;
                break;
            }
        if (!found)
            throw Error(CPD_E_IO, path + ": diff line " + std::to_string(lineno + 1) +
                                      " names a missing edge");
    });
    return w;
}

void write_diff(const std::string& path, const XYGraph& g, const std::vector<uint32_t>& wc) {
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw Error(CPD_E_IO, "cannot write " + path);
    std::unique_ptr<std::FILE, int (*)(std::FILE*)> guard(f, std::fclose);
    std::fprintf(f, "c cpd-mi355x congestion diff: e from to new_cost\n");
    for (uint32_t v = 0; v < g.n; ++v)
        for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e)
            if (wc[e] != g.w[e]) std::fprintf(f, "e %u %u %u\n", v, g.dst[e], wc[e]);
}

Pairs read_scen(const std::string& path) {
    std::string s = slurp(path);
    Pairs q;
    for_lines(s, [&](Line ln, size_t lineno) {
        if (ln.p >= ln.e || *ln.p != 'q') return;  // read_p2p: line[0] == "q"
        ++ln.p;
        int64_t a, b;
        if (!ln.i64(a) || !ln.i64(b))
            throw Error(CPD_E_IO, path + ": bad q line " + std::to_string(lineno + 1));
        q.push_back({to_u32(a, "query source"), to_u32(b, "query target")});
    });
    return q;
}

void write_scen(const std::string& path, const Pairs& q) {
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw Error(CPD_E_IO, "cannot write " + path);
    std::unique_ptr<std::FILE, int (*)(std::FILE*)> guard(f, std::fclose);
    std::fprintf(f, "p aux sp p2p %zu\n", q.size());
    for (auto& p : q) std::fprintf(f, "q %u %u\n", p.first, p.second);
}

Pairs read_query_file(const std::string& path) {
    std::vector<uint32_t> s, t;
    read_query_file(path, 1, s, t);
    Pairs q(s.size());
    for (size_t i = 0; i < s.size(); ++i) q[i] = {s[i], t[i]};
    return q;
}

// The whole file in one buffer: its size from fstat, then pread in pieces
// of up to 1 GiB (split over `threads` when large) — no growth by appends.
// The file into `out` (resized to it; a buffer kept across calls, so a
// server's requests after the first read into pages already mapped — a
// fresh 14-MB buffer cost ~8 ms of page faults per 1M-query request), by up
// to `threads` positional reads of >= 4 MB.
static void read_whole(const std::string& path, int threads, std::vector<char>& out) {
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) throw Error(CPD_E_IO, "cannot open " + path);
    struct stat st {};
    if (::fstat(fd, &st) != 0) {
        ::close(fd);
        throw Error(CPD_E_IO, "cannot stat " + path);
    }
    out.resize((size_t)st.st_size);
    const size_t total = out.size();
    const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), total >> 22));
    std::vector<char> ok(T, 1);
    auto piece = [&](size_t k) {
        size_t a = total * k / T, b = total * (k + 1) / T;
        while (a < b) {
            const ssize_t r = ::pread(fd, out.data() + a, std::min<size_t>(b - a, size_t(1) << 30), (off_t)a);
            if (r <= 0) {
                ok[k] = 0;
                return;
            }
            a += (size_t)r;
        }
    };
    if (T == 1) {
        piece(0);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 0; k < T; ++k) th.emplace_back(piece, k);
        for (auto& x : th) x.join();
    }
    ::close(fd);
    for (char c : ok)
        if (!c) throw Error(CPD_E_IO, path + ": short read");
}

void read_query_file(const std::string& path, int threads, std::vector<uint32_t>& s,
                     std::vector<uint32_t>& t) {
    // buffers kept per calling thread across calls (fifo_auto's requests)
    thread_local std::vector<char> text_buf;
    thread_local std::vector<std::vector<uint32_t>> ps_buf, pt_buf;
    // (the parse threads reach them through these references: a
    // thread_local named in their code would be their own, empty)
    std::vector<char>& text = text_buf;
    std::vector<std::vector<uint32_t>>& ps = ps_buf;
    std::vector<std::vector<uint32_t>>& pt = pt_buf;
    read_whole(path, threads, text);
    const char* const b = text.data();
    const char* const e = b + text.size();
    // header: the query count (process_query.py:95); a file without one is empty
    const char* body = static_cast<const char*>(std::memchr(b, '\n', text.size()));
    body = body ? body + 1 : e;
    int64_t expect = 0;
    {
        Line h{b, body};
        if (!text.empty() && !h.i64(expect)) throw Error(CPD_E_IO, path + ": missing query count");
    }
    // the body cut into pieces at line starts, each parsed by a thread into
    // its own arrays, then copied into place: a 1M-query file (~14 MB) is a
    // ~30-ms scan for one thread (process_query.py:93-96 writes one per worker
    // per batch)
    const size_t len = (size_t)(e - body);
    const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), len >> 20));
    std::vector<const char*> cut(T + 1, e);
    cut[0] = body;
    for (size_t k = 1; k < T; ++k) {
        const char* p = body + len * k / T;
        if (p < cut[k - 1]) p = cut[k - 1];
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
        cut[k] = nl ? nl + 1 : e;
    }
    if (ps.size() < T) {
        ps.resize(T);
        pt.resize(T);
    }
    std::vector<const char*> bad(T, nullptr);
    auto parse = [&](size_t k) {
        const char* p = cut[k];
        const char* end = cut[k + 1];
        // into vectors of this thread's own (taken over from ps[k] / pt[k]
        // and handed back at the end): pushing through ps[k] rewrote its
        // end pointer, which shares a cache line with its neighbours' —
        // 4 threads parsed 3-5x slower than 1 (profiles/query_parse/)
        std::vector<uint32_t> ls, lt;
        ls.swap(ps[k]);
        lt.swap(pt[k]);
        ls.clear();
        lt.clear();
        ls.reserve((size_t)(end - p) / 12 + 1);
        lt.reserve((size_t)(end - p) / 12 + 1);
        struct Back {  // the vectors go back on every exit
            std::vector<uint32_t>& a;
            std::vector<uint32_t>& b;
            std::vector<uint32_t>& la;
            std::vector<uint32_t>& lb;
            ~Back() {
                a.swap(la);
                b.swap(lb);
            }
        } back{ps[k], pt[k], ls, lt};
        // one scan per line (what Line::i64 twice accepts: blanks, tabs and
        // CRs around, a sign; a line whose first field is no number is
        // skipped as blank); magnitudes clamp above 2^32 so they are refused
        auto ws = [](char c) { return c == ' ' || c == '\t' || c == '\r'; };
        auto num = [&](const char*& q, int64_t& v) {
            while (q < end && ws(*q)) ++q;
            bool neg = false;
            if (q < end && (*q == '-' || *q == '+')) neg = *q++ == '-';
            if (q >= end || *q < '0' || *q > '9') return false;
            int64_t r = 0;
            while (q < end && *q >= '0' && *q <= '9') {
                r = std::min<int64_t>(r * 10 + (*q++ - '0'), int64_t(1) << 33);
            }
            v = neg ? -r : r;
            return true;
        };
        while (p < end) {
            const char* q = p;
            int64_t x, y;
            if (!num(q, x)) {  // blank (or no number first): the next line
                const char* nl = static_cast<const char*>(std::memchr(q, '\n', (size_t)(end - q)));
                p = nl ? nl + 1 : end;
                continue;
            }
            if (!num(q, y) || x < 0 || y < 0 || x > 0xFFFFFFFFll || y > 0xFFFFFFFFll) {
                bad[k] = p;
                return;
            }
            ls.push_back((uint32_t)x);
            lt.push_back((uint32_t)y);
            if (q < end && *q == '\n') {
                p = q + 1;
            } else {
                const char* nl = static_cast<const char*>(std::memchr(q, '\n', (size_t)(end - q)));
                p = nl ? nl + 1 : end;
            }
        }
    };
    if (T == 1) {
        parse(0);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 0; k < T; ++k) th.emplace_back(parse, k);
        for (auto& x : th) x.join();
    }
    for (size_t k = 0; k < T; ++k)
        if (bad[k]) {
            const size_t lineno = 1 + (size_t)std::count(b, bad[k], '\n');
            throw Error(CPD_E_IO, path + ": bad query line " + std::to_string(lineno));
        }
    std::vector<size_t> at(T + 1, 0);
    for (size_t k = 0; k < T; ++k) at[k + 1] = at[k] + ps[k].size();
    if ((int64_t)at[T] != expect)
        throw Error(CPD_E_IO, path + ": header says " + std::to_string(expect) + " queries, file has " +
                                  std::to_string(at[T]));
    s.resize(at[T]);
    t.resize(at[T]);
    for (size_t k = 0; k < T; ++k) {
        std::copy(ps[k].begin(), ps[k].end(), s.begin() + (std::ptrdiff_t)at[k]);
        std::copy(pt[k].begin(), pt[k].end(), t.begin() + (std::ptrdiff_t)at[k]);
    }
}

uint64_t graph_fingerprint(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                           const uint32_t* w) {
    uint64_t h = 1469598103934665603ull;
    auto mixin = [&](const void* p, size_t bytes) {
        const unsigned char* c = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < bytes; ++i) h = (h ^ c[i]) * 1099511628211ull;
    };
    mixin(&n, 4);
    mixin(row_ptr, (size_t)(n + 1) * 4);
    mixin(dst, (size_t)row_ptr[n] * 4);
    mixin(w, (size_t)row_ptr[n] * 4);
    return h;
}

std::string xy_stem(const std::string& xy_path) {
    size_t s = xy_path.find_last_of('/');
    return s == std::string::npos ? xy_path : xy_path.substr(s + 1);
}

std::string bucket_path(const std::string& outdir, const std::string& xy_path,
                        const std::string& method, uint32_t key, uint32_t bid) {
    return outdir + "/" + xy_stem(xy_path) + "-" + method + "-" + std::to_string(key) + "-" +
           std::to_string(bid) + ".cpd";
}

std::string order_path(const std::string& outdir, const std::string& xy_path) {
    return outdir + "/" + xy_stem(xy_path) + ".order";
}

void write_bucket(const std::string& path, const CpdBucket& b) {
    std::string tmp = path + ".tmp";
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) throw Error(CPD_E_IO, "cannot write " + tmp);
        uint32_t nrows = (uint32_t)b.targets.size();
        uint64_t total = b.offsets.empty() ? 0 : b.offsets.back();
        f.write(kBucketMagic, 8);
        uint32_t h32[6] = {b.n, nrows, b.bid, b.method, b.key, b.maxworker};
        f.write(reinterpret_cast<const char*>(h32), sizeof h32);
        f.write(reinterpret_cast<const char*>(&total), 8);
        f.write(reinterpret_cast<const char*>(&b.fingerprint), 8);
        f.write(reinterpret_cast<const char*>(b.targets.data()), nrows * 4ull);
        f.write(reinterpret_cast<const char*>(b.offsets.data()), (nrows + 1) * 8ull);
        f.write(reinterpret_cast<const char*>(b.runs.data()), total * 4ull);
        if (!f) throw Error(CPD_E_IO, "write failed: " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw Error(CPD_E_IO, "rename failed: " + path);
}

// bucket layout: magic 8 | n nrows bid method key maxworker (6 x u32) |
// total u64 | fingerprint u64 | targets u32[nrows] | offsets u64[nrows+1] |
// runs u32[total]
static constexpr uint64_t kBucketHeader = 8 + 24 + 8 + 8;

BucketFile::BucketFile(const std::string& path, const CpdBucket& b)
    : path_(path), tmp_(path + ".tmp"), nrows_((uint32_t)b.targets.size()) {
    fd_ = ::open(tmp_.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd_ < 0) throw Error(CPD_E_IO, "cannot write " + tmp_);
    char h[kBucketHeader] = {};
    std::memcpy(h, kBucketMagic, 8);
    const uint32_t h32[6] = {b.n, nrows_, b.bid, b.method, b.key, b.maxworker};
    std::memcpy(h + 8, h32, sizeof h32);
    std::memcpy(h + 40, &b.fingerprint, 8);  // total (h + 32) is written by close()
    pwrite_all(h, sizeof h, 0);
    pwrite_all(b.targets.data(), nrows_ * 4ull, kBucketHeader);
}

BucketFile::~BucketFile() {
    if (fd_ >= 0) {
        ::close(fd_);
        ::unlink(tmp_.c_str());
    }
}

void BucketFile::pwrite_all(const void* p, size_t bytes, uint64_t pos) {
    const char* c = static_cast<const char*>(p);
    while (bytes > 0) {
        const ssize_t k = ::pwrite(fd_, c, std::min<size_t>(bytes, size_t(1) << 30), (off_t)pos);
        if (k <= 0) throw Error(CPD_E_IO, "write failed: " + tmp_);
        c += k;
        pos += (uint64_t)k;
        bytes -= (size_t)k;
    }
}

void BucketFile::write_offsets(uint32_t first_row, const uint64_t* off, uint32_t count) {
    if (first_row > nrows_ + 1u || count > nrows_ + 1u - first_row)
        throw Error(CPD_E_ARG, "bucket offsets out of range: " + tmp_);
    pwrite_all(off, count * 8ull, kBucketHeader + 4ull * nrows_ + 8ull * first_row);
}

void BucketFile::write_runs(uint64_t first_run, const uint32_t* runs, uint64_t count) {
    pwrite_all(runs, count * 4ull, kBucketHeader + 4ull * nrows_ + 8ull * (nrows_ + 1ull) + 4ull * first_run);
}

void BucketFile::close(uint64_t total) {
    pwrite_all(&total, 8, 32);
    const int fd = fd_;
    fd_ = -1;
    if (::close(fd) != 0) throw Error(CPD_E_IO, "close failed: " + tmp_);
    if (std::rename(tmp_.c_str(), path_.c_str()) != 0) throw Error(CPD_E_IO, "rename failed: " + path_);
}

CpdBucket read_bucket_head(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw Error(CPD_E_IO, "cannot open " + path);
    const uint64_t size = (uint64_t)f.tellg();
    f.seekg(0);
    char magic[8];
    f.read(magic, 8);
    if (!f || std::memcmp(magic, kBucketMagic, 8) != 0) throw Error(CPD_E_IO, path + ": not a CPD bucket file");
    CpdBucket b;
    uint32_t h32[6];
    uint64_t total = 0;
    f.read(reinterpret_cast<char*>(h32), sizeof h32);
    f.read(reinterpret_cast<char*>(&total), 8);
    f.read(reinterpret_cast<char*>(&b.fingerprint), 8);
    if (!f) throw Error(CPD_E_IO, path + ": truncated header");
    b.n = h32[0];
    const uint32_t nrows = h32[1];
    b.bid = h32[2];
    b.method = h32[3];
    b.key = h32[4];
    b.maxworker = h32[5];
    if (size != kBucketHeader + 4ull * nrows + 8ull * (nrows + 1ull) + 4ull * total)
        throw Error(CPD_E_IO, path + ": size does not match its header");
    b.targets.resize(nrows);
    b.offsets.resize((size_t)nrows + 1);
    f.read(reinterpret_cast<char*>(b.targets.data()), nrows * 4ull);
    f.read(reinterpret_cast<char*>(b.offsets.data()), (nrows + 1) * 8ull);
    if (!f) throw Error(CPD_E_IO, path + ": truncated body");
    if (b.offsets[0] != 0 || b.offsets[nrows] != total) throw Error(CPD_E_IO, path + ": bad offsets");
    return b;
}

void read_bucket_runs(const std::string& path, const CpdBucket& head, uint64_t first,
                      uint64_t count, uint32_t* out) {
    const uint64_t nrows = head.targets.size();
    if (first + count > head.offsets.back()) throw Error(CPD_E_ARG, path + ": runs out of range");
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) throw Error(CPD_E_IO, "cannot open " + path);
    uint64_t pos = kBucketHeader + 4ull * nrows + 8ull * (nrows + 1ull) + 4ull * first;
    char* c = reinterpret_cast<char*>(out);
    uint64_t left = 4ull * count;
    while (left) {
        const ssize_t k = ::pread(fd, c, std::min<uint64_t>(left, 1ull << 30), (off_t)pos);
        if (k <= 0) {
            ::close(fd);
            throw Error(CPD_E_IO, path + ": truncated runs");
        }
        c += k;
        pos += (uint64_t)k;
        left -= (uint64_t)k;
    }
    ::close(fd);
}

CpdBucket read_bucket(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error(CPD_E_IO, "cannot open " + path);
    char magic[8];
    f.read(magic, 8);
    if (!f || std::memcmp(magic, kBucketMagic, 8) != 0) throw Error(CPD_E_IO, path + ": not a CPD bucket file");
    CpdBucket b;
    uint32_t h32[6];
    uint64_t total = 0;
    f.read(reinterpret_cast<char*>(h32), sizeof h32);
    f.read(reinterpret_cast<char*>(&total), 8);
    f.read(reinterpret_cast<char*>(&b.fingerprint), 8);
    if (!f) throw Error(CPD_E_IO, path + ": truncated header");
    b.n = h32[0];
    uint32_t nrows = h32[1];
    b.bid = h32[2];
    b.method = h32[3];
    b.key = h32[4];
    b.maxworker = h32[5];
    b.targets.resize(nrows);
    b.offsets.resize((size_t)nrows + 1);
    b.runs.resize(total);
    f.read(reinterpret_cast<char*>(b.targets.data()), nrows * 4ull);
    f.read(reinterpret_cast<char*>(b.offsets.data()), (nrows + 1) * 8ull);
    f.read(reinterpret_cast<char*>(b.runs.data()), total * 4ull);
    if (!f) throw Error(CPD_E_IO, path + ": truncated body");
    if (b.offsets[0] != 0 || b.offsets[nrows] != total) throw Error(CPD_E_IO, path + ": bad offsets");
    return b;
}

int bucket_format(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error(CPD_E_IO, "cannot open " + path);
    char magic[8];
    f.read(magic, 8);
    if (f && std::memcmp(magic, kBucketMagic, 8) == 0) return 1;
    if (f && (std::memcmp(magic, kMoveBucketMagic, 8) == 0 ||
              std::memcmp(magic, kMoveStripedMagic, 8) == 0))
        return 2;
    throw Error(CPD_E_IO, path + ": not a CPD bucket file");
}

// DOSCPD02 layout: magic 8 | 8 x u32 | total u64 | fingerprint u64 (= 56 B) |
// targets | counts | pad | rows from rows_offset().  DOSCPD03: the same 56 B
// + stripes u32 + stripe_rows u32 | targets | counts, and the rows in part
// files {path}.{fingerprint}.p{j}: unit u (rows [u S, u S + S)) is unit u / K
// of part u % K.  The parts carry the graph's fingerprint in their names, so a
// main file only ever pairs with parts built for its graph (a rebuild that
// stops between renaming its parts and its main file leaves the old main file
// with the old parts).
static constexpr uint64_t kMoveHeader = 8 + 32 + 8 + 8;
static constexpr uint64_t kStripedHeader = kMoveHeader + 8;
static constexpr uint64_t kMoveRowsAlign = 4096;

uint64_t MoveBucket::rows_offset() const {
    const uint64_t end = kMoveHeader + 8ull * targets.size();
    return (end + kMoveRowsAlign - 1) / kMoveRowsAlign * kMoveRowsAlign;
}

uint64_t MoveBucket::head_bytes() const { return kStripedHeader + 8ull * targets.size(); }

uint64_t MoveBucket::part_rows(uint32_t j) const {
    const uint64_t nr = targets.size(), S = stripe_rows, K = stripes;
    if (!S || !K) return 0;
    const uint64_t units = (nr + S - 1) / S;
    uint64_t rows = 0;
    if (j < units) {
        const uint64_t mine = (units - 1 - j) / K + 1;  // units j, j + K, ...
        rows = mine * S;
        const uint64_t last = j + (mine - 1) * K;         // a short final unit
        if (last == units - 1) rows -= units * S - nr;
    }
    return rows;
}

std::string move_part_path(const std::string& path, uint64_t fingerprint, uint32_t j) {
    char fp[17];
    std::snprintf(fp, sizeof fp, "%016llx", (unsigned long long)fingerprint);
    return path + "." + fp + ".p" + std::to_string(j);
}

constexpr uint32_t kMaxStripes = 4096;

MoveBucketFile::MoveBucketFile(const std::string& path, const MoveBucket& b, uint32_t stripes,
                               uint32_t stripe_rows)
    : path_(path), tmp_(path + ".tmp"), nrows_((uint32_t)b.targets.size()), words_(b.words),
      stripes_(std::max(1u, stripes)), stripe_rows_(std::max(1u, stripe_rows)), fp_(b.fingerprint) {
    if (!(b.bits == 1 || b.bits == 2 || b.bits == 4) ||
        b.words != ((uint64_t)b.n * b.bits + 31u) / 32u)
        throw Error(CPD_E_ARG, "move bucket: words != ceil(n * bits / 32)");
    if (stripes_ > kMaxStripes)  // what read_move_bucket_head accepts
        throw Error(CPD_E_ARG, "move bucket: at most " + std::to_string(kMaxStripes) + " stripes");
    const bool striped = stripes_ > 1;
    rows_off_ = striped ? 0 : b.rows_offset();
    fd_ = ::open(tmp_.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd_ < 0) throw Error(CPD_E_IO, "cannot write " + tmp_);
    // header, targets, zero counts (and pad)
    const uint64_t head = striped ? kStripedHeader + 8ull * nrows_ : b.rows_offset();
    std::vector<char> h(head, 0);
    std::memcpy(h.data(), striped ? kMoveStripedMagic : kMoveBucketMagic, 8);
    const uint32_t h32[8] = {b.n, nrows_, b.bid, b.method, b.key, b.maxworker, b.words, b.bits};
    std::memcpy(h.data() + 8, h32, sizeof h32);
    std::memcpy(h.data() + 48, &b.fingerprint, 8);  // total (h + 40) is written by close()
    const uint64_t tgt = striped ? kStripedHeader : kMoveHeader;
    if (striped) {
        const uint32_t st[2] = {stripes_, stripe_rows_};
        std::memcpy(h.data() + kMoveHeader, st, sizeof st);
    }
    std::memcpy(h.data() + tgt, b.targets.data(), 4ull * nrows_);
    try {
        pwrite_all(fd_, h.data(), h.size(), 0);
        for (uint32_t j = 0; striped && j < stripes_; ++j) {
            const std::string pt = move_part_path(path_, fp_, j) + ".tmp";
            const int pf = ::open(pt.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
            if (pf < 0) throw Error(CPD_E_IO, "cannot write " + pt);
            part_fd_.push_back(pf);
        }
    } catch (...) {  // the destructor does not run: close and remove what was opened
        discard();
        throw;
    }
}

void MoveBucketFile::discard() {
    for (uint32_t j = 0; j < part_fd_.size(); ++j) {
        if (part_fd_[j] < 0) continue;
        ::close(part_fd_[j]);
        ::unlink((move_part_path(path_, fp_, j) + ".tmp").c_str());
        part_fd_[j] = -1;
    }
    if (fd_ >= 0) {
        ::close(fd_);
        ::unlink(tmp_.c_str());
        fd_ = -1;
    }
}

MoveBucketFile::~MoveBucketFile() { discard(); }

void MoveBucketFile::pwrite_all(int fd, const void* p, size_t bytes, uint64_t pos) {
    const char* c = static_cast<const char*>(p);
    while (bytes > 0) {
        const ssize_t k = ::pwrite(fd, c, std::min<size_t>(bytes, size_t(1) << 30), (off_t)pos);
        if (k <= 0) throw Error(CPD_E_IO, "write failed: " + tmp_);
        c += k;
        pos += (uint64_t)k;
        bytes -= (size_t)k;
    }
}

void MoveBucketFile::write_counts(uint32_t first_row, const uint32_t* counts, uint32_t count) {
    if (first_row > nrows_ || count > nrows_ - first_row)
        throw Error(CPD_E_ARG, "bucket counts out of range: " + tmp_);
    const uint64_t tgt = stripes_ > 1 ? kStripedHeader : kMoveHeader;
    pwrite_all(fd_, counts, 4ull * count, tgt + 4ull * nrows_ + 4ull * first_row);
}

void MoveBucketFile::write_rows(uint32_t first_row, const uint32_t* rows, uint32_t count) {
    if (first_row > nrows_ || count > nrows_ - first_row)
        throw Error(CPD_E_ARG, "bucket rows out of range: " + tmp_);
    const uint64_t rb = 4ull * words_;
    if (stripes_ == 1) {
        pwrite_all(fd_, rows, rb * count, rows_off_ + rb * first_row);
        return;
    }
    const uint64_t S = stripe_rows_, K = stripes_;
    for (uint64_t r = first_row, end = (uint64_t)first_row + count; r < end;) {
        const uint64_t u = r / S, take = std::min(end - r, (u + 1) * S - r);
        const uint64_t at = ((u / K) * S + r % S) * rb;
        pwrite_all(part_fd_[u % K], rows + (r - first_row) * words_, take * rb, at);
        r += take;
    }
}

void MoveBucketFile::close(uint64_t total_runs) {
    pwrite_all(fd_, &total_runs, 8, 40);
    // a bucket file already here from an earlier build: its parts go once the
    // new main file is in place (when they are not the ones just written)
    uint64_t old_fp = 0;
    uint32_t old_k = 0;
    try {
        const MoveBucket old = read_move_bucket_head(path_, false);
        old_fp = old.fingerprint;
        old_k = old.stripes > 1 ? old.stripes : 0;
    } catch (const Error&) {
    }
    for (uint32_t j = 0; j < part_fd_.size(); ++j) {
        const int pf = part_fd_[j];
        part_fd_[j] = -1;
        const std::string pp = move_part_path(path_, fp_, j);
        if (::close(pf) != 0) throw Error(CPD_E_IO, "close failed: " + pp + ".tmp");
        if (std::rename((pp + ".tmp").c_str(), pp.c_str()) != 0) throw Error(CPD_E_IO, "rename failed: " + pp);
    }
    const int fd = fd_;
    fd_ = -1;
    if (::close(fd) != 0) throw Error(CPD_E_IO, "close failed: " + tmp_);
    if (std::rename(tmp_.c_str(), path_.c_str()) != 0) throw Error(CPD_E_IO, "rename failed: " + path_);
    for (uint32_t j = 0; j < old_k; ++j)
        if (old_fp != fp_ || j >= part_fd_.size()) ::unlink(move_part_path(path_, old_fp, j).c_str());
}

MoveBucket read_move_bucket_head(const std::string& path, bool check_parts) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw Error(CPD_E_IO, "cannot open " + path);
    const uint64_t size = (uint64_t)f.tellg();
    f.seekg(0);
    char magic[8];
    f.read(magic, 8);
    const bool striped = f && std::memcmp(magic, kMoveStripedMagic, 8) == 0;
    if (!f || !(striped || std::memcmp(magic, kMoveBucketMagic, 8) == 0))
        throw Error(CPD_E_IO, path + ": not a compact (DOSCPD02/03) CPD bucket file");
    MoveBucket b;
    uint32_t h32[8];
    f.read(reinterpret_cast<char*>(h32), sizeof h32);
    f.read(reinterpret_cast<char*>(&b.total_runs), 8);
    f.read(reinterpret_cast<char*>(&b.fingerprint), 8);
    if (striped) {
        uint32_t st[2];
        f.read(reinterpret_cast<char*>(st), sizeof st);
        b.stripes = st[0];
        b.stripe_rows = st[1];
    }
    if (!f) throw Error(CPD_E_IO, path + ": truncated header");
    b.n = h32[0];
    const uint32_t nrows = h32[1];
    b.bid = h32[2];
    b.method = h32[3];
    b.key = h32[4];
    b.maxworker = h32[5];
    b.words = h32[6];
    b.bits = h32[7];
    if (!(b.bits == 1 || b.bits == 2 || b.bits == 4) ||
        b.words != ((uint64_t)b.n * b.bits + 31u) / 32u)
        throw Error(CPD_E_IO, path + ": row width does not match n and bits per move");
    if (striped && (b.stripes < 2 || b.stripes > kMaxStripes || b.stripe_rows == 0))
        throw Error(CPD_E_IO, path + ": bad stripe layout");
    b.targets.resize(nrows);
    b.counts.resize(nrows);
    if (striped) {
        if (size != b.head_bytes()) throw Error(CPD_E_IO, path + ": size does not match its header");
        for (uint32_t j = 0; check_parts && j < b.stripes; ++j) {
            const std::string pp = move_part_path(path, b.fingerprint, j);
            struct stat st {};
            if (::stat(pp.c_str(), &st) != 0) {
                // round-4 builds named their parts {path}.p{j} (no fingerprint)
                struct stat old {};
                if (::stat((path + ".p" + std::to_string(j)).c_str(), &old) == 0)
                    throw Error(CPD_E_IO, path + ": its part files use the older {bucket}.p{j} "
                                          "names (built by an earlier make_cpd_auto): rebuild it");
                throw Error(CPD_E_IO, "cannot open " + pp);
            }
            if ((uint64_t)st.st_size != b.part_rows(j) * 4ull * b.words)
                throw Error(CPD_E_IO, pp + ": size does not match its bucket");
        }
    } else if (size != b.rows_offset() + 4ull * b.words * nrows) {
        throw Error(CPD_E_IO, path + ": size does not match its header");
    }
    f.read(reinterpret_cast<char*>(b.targets.data()), nrows * 4ull);
    f.read(reinterpret_cast<char*>(b.counts.data()), nrows * 4ull);
    if (!f) throw Error(CPD_E_IO, path + ": truncated body");
    uint64_t tot = 0;
    for (uint32_t c : b.counts) {
        if (c == 0) throw Error(CPD_E_IO, path + ": a row without runs");
        tot += c;
    }
    if (tot != b.total_runs) throw Error(CPD_E_IO, path + ": run counts do not add up");
    return b;
}

void read_move_bucket_rows(const std::string& path, const MoveBucket& head, uint32_t first,
                           uint32_t count, uint32_t* out, int threads) {
    if ((uint64_t)first + count > head.targets.size()) throw Error(CPD_E_ARG, path + ": rows out of range");
    const uint64_t rb = 4ull * head.words;
    // spans (file, file offset, bytes into out, bytes): one per stripe unit
    // touched, or pieces of the one rows region
    struct Span {
        uint32_t file;
        uint64_t pos, at, bytes;
    };
    std::vector<Span> spans;
    std::vector<std::string> files;
    if (head.stripes > 1) {
        for (uint32_t j = 0; j < head.stripes; ++j) files.push_back(move_part_path(path, head.fingerprint, j));
        const uint64_t S = head.stripe_rows, K = head.stripes;
        for (uint64_t r = first, end = (uint64_t)first + count; r < end;) {
            const uint64_t u = r / S, take = std::min(end - r, (u + 1) * S - r);
            spans.push_back({(uint32_t)(u % K), ((u / K) * S + r % S) * rb, (r - first) * rb, take * rb});
            r += take;
        }
    } else {
        files.push_back(path);
        // a read from the page cache is a copy one thread does at ~10 GB/s:
        // large pieces are split over threads (>= 16 MB each)
        const uint64_t total = rb * count, pos0 = head.rows_offset() + rb * first;
        const uint64_t parts = std::max<uint64_t>(
            1, std::min<uint64_t>((uint64_t)std::max(1, threads), total >> 24));
        const uint64_t step = (total / parts + 4095) / 4096 * 4096;
        for (uint64_t a = 0; a < total; a += step) spans.push_back({0, pos0 + a, a, std::min(step, total - a)});
    }
    std::vector<int> fds(files.size(), -1);
    for (size_t i = 0; i < files.size(); ++i) {
        fds[i] = ::open(files[i].c_str(), O_RDONLY | O_CLOEXEC);
        if (fds[i] < 0) {
            for (int fd : fds)
                if (fd >= 0) ::close(fd);
            throw Error(CPD_E_IO, "cannot open " + files[i]);
        }
    }
    auto read_span = [&](const Span& sp) {
        char* c = reinterpret_cast<char*>(out) + sp.at;
        uint64_t pos = sp.pos, left = sp.bytes;
        while (left) {
            const ssize_t k = ::pread(fds[sp.file], c, std::min<uint64_t>(left, 1ull << 30), (off_t)pos);
            if (k <= 0) return false;
            c += k;
            pos += (uint64_t)k;
            left -= (uint64_t)k;
        }
        return true;
    };
    const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), spans.size()));
    bool ok = true;
    if (T == 1) {
        for (const Span& sp : spans) ok = ok && read_span(sp);
    } else {
        std::vector<std::thread> th;
        std::vector<char> good(T, 1);
        for (size_t t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (size_t i = t; i < spans.size(); i += T) good[t] = good[t] && read_span(spans[i]);
            });
        for (auto& x : th) x.join();
        for (char g : good) ok = ok && g;
    }
    for (int fd : fds) ::close(fd);
    if (!ok) throw Error(CPD_E_IO, path + ": truncated rows");
}

void write_order(const std::string& path, uint64_t fp, const std::vector<uint32_t>& order) {
    std::string tmp = path + ".tmp." + std::to_string(::getpid());
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) throw Error(CPD_E_IO, "cannot write " + tmp);
        uint32_t n = (uint32_t)order.size();
        f.write(kOrderMagic, 8);
        f.write(reinterpret_cast<const char*>(&n), 4);
        f.write(reinterpret_cast<const char*>(&fp), 8);
        f.write(reinterpret_cast<const char*>(order.data()), n * 4ull);
        if (!f) throw Error(CPD_E_IO, "write failed: " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw Error(CPD_E_IO, "rename failed: " + path);
}

uint32_t read_order_n(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error(CPD_E_IO, "cannot open " + path);
    char magic[8];
    uint32_t n = 0;
    f.read(magic, 8);
    f.read(reinterpret_cast<char*>(&n), 4);
    if (!f || std::memcmp(magic, kOrderMagic, 8) != 0) throw Error(CPD_E_IO, path + ": not an order file");
    return n;
}

std::vector<uint32_t> read_order(const std::string& path, uint64_t fp) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error(CPD_E_IO, "cannot open " + path);
    char magic[8];
    uint32_t n = 0;
    uint64_t got = 0;
    f.read(magic, 8);
    f.read(reinterpret_cast<char*>(&n), 4);
    f.read(reinterpret_cast<char*>(&got), 8);
    if (!f || std::memcmp(magic, kOrderMagic, 8) != 0) throw Error(CPD_E_IO, path + ": not an order file");
    if (got != fp) throw Error(CPD_E_IO, path + ": built for a different graph");
    std::vector<uint32_t> order(n);
    f.read(reinterpret_cast<char*>(order.data()), n * 4ull);
    if (!f) throw Error(CPD_E_IO, path + ": truncated");
    return order;
}

}  // namespace io
}  // namespace cpd

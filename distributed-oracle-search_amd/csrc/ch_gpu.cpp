// Contraction hierarchy built on the GPU (kernels: ch_kernels.hip).
//
// The same parallel independent-set contraction as ch.cpp — same priority
// (8 x edge difference + 2 x contracted neighbours + 12 x depth, ties by a
// hash of the node id), same independent set, same bounded witness searches
// (settle limits, via bounds, heap order), same lightest-arc shortcut merges
// — so the hierarchy is the host's, rank for rank and arc for arc
// (tests/test_ch_gpu.py compares them).  Only where the work runs changes:
// a round's witness searches (one lane each, ~10M over a 1M-node build), the
// independent-set test, the list updates and the priority updates are
// kernels over the overlay graph resident in HBM; the host only sizes the
// next launch from a few counters per round.
//
// Overlay graph in HBM: an arena of (neighbour, weight) arcs, per node the
// offset and degree of its out- and in-list; a node whose lists change gets
// fresh space at the arena top (bump allocation, compacted when full).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "ch_kernels.hpp"
#include "cpd_internal.hpp"

namespace cpd {
namespace {

#define CH_HIP(expr)                                                                  \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess)                                                         \
            throw ::cpd::Error(_e == hipErrorOutOfMemory ? CPD_E_OOM : CPD_E_HIP,     \
                               std::string("ch_gpu: ") + #expr + ": " +               \
                                   hipGetErrorString(_e));                            \
    } while (0)

// Device buffer of T; ensure() discards the contents, grow() keeps them.
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void ensure(size_t k) {
        if (k <= n && p) return;
        release();
        CH_HIP(hipMalloc(&p, std::max<size_t>(k, 1) * sizeof(T)));
        n = k;
    }
    void grow(size_t k, hipStream_t s) {
        if (k <= n && p) return;
        const size_t want = std::max(k, n + n / 2);
        T* q = nullptr;
        CH_HIP(hipMalloc(&q, std::max<size_t>(want, 1) * sizeof(T)));
        if (p && n) CH_HIP(hipMemcpyAsync(q, p, n * sizeof(T), hipMemcpyDeviceToDevice, s));
        CH_HIP(hipStreamSynchronize(s));
        release();
        p = q;
        n = want;
    }
};

struct Stream {
    hipStream_t s = nullptr;
    ~Stream() {
        if (s) (void)hipStreamDestroy(s);
    }
};

struct PinnedWords {
    uint32_t* p = nullptr;
    ~PinnedWords() {
        if (p) (void)hipHostFree(p);
    }
};

}  // namespace

Hierarchy build_hierarchy_gpu(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                              const uint32_t* w, int device, uint32_t settle_limit, int verbose) {
    CPD_REQUIRE(n < 0x80000000u, CPD_E_ARG, "GPU contraction: node ids must be below 2^31");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        throw Error(CPD_E_HIP, "GPU contraction: no GPU visible");
    CPD_REQUIRE(device >= 0 && device < ndev, CPD_E_ARG, "GPU contraction: bad device");
    CH_HIP(hipSetDevice(device));
    const double t0 = now_seconds();
    const uint32_t settle_c = settle_limit ? settle_limit : 400;
    const uint32_t settle_s = std::max<uint32_t>(50, settle_c / 4);
    int64_t pa = 8, pb = 2, pc = 12;  // ch.cpp Contractor::prio_* (CPD_CH_PRIO as there)
    if (const char* e = std::getenv("CPD_CH_PRIO")) {
        long a, b, c;
        if (std::sscanf(e, "%ld,%ld,%ld", &a, &b, &c) == 3) {
            pa = a;
            pb = b;
            pc = c;
        }
    }

    // Initial overlay (ch.cpp: no self loops, parallel edges reduced to the
    // lightest, lists sorted by neighbour id): out-lists at [0, M), in-lists
    // at [M, 2M) of the arena.
    std::vector<uint32_t> odeg(n), ooff(n + 1), ideg(n, 0), ioff(n + 1);
    std::vector<uint32_t> tmp(2ull * row_ptr[n]);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t vi = 0; vi < (int64_t)n; ++vi) {
        const uint32_t v = (uint32_t)vi;
        uint32_t* t = tmp.data() + 2ull * row_ptr[v];
        uint32_t k = 0;
        for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
            if (dst[e] != v) {
                t[2 * k] = dst[e];
                t[2 * k + 1] = w[e];
                ++k;
            }
        auto* pr = reinterpret_cast<std::pair<uint32_t, uint32_t>*>(t);
        std::sort(pr, pr + k);  // by (neighbour, weight)
        uint32_t u = 0;
        for (uint32_t j = 0; j < k; ++j)
            if (u == 0 || pr[u - 1].first != pr[j].first) pr[u++] = pr[j];
        odeg[v] = u;
    }
    ooff[0] = 0;
    for (uint32_t v = 0; v < n; ++v) ooff[v + 1] = ooff[v] + odeg[v];
    const uint32_t M = ooff[n];
    std::vector<uint32_t> arena0(4ull * M);
    for (uint32_t v = 0; v < n; ++v) {
        const uint32_t* t = tmp.data() + 2ull * row_ptr[v];
        std::memcpy(arena0.data() + 2ull * ooff[v], t, 8ull * odeg[v]);
        for (uint32_t j = 0; j < odeg[v]; ++j) ++ideg[t[2 * j]];
    }
    ioff[0] = M;
    for (uint32_t v = 0; v < n; ++v) ioff[v + 1] = ioff[v] + ideg[v];
    {
        std::vector<uint32_t> cur(ioff.begin(), ioff.end() - 1);
        for (uint32_t v = 0; v < n; ++v)  // tails ascending: in-lists come out sorted
            for (uint32_t j = 0; j < odeg[v]; ++j) {
                const uint32_t x = arena0[2ull * (ooff[v] + j)];
                const uint32_t p = cur[x]++;
                arena0[2ull * p] = v;
                arena0[2ull * p + 1] = arena0[2ull * (ooff[v] + j) + 1];
            }
    }
    std::vector<uint32_t>().swap(tmp);
    uint32_t maxdeg0 = 0;
    for (uint32_t v = 0; v < n; ++v) maxdeg0 = std::max({maxdeg0, odeg[v], ideg[v]});

    Stream S_;
    CH_HIP(hipStreamCreateWithFlags(&S_.s, hipStreamNonBlocking));
    hipStream_t st = S_.s;
    PinnedWords hv;
    CH_HIP(hipHostMalloc(reinterpret_cast<void**>(&hv.p), 64 * sizeof(uint32_t), hipHostMallocDefault));

    // arena offsets are 32-bit (the merge kernel takes them as u32)
    CPD_REQUIRE(2ull * M < (1ull << 32), CPD_E_RANGE, "GPU contraction: graph has >= 2^31 arcs");
    size_t arena_cap = std::min<size_t>(std::max<size_t>(16ull * M, 1u << 22),
                                        (1ull << 32) - 1);  // arcs
    DBuf<uint32_t> arena, arena2;
    arena.ensure(2 * arena_cap);
    CH_HIP(hipMemcpyAsync(arena.p, arena0.data(), arena0.size() * 4, hipMemcpyHostToDevice, st));
    uint64_t top = 2ull * M;  // arcs used
    DBuf<uint32_t> d_ooff, d_odeg, d_ioff, d_ideg;
    d_ooff.ensure(n);
    d_odeg.ensure(n);
    d_ioff.ensure(n);
    d_ideg.ensure(n);
    CH_HIP(hipMemcpyAsync(d_ooff.p, ooff.data(), 4ull * n, hipMemcpyHostToDevice, st));
    CH_HIP(hipMemcpyAsync(d_odeg.p, odeg.data(), 4ull * n, hipMemcpyHostToDevice, st));
    CH_HIP(hipMemcpyAsync(d_ioff.p, ioff.data(), 4ull * n, hipMemcpyHostToDevice, st));
    CH_HIP(hipMemcpyAsync(d_ideg.p, ideg.data(), 4ull * n, hipMemcpyHostToDevice, st));

    DBuf<int64_t> prio;
    DBuf<uint32_t> deleted, depth, aff, cnt_o, cnt_i, cur_o, cur_i, bo_o, bo_i, sc, rank;
    DBuf<uint8_t> state;
    prio.ensure(n);
    for (DBuf<uint32_t>* b : {&deleted, &depth, &aff, &cnt_o, &cnt_i, &cur_o, &cur_i, &bo_o,
                              &bo_i, &sc, &rank}) {
        b->ensure(n);
        CH_HIP(hipMemsetAsync(b->p, 0, 4ull * n, st));
    }
    state.ensure(n);
    CH_HIP(hipMemsetAsync(state.p, 0, n, st));
    DBuf<uint32_t> rem, rem2, Sl, Al, junk, flag, pos, c[4], s[4];
    for (DBuf<uint32_t>* b : {&rem, &rem2, &Sl, &Al, &junk}) b->ensure(n + 1);
    for (DBuf<uint32_t>* b : {&flag, &pos, &c[0], &c[1], &c[2], &c[3], &s[0], &s[1], &s[2], &s[3]})
        b->ensure(n + 1);
    DBuf<uint32_t> rec_v, rec_un, rec_dn;
    DBuf<uint64_t> rec_uo, rec_do;
    rec_v.ensure(n);
    rec_un.ensure(n);
    rec_dn.ensure(n);
    rec_uo.ensure(n);
    rec_do.ensure(n);
    DBuf<uint32_t> upool, dpool, pairs, slots, sflag, spos, sclist, bk_o, bk_i, ovf, ovf2, ctr;
    upool.ensure(2ull * std::max<size_t>(M, 1024) * 2);
    dpool.ensure(2ull * std::max<size_t>(M, 1024) * 2);
    ctr.ensure(8);
    CH_HIP(hipMemsetAsync(ctr.p, 0, 32, st));
    CH_HIP(hipMemcpyAsync(ctr.p + 2, &maxdeg0, 4, hipMemcpyHostToDevice, st));
    {
        std::vector<uint32_t> iota(n);
        std::iota(iota.begin(), iota.end(), 0u);
        CH_HIP(hipMemcpyAsync(rem.p, iota.data(), 4ull * n, hipMemcpyHostToDevice, st));
        CH_HIP(hipMemcpyAsync(Al.p, iota.data(), 4ull * n, hipMemcpyHostToDevice, st));
        CH_HIP(hipStreamSynchronize(st));
    }
    DBuf<uint8_t> scan_tmp;
    auto scan = [&](const uint32_t* in, uint32_t* out, uint32_t cnt) {
        size_t b = 0;
        chk::scan_u32(nullptr, &b, in, out, cnt, st);
        scan_tmp.ensure(b);
        b = scan_tmp.n;
        chk::scan_u32(scan_tmp.p, &b, in, out, cnt, st);
    };
    // read k device words (each at its own address) with one sync
    auto read = [&](std::initializer_list<const uint32_t*> ptrs) {
        uint32_t i = 0;
        for (const uint32_t* q : ptrs)
            CH_HIP(hipMemcpyAsync(hv.p + i++, q, 4, hipMemcpyDeviceToHost, st));
        CH_HIP(hipStreamSynchronize(st));
    };

    // Witness lane workspaces: a small one for every search, a large one (sized
    // from the largest degree, so that nothing can overflow it) for the rare
    // search that outgrows the first.
    chk::WitnessCaps caps1{1024, 512, 32};
    if (const char* e = std::getenv("CPD_CH_WS")) {  // test knob: "hash,heap,targets"
        unsigned a = 0, b = 0, c = 0;
        if (std::sscanf(e, "%u,%u,%u", &a, &b, &c) == 3 && a >= 2 && !(a & (a - 1)) && b && c)
            caps1 = {a, b, c};
    }
    const uint64_t lb1 = chk::witness_lane_bytes(caps1);
    // lanes: up to 262144 (4096 waves: 6.4 GB of workspaces), fewer for small
    // graphs (a round has at most ~4n searches)
    uint64_t lane_max = 262144;  // CPD_CH_LANES (1M: 65536 / 131072 / 262144 lanes: 1.30 / 1.20 / 1.18 s)
    if (const char* e = std::getenv("CPD_CH_LANES")) lane_max = std::max(256ul, std::strtoul(e, nullptr, 10));
    const uint32_t lanes1 =
        (uint32_t)std::min<uint64_t>(lane_max, std::max<uint64_t>(256, (4ull * n + 255) / 256 * 256));
    DBuf<uint8_t> ws1, ws2;
    ws1.ensure(lb1 * lanes1);
    CH_HIP(hipMemsetAsync(ws1.p, 0, ws1.n, st));
    uint32_t tag1 = 0, tag2 = 0;
    uint64_t searches = 0, big_searches = 0;

    auto overlay = [&]() {
        return chk::Overlay{d_ooff.p, d_odeg.p, d_ioff.p, d_ideg.p, arena.p};
    };
    // Searches go to the lane kernel (many small ones: the early rounds), or
    // straight to the wave kernel when a round has few (the core rounds:
    // large searches); what outgrows a workspace moves on: lane -> wave ->
    // the large HBM workspace, which cannot overflow.
    uint32_t wave_max = 65536, wave_blocks = 8192;
    // the 13-KB stage for simulation searches (1M: 1.15 against 1.26 s);
    // CPD_CH_TINY=0 skips it (A/B)
    const bool tiny_on = !(std::getenv("CPD_CH_TINY") && *std::getenv("CPD_CH_TINY") == '0');
    if (const char* e = std::getenv("CPD_CH_WAVE")) wave_max = (uint32_t)std::strtoul(e, nullptr, 10);
    // test knob: no wave stage (lane -> large workspace only)
    const bool no_wave = std::getenv("CPD_CH_NOWAVE") != nullptr;
    if (no_wave) wave_max = 0;
    // pops + relaxations a lane search may take before a wave takes it over
    // (A/B at 1M nodes: 512 -> 2.6 s, 2048 -> 2.4 s, none -> 2.1 s: default none)
    uint32_t lane_cap = 0xFFFFFFFFu;
    if (const char* e = std::getenv("CPD_CH_LANE_CAP")) lane_cap = (uint32_t)std::strtoul(e, nullptr, 10);
    uint64_t wave_searches = 0;
    double t_lane = 0, t_wave = 0, t_big = 0;  // witness kernel wall times (verbose)
    DBuf<uint32_t> ovf3;
    auto witness = [&](uint32_t np, bool contract, uint32_t settle) {
        if (!np) return;
        ovf.ensure(np);
        CH_HIP(hipMemsetAsync(ctr.p, 0, 8, st));  // ovf_n, err
        const uint32_t* list = nullptr;
        uint32_t cnt = np;
        searches += np;
        double tw = now_seconds();
        if (np > wave_max) {
            if ((uint64_t)tag1 + np + 1 >= (1ull << 32)) {  // tags would wrap: clear the tables
                CH_HIP(hipMemsetAsync(ws1.p, 0, ws1.n, st));
                tag1 = 0;
            }
            chk::launch_witness(pairs.p, nullptr, np, overlay(), state.p, contract, settle, ws1.p,
                                caps1, lanes1, tag1, no_wave ? 0xFFFFFFFFu : lane_cap, slots.p,
                                sflag.p, sc.p, ovf.p, ctr.p, ctr.p + 1, st);
            tag1 += np + 1;
            read({ctr.p});
            cnt = hv.p[0];
            list = ovf.p;
            t_lane += now_seconds() - tw;
            tw = now_seconds();
        }
        // waves: LDS workspaces of 13 KB (simulations only, twelve
        // workgroups per CU), 27 KB (five) and 55 KB (two), each taking
        // what outgrew the one before
        const int first = tiny_on && !contract ? 0 : 1;
        for (int size = first; size < 3 && cnt && !no_wave; ++size) {
            DBuf<uint32_t>& out = size == first ? ovf2 : (list == ovf2.p ? ovf3 : ovf2);
            out.ensure(cnt);
            CH_HIP(hipMemsetAsync(ctr.p + 4, 0, 4, st));
            chk::launch_witness_wave(pairs.p, list, cnt, overlay(), state.p, contract, settle,
                                     wave_blocks, size, slots.p, sflag.p, sc.p, out.p, ctr.p + 4,
                                     ctr.p + 1, st);
            wave_searches += cnt;
            read({ctr.p + 4});
            cnt = hv.p[0];
            list = out.p;
            t_wave += now_seconds() - tw;
            tw = now_seconds();
        }
        read({ctr.p + 1, ctr.p + 2});
        const uint32_t err = hv.p[0], maxdeg = hv.p[1];
        CPD_REQUIRE(!err, CPD_E_RANGE, "shortcut weight >= 2^32-1");
        if (!cnt) return;
        const uint32_t novf = cnt;
        big_searches += novf;
        // pushes <= 1 + settle x maxdeg, touched nodes <= that + targets
        const uint64_t heap = 1ull + (uint64_t)settle * maxdeg;
        uint64_t hash = 1;
        while (hash * 3 < (heap + maxdeg + 2) * 4) hash <<= 1;
        CPD_REQUIRE(hash < (1ull << 31) && heap < (1ull << 31), CPD_E_RANGE,
                    "GPU contraction: witness workspace too large");
        const chk::WitnessCaps caps2{(uint32_t)hash, (uint32_t)heap, std::max(maxdeg, 1u)};
        const uint64_t lb2 = chk::witness_lane_bytes(caps2);
        // as many lanes as searches (whole waves), at most what 8 GB holds;
        // the kernel strides over the searches when there are fewer lanes
        const uint64_t budget = 8ull << 30;
        const uint32_t lanes2 =
            (uint32_t)std::max<uint64_t>(64, std::min<uint64_t>((novf + 63) / 64 * 64,
                                                                budget / lb2 / 64 * 64));
        if (ws2.n < lb2 * lanes2 || (uint64_t)tag2 + novf + 1 >= (1ull << 32)) {
            ws2.ensure(lb2 * lanes2);
            CH_HIP(hipMemsetAsync(ws2.p, 0, ws2.n, st));
            tag2 = 0;
        }
        DBuf<uint32_t>& lost = list == ovf.p ? ovf2 : ovf;  // not the list being read
        lost.ensure(novf);
        CH_HIP(hipMemsetAsync(ctr.p + 3, 0, 4, st));
        chk::launch_witness(pairs.p, list, novf, overlay(), state.p, contract, settle, ws2.p,
                            caps2, lanes2, tag2, 0xFFFFFFFFu, slots.p, sflag.p, sc.p, lost.p,
                            ctr.p + 3, ctr.p + 1, st);
        tag2 += novf + 1;
        read({ctr.p + 3, ctr.p + 1});
        CPD_REQUIRE(!hv.p[0], CPD_E_HIP, "GPU contraction: witness workspace overflow");
        CPD_REQUIRE(!hv.p[1], CPD_E_RANGE, "shortcut weight >= 2^32-1");
        t_big += now_seconds() - tw;
    };
    // priorities of list[0..k) (ch.cpp Contractor::priority / step 6)
    uint32_t last_sim = 0;  // simulation searches of the last priorities() (verbose)
    auto priorities = [&](const uint32_t* list, uint32_t k) {
        last_sim = 0;
        if (!k) return;
        chk::launch_sim_counts(list, k, overlay(), c[0].p, sc.p, st);
        scan(c[0].p, s[0].p, k + 1);
        read({s[0].p + k});
        const uint32_t np = hv.p[0];
        last_sim = np;
        pairs.ensure(4ull * std::max(np, 1u));
        chk::launch_make_pairs(list, k, overlay(), s[0].p, nullptr, pairs.p, st);
        witness(np, false, settle_s);
        chk::launch_prio(list, k, overlay(), sc.p, deleted.p, depth.p, pa, pb, pc, prio.p, aff.p,
                         cnt_o.p, cnt_i.p, cur_o.p, cur_i.p, st);
    };

    const double t_init = now_seconds();
    priorities(Al.p, n);
    const double t_prio0 = now_seconds();

    uint32_t R = n, rank0 = 0, round = 0;
    uint64_t utop = 0, dtop = 0;
    double tph[5] = {0, 0, 0, 0, 0};  // pick, contract, record, lists, priorities (verbose)
    double ta = now_seconds();
    auto phase = [&](int k) {
        const double tb = now_seconds();
        tph[k] += tb - ta;
        ta = tb;
    };
    double t_round = now_seconds();
    while (R) {
        // 1. independent set of local priority minima
        chk::launch_pick(rem.p, R, overlay(), prio.p, flag.p, st);
        scan(flag.p, pos.p, R + 1);
        read({pos.p + R});
        const uint32_t nS = hv.p[0];
        CPD_REQUIRE(nS > 0, CPD_E_HIP, "GPU contraction: empty independent set");
        chk::launch_split(rem.p, flag.p, pos.p, R, Sl.p, rem2.p, st);
        const uint32_t nR = R - nS;
        phase(0);
        // 2. witness searches for every (selected node, in-neighbour)
        chk::launch_sel_counts(Sl.p, nS, overlay(), state.p, c[0].p, c[1].p, c[2].p, c[3].p, st);
        for (int k = 0; k < 4; ++k) scan(c[k].p, s[k].p, nS + 1);
        read({s[0].p + nS, s[1].p + nS, s[2].p + nS, s[3].p + nS});
        const uint32_t np = hv.p[0], nq = hv.p[1], nout = hv.p[2], nin = hv.p[3];
        pairs.ensure(4ull * std::max(np, 1u));
        slots.ensure(4ull * std::max(nq, 1u));
        sflag.ensure(nq + 1ull);
        spos.ensure(nq + 1ull);
        chk::launch_make_pairs(Sl.p, nS, overlay(), s[0].p, s[1].p, pairs.p, st);
        if (nq) CH_HIP(hipMemsetAsync(sflag.p, 0, 4ull * nq, st));
        CH_HIP(hipMemsetAsync(sflag.p + nq, 0, 4, st));
        witness(np, true, settle_c);
        phase(1);
        // 3. record ranks and hierarchy arcs; 4. neighbours' counters
        upool.grow(2 * (utop + nout), st);
        dpool.grow(2 * (dtop + nin), st);
        chk::launch_record(Sl.p, nS, rank0, overlay(), s[2].p, s[3].p, utop, dtop, rank.p, rec_v.p,
                           rec_uo.p, rec_un.p, rec_do.p, rec_dn.p, upool.p, dpool.p, deleted.p,
                           depth.p, aff.p, state.p, st);
        utop += nout;
        dtop += nin;
        // 5. shortcuts into the lists of the affected nodes
        scan(sflag.p, spos.p, nq + 1);
        read({spos.p + nq});
        phase(2);
        const uint32_t K = hv.p[0];
        sclist.ensure(4ull * std::max(K, 1u));
        chk::launch_compact_shortcuts(slots.p, sflag.p, spos.p, nq, sclist.p, cnt_o.p, cnt_i.p,
                                      aff.p, st);
        chk::launch_gather_flag(rem2.p, nR, aff.p, flag.p, st);
        scan(flag.p, pos.p, nR + 1);
        read({pos.p + nR});
        const uint32_t nA = hv.p[0];
        chk::launch_split(rem2.p, flag.p, pos.p, nR, Al.p, junk.p, st);
        chk::launch_aff_counts(Al.p, nA, overlay(), cnt_o.p, cnt_i.p, c[0].p, c[1].p, c[2].p,
                               c[3].p, st);
        for (int k = 0; k < 4; ++k) scan(c[k].p, s[k].p, nA + 1);
        read({s[0].p + nA, s[1].p + nA});
        const uint32_t to = hv.p[0], ti = hv.p[1];
        if (top + to + ti > arena_cap) {  // compact every remaining node's lists
            DBuf<uint32_t> e0, e1, f0, f1;
            e0.ensure(nR + 1ull);
            e1.ensure(nR + 1ull);
            f0.ensure(nR + 1ull);
            f1.ensure(nR + 1ull);
            chk::launch_deg_counts(rem2.p, nR, overlay(), e0.p, e1.p, st);
            scan(e0.p, f0.p, nR + 1);
            scan(e1.p, f1.p, nR + 1);
            read({f0.p + nR, f1.p + nR});
            const uint64_t used = (uint64_t)hv.p[0] + hv.p[1];
            const size_t cap2 = std::max<size_t>(arena_cap, 2 * (used + to + ti));
            CPD_REQUIRE(cap2 < (1ull << 32), CPD_E_RANGE, "GPU contraction: overlay too large");
            arena2.ensure(2 * cap2);
            chk::launch_compact_lists(rem2.p, nR, d_ooff.p, d_odeg.p, d_ioff.p, d_ideg.p, arena.p,
                                      arena2.p, f0.p, f1.p, hv.p[0], st);
            CH_HIP(hipStreamSynchronize(st));
            std::swap(arena.p, arena2.p);
            std::swap(arena.n, arena2.n);
            arena2.release();
            arena_cap = cap2;
            top = used;
        }
        chk::launch_bucket_starts(Al.p, nA, s[2].p, s[3].p, bo_o.p, bo_i.p, st);
        bk_o.ensure(2ull * std::max(K, 1u));
        bk_i.ensure(2ull * std::max(K, 1u));
        chk::launch_fill_buckets(sclist.p, K, bo_o.p, bo_i.p, cur_o.p, cur_i.p, bk_o.p, bk_i.p, st);
        CPD_REQUIRE(top + to + ti < (1ull << 32), CPD_E_RANGE, "GPU contraction: overlay too large");
        chk::launch_merge(Al.p, nA, d_ooff.p, d_odeg.p, d_ioff.p, d_ideg.p, arena.p, state.p,
                          s[0].p, s[1].p, (uint32_t)top, (uint32_t)(top + to), bo_o.p, bo_i.p,
                          cnt_o.p, cnt_i.p, bk_o.p, bk_i.p, ctr.p + 2, st);
        top += to + ti;
        phase(3);
        // 6. priorities of the affected nodes
        priorities(Al.p, nA);
        CH_HIP(hipStreamSynchronize(st));
        phase(4);
        std::swap(rem.p, rem2.p);
        std::swap(rem.n, rem2.n);
        R = nR;
        rank0 += nS;
        ++round;
        if (verbose > 1 || (verbose && (round % 10 == 0 || R == 0)))
            std::fprintf(stderr,
                         "[ch-gpu] round %u contracted %u remaining %u shortcuts %u affected %u "
                         "searches %u + %u, %.2f ms (%.2fs)\n",
                         round, nS, R, K, nA, np, last_sim, (now_seconds() - t_round) * 1e3,
                         now_seconds() - t0);
        t_round = now_seconds();
    }

    // Download the records and assemble the CSRs as ch.cpp does.
    std::vector<uint32_t> h_rank(n), h_rec_v(n), h_un(n), h_dn(n);
    std::vector<uint64_t> h_uo(n), h_do(n);
    std::vector<uint32_t> h_up(2 * utop), h_dp(2 * dtop);
    CH_HIP(hipMemcpyAsync(h_rank.data(), rank.p, 4ull * n, hipMemcpyDeviceToHost, st));
    CH_HIP(hipMemcpyAsync(h_un.data(), rec_un.p, 4ull * n, hipMemcpyDeviceToHost, st));
    CH_HIP(hipMemcpyAsync(h_dn.data(), rec_dn.p, 4ull * n, hipMemcpyDeviceToHost, st));
    CH_HIP(hipMemcpyAsync(h_uo.data(), rec_uo.p, 8ull * n, hipMemcpyDeviceToHost, st));
    CH_HIP(hipMemcpyAsync(h_do.data(), rec_do.p, 8ull * n, hipMemcpyDeviceToHost, st));
    CH_HIP(hipMemcpyAsync(h_rec_v.data(), rec_v.p, 4ull * n, hipMemcpyDeviceToHost, st));
    if (utop) CH_HIP(hipMemcpyAsync(h_up.data(), upool.p, 8ull * utop, hipMemcpyDeviceToHost, st));
    if (dtop) CH_HIP(hipMemcpyAsync(h_dp.data(), dpool.p, 8ull * dtop, hipMemcpyDeviceToHost, st));
    CH_HIP(hipStreamSynchronize(st));
    const double t_dev = now_seconds();

    Hierarchy H;
    H.rank = std::move(h_rank);
    H.up_off.assign(n + 1, 0);
    for (uint32_t v = 0; v < n; ++v) H.up_off[v + 1] = H.up_off[v] + h_un[H.rank[v]];
    H.up_dst.resize(H.up_off[n]);
    H.up_w.resize(H.up_off[n]);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t vi = 0; vi < (int64_t)n; ++vi) {
        const uint32_t v = (uint32_t)vi, r = H.rank[v];
        for (uint32_t k = 0; k < h_un[r]; ++k) {
            H.up_dst[H.up_off[v] + k] = h_up[2 * (h_uo[r] + k)];
            H.up_w[H.up_off[v] + k] = h_up[2 * (h_uo[r] + k) + 1];
        }
    }
    // down arcs u -> v (v contracted, u an in-neighbour), sorted (u, v, w)
    H.dn_off.assign(n + 1, 0);
    for (uint32_t r = 0; r < n; ++r)
        for (uint32_t k = 0; k < h_dn[r]; ++k) ++H.dn_off[h_dp[2 * (h_do[r] + k)] + 1];
    for (uint32_t v = 0; v < n; ++v) H.dn_off[v + 1] += H.dn_off[v];
    H.dn_dst.resize(H.dn_off[n]);
    H.dn_w.resize(H.dn_off[n]);
    {
        std::vector<uint64_t> cur(H.dn_off.begin(), H.dn_off.end() - 1);
        for (uint32_t r = 0; r < n; ++r) {
            const uint32_t v = h_rec_v[r];
            for (uint32_t k = 0; k < h_dn[r]; ++k) {
                const uint32_t u = h_dp[2 * (h_do[r] + k)];
                const uint64_t p = cur[u]++;
                H.dn_dst[p] = v;
                H.dn_w[p] = h_dp[2 * (h_do[r] + k) + 1];
            }
        }
    }
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t ui = 0; ui < (int64_t)n; ++ui) {
        const uint64_t a = H.dn_off[ui], b = H.dn_off[ui + 1];
        if (b - a < 2) continue;
        std::vector<std::pair<uint32_t, uint32_t>> t(b - a);
        for (uint64_t e = a; e < b; ++e) t[e - a] = {H.dn_dst[e], H.dn_w[e]};
        std::sort(t.begin(), t.end());
        for (uint64_t e = a; e < b; ++e) {
            H.dn_dst[e] = t[e - a].first;
            H.dn_w[e] = t[e - a].second;
        }
    }
    hierarchy_levels(H, n);
    if (verbose)
        std::fprintf(stderr,
                     "[ch-gpu] %u rounds, %llu witness searches (%llu by waves, %llu in the large "
                     "workspace), "
                     "up arcs %llu, down arcs %llu, levels up %u down %u; setup %.2fs, initial "
                     "priorities %.2fs, rounds %.2fs (pick %.2f contract %.2f record %.2f lists "
                     "%.2f priorities %.2f; witness kernels: lane %.2f wave %.2f large %.2f), "
                     "assembly %.2fs\n",
                     round, (unsigned long long)searches, (unsigned long long)wave_searches,
                     (unsigned long long)big_searches,
                     (unsigned long long)H.up_off[n], (unsigned long long)H.dn_off[n], H.nlev_up,
                     H.nlev_dn, t_init - t0, t_prio0 - t_init, t_dev - t_prio0, tph[0], tph[1],
                     tph[2], tph[3], tph[4], t_lane, t_wave, t_big, now_seconds() - t_dev);
    return H;
}

}  // namespace cpd

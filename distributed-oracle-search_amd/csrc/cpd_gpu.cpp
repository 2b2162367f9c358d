// GPU half of the C ABI: graph upload, batched CPD row build, table-search
// index, per-kernel timing.  All device work runs on one non-blocking HIP
// stream per graph; every entry point selects the graph's device first.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <cmath>
#include <cstring>
#include <thread>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <type_traits>
#include <vector>

#include "cpd_internal.hpp"
#include "cpd_kernels.hpp"

using namespace cpd;

#define HIP_CHECK(expr)                                                          \
    do {                                                                         \
        hipError_t _e = (expr);                                                  \
        if (_e != hipSuccess)                                                    \
            throw ::cpd::Error(_e == hipErrorOutOfMemory ? CPD_E_OOM : CPD_E_HIP, \
                               std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

namespace {

// Per-device HBM arena (cpd_device_arena): one block committed up front —
// e.g. on a host thread while the plan is being contracted — that the
// long-lived bulk buffers on that device are carved from (bump allocation:
// a carved buffer is never returned to it, the whole block is freed by
// cpd_device_arena_release).  Only allocations inside an ArenaScope are
// carved — a build's batch buffers, its row sets, an index's move tables —
// so short-lived scratch never fills it; what does not fit
// falls back to hipMalloc.  `live` counts the carved buffers still held:
// the release refuses while any is.
struct Arena {
    char* base = nullptr;
    size_t cap = 0, top = 0;
    size_t live = 0;
};
std::mutex g_arena_mu;
std::map<int, Arena> g_arena;
thread_local int t_arena_scope = 0;

struct ArenaScope {
    ArenaScope() { ++t_arena_scope; }
    ~ArenaScope() { --t_arena_scope; }
    ArenaScope(const ArenaScope&) = delete;
    ArenaScope& operator=(const ArenaScope&) = delete;
};

void* arena_take(size_t bytes) {
    if (t_arena_scope <= 0) return nullptr;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> l(g_arena_mu);
    auto it = g_arena.find(d);
    if (it == g_arena.end() || !it->second.base) return nullptr;
    Arena& a = it->second;
    const size_t at = (a.top + 255u) & ~(size_t)255u;
    if (at + bytes > a.cap) return nullptr;
    a.top = at + bytes;
    ++a.live;
    return a.base + at;
}

// true (and one live buffer fewer) when p was carved from an arena
bool arena_drop(const void* p) {
    std::lock_guard<std::mutex> l(g_arena_mu);
    for (auto& kv : g_arena) {
        const char* c = static_cast<const char*>(p);
        if (kv.second.base && c >= kv.second.base && c < kv.second.base + kv.second.cap) {
            if (kv.second.live) --kv.second.live;
            return true;
        }
    }
    return false;
}

// Owning device buffer.
template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p && !arena_drop(p)) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        if (count <= n && p) return;
        release();
        const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
        if (void* q = arena_take(bytes)) p = static_cast<T*>(q);
        else HIP_CHECK(hipMalloc(&p, bytes));
        n = count;
    }
    void upload(const T* src, size_t count, hipStream_t s) {
        alloc(count);
        if (count) HIP_CHECK(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s));
    }
};

// Page-locked host buffer: the staging side of every host<->device copy on
// the build's path.  A pageable source or destination makes hipMemcpyAsync
// wait for the device (the early up-sweep's target upload then waited for
// the whole previous batch).
template <class T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    HostBuf() = default;
    HostBuf(const HostBuf&) = delete;
    HostBuf& operator=(const HostBuf&) = delete;
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
    void alloc(size_t count) {
        if (count <= n && p) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(count, 1) * sizeof(T),
                                hipHostMallocDefault));
        n = count;
    }
};

// One timed interval: a single launch (events on its dispatch packet) or a
// group of consecutive launches of one kernel (events recorded around them).
struct Pending {
    const char* name;
    hipEvent_t a, b;
    double bytes;  // launches whose bytes are known at launch time
    std::vector<std::function<double()>> late;  // bytes known only after the batch ran
    uint64_t launches = 1;
};

struct Agg {
    uint64_t launches = 0;
    double ms = 0.0, bytes = 0.0;
};

bool async_on();  // CPD_ASYNC (defined with the other switches)
hipStream_t thread_stream(int device);

// Largest auto batch (CPD_BATCH_MAX, a multiple of 1024 <= 32768; A/B knob).
// 28672 since the rows are built at the packed width (8.0 MB per target at
// 1M nodes; profiles/batch_ab/r05am: 387.3k against 380.8k rows/s at 24576).
uint32_t batch_max() {
    static const uint32_t v = [] {
        const char* e = std::getenv("CPD_BATCH_MAX");
        const unsigned long b = e && *e ? std::strtoul(e, nullptr, 10) : 28672ul;
        return (uint32_t)std::max(1024ul, std::min(32768ul, b / 1024ul * 1024ul));
    }();
    return v;
}

// CPD_RLE_FUSED=0: the count / seam repair / emit passes instead of the
// fused one-pass emit (4-bit sets; A/B, identical rows)
bool rle_fused_on() {
    static const bool on = [] {
        const char* e = std::getenv("CPD_RLE_FUSED");
        return !(e && *e == '0');
    }();
    return on;
}
bool rle_fused(uint32_t fmb) { return fmb == 4 && rle_fused_on(); }

// Pool rows (1 KiB: one 256-target group row kept 32-bit) of a narrow batch
// of B targets: an eighth of its group rows, and at least every group row of
// one 1024-target slab, so that a batch whose wide rows overflow the pool is
// rebuilt in pieces of pool_cap / (4 n) slabs that cannot.
uint64_t pool_rows(uint32_t n, uint32_t B) {
    return std::max<uint64_t>((uint64_t)n * (B / 256u) / 8u, 4ull * n);
}

// HBM per row of batch width: the final rows (narrow: 2n of u16 offsets, the
// bases and the wide-row pool; else 4n of u32) + two compact up stores (4 B
// per node of up-level >= 2 each: batch k + 1's up-sweep runs beside batch
// k's down-sweep) + three buffer sets of first-move rows and RLE segment states
// (emit overlap) + the chunked count's chunk states (12 B per chunk: exit,
// count, entry) + leaf sets + two rows of move tables (npad / 2 each: the
// row set being built and the one a caller such as make_cpd_auto is
// exporting).  The pool's 1024-row floor is in the fixed part (pool_rows).
double batch_bytes_per_row(uint32_t n, uint32_t n_up, uint32_t npad, uint32_t fmb, bool narrow,
                           bool leaf_fm, uint32_t mbits) {
    // the fused emit keeps no segment states: 12 B per chunk of 32k columns
    const double rle = rle_fused(fmb) ? 12.0 * rle_emit_chunks(npad)
                                      : 3.0 * 5.0 / 32.0 * npad +
                                            (fmb == 4 ? 12.0 * rle_count_chunks(npad) : 0.0);
    const double fin = narrow ? (2.0 + 4.0 / 256.0 + 0.5) * n : 4.0 * n;
    return fin + 8.0 * n_up + 3.0 * fmb / 8.0 * npad + rle + (leaf_fm ? 0.5 * n : 0.0) +
           2.0 * mbits / 8.0 * npad;
}
bool lane_key_on();
bool seg_order_on();
bool search_trace();
std::vector<uint32_t> hilbert_keys(const int32_t* x, const int32_t* y, uint32_t n);

}  // namespace

struct cpd_graph {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t n = 0, m = 0, npad = 0;
    std::vector<uint32_t> order;       // node -> column
    std::vector<uint32_t> inv;         // column -> node
    DevBuf<uint32_t> order_d;          // node -> column (query preparation)
    std::vector<uint32_t> edge_perm;   // column-space edge -> file edge
    std::vector<uint32_t> w_free_col;  // free-flow weights, column-space edges
    std::vector<uint32_t> rowc_host;   // column-space row_ptr (host copy)
    std::vector<uint32_t> dst_col_host;  // column-space edge heads (host copy)
    // column-space CSR of the original graph
    DevBuf<uint32_t> row_ptr, dst, w;
    // packed fixed-stride adjacency for table-search: (dst col, w) pairs,
    // 2^adj_shift slots per column, dst = 0xFFFFFFFF past the out-degree
    uint32_t adj_shift = 0;
    DevBuf<uint32_t> adj;

    std::vector<uint32_t> packed_adjacency(const std::vector<uint32_t>& wcol) const {
        const size_t stride = (size_t)1 << adj_shift;
        std::vector<uint32_t> a(2 * stride * n, 0xFFFFFFFFu);
        for (uint32_t c = 0; c < n; ++c)
            for (uint32_t e = rowc_host[c]; e < rowc_host[c + 1]; ++e) {
                size_t slot = ((size_t)c * stride + (e - rowc_host[c])) * 2;
                a[slot] = dst_col_host[e];
                a[slot + 1] = wcol[e];
            }
        return a;
    }
    // sweeps: level-ordered node lists, per-slot arc offsets, (col, w) arcs
    DevBuf<uint32_t> asc_nodes, asc_off, asc_arcs;
    DevBuf<uint32_t> dsc_nodes, dsc_off, dsc_arcs, dsc_desc;
    std::vector<uint32_t> asc_lvl, dsc_lvl;         // level -> first slot
    // bytes model: gathered arcs and own-row reads per level
    std::vector<double> asc_lvl_arcs, dsc_lvl_arcs, dsc_lvl_reads;
    std::vector<uint32_t> asc_off_host;
    uint64_t ch_arcs = 0;
    bool has_ch = false;
    // batch workspace
    uint32_t B = 0;
    uint32_t fmb = 16;  // bits per first-move set (fm_bits(adj_shift))
    // bits per move in the packed compact form: every move indexes its
    // column's out-list (wildcard runs take bit 0), so out-degrees <= 2^bits
    uint32_t move_bits = 4;
    // the move tables in HBM (built rows, dense indexes) at the same width:
    // 2^tlb bits per column
    uint32_t tlb = 2;
    // dist: the dense final rows (narrow rows off only); counts: run counts
    DevBuf<uint32_t> dist, counts;
    // The compact up stores, one per batch slot (see BatchSlot): up[u][B],
    // u = ascending slot - ubase for the n_up nodes of up-level >= 2, their
    // live masks and the batch's target masks.
    uint32_t ubase = 0, n_up = 0;
    DevBuf<uint32_t> upx[2], livex[2], tmaskx[2];
    DevBuf<uint32_t> dsc_up;  // descending slot -> up index (~0: closed form)
    // Emit overlap (CPD_ASYNC, default on): a batch's move-table emit
    // (rle_moves) runs on `estream` while the next batch's sweeps start on
    // `stream` — the sweeps' narrow, latency-bound levels overlap the emit.
    // The buffers the emit reads (first-move rows, RLE segment states, lane ->
    // row map) come in up to kSets sets used round robin: set x is reused
    // only after the emit that read it (ev_emit[x]) has finished.  Three
    // sets give an emit two steps to finish: it runs at low occupancy beside
    // the sweeps, and with two sets the next-but-one batch's first moves
    // waited ~16 ms per step for it (profiles/up_store_ab/, round 6).
    static constexpr uint32_t kSets = 3;
    hipStream_t estream = nullptr;
    bool async = false;
    uint32_t nsets = 1, cur = 0;
    hipEvent_t ev_emit[kSets] = {nullptr, nullptr, nullptr};
    bool emit_pending[kSets] = {false, false, false};
    DevBuf<uint32_t> fmx[kSets];      // [B][npad] fmb-bit sets
    DevBuf<uint32_t> rle_stx[kSets];  // [B][npad/32] RLE segment entry states
    DevBuf<uint8_t> rle_rcx[kSets];   // [B][npad/32] runs ending in each segment
    DevBuf<uint32_t> lane_rowx[kSets];  // [B] table row of each batch lane
    // chunk exit states / run counts of the chunked count (read by rle_fix on
    // the same stream before the next batch: one set)
    DevBuf<uint32_t> rle_xs, rle_cc, rle_hard;
    DevBuf<uint32_t> emit_ck;  // fused emit: the chunks' guessed entries, exits, breaks
    HostBuf<uint32_t> rle_hard_h;          // [1]
    // the buffer set the next batch uses, once the emit that last read it is done
    uint32_t acquire_set() {
        const uint32_t x = cur;
        cur = (cur + 1u) % nsets;
        if (emit_pending[x]) {
            HIP_CHECK(hipStreamWaitEvent(stream, ev_emit[x], 0));
            emit_pending[x] = false;
        }
        return x;
    }
    void drain_emits() {
        if (estream) HIP_CHECK(hipStreamSynchronize(estream));
        for (auto& p : emit_pending) p = false;
    }
    // leaf first moves from the down-sweep (4-bit sets only): leafbits[col/32]
    // bit = column is a CH leaf; fmleaf [col][B/4] u16 = its sets, 4 per lane
    bool leaf_fm = false;
    DevBuf<uint32_t> leafbits;
    DevBuf<uint16_t> fmleaf;
    // narrow final-distance rows (NarrowRows, cpd_kernels.hpp): on unless
    // CPD_NARROW=0 at graph creation or a finite distance could reach the
    // wide-row marker; group rows that do not fit are kept wide in the pool
    // (counted: ovf)
    bool narrow = false;
    // the first kNarrowProbe full batches count their wide group rows; if
    // most are wide (long edges: the spread of 256 distances passes 0xFFFF),
    // narrow rows only add a base load per gather and are switched off for
    // the graph's lifetime — the results are identical either way
    static constexpr uint32_t kNarrowProbe = 2;
    uint32_t narrow_probe = kNarrowProbe;
    HostBuf<uint32_t> ovf_hb;  // [1] wide group rows of the last down-sweep
    uint32_t ovf_h() const { return ovf_hb.p ? ovf_hb.p[0] : 0u; }
    DevBuf<uint16_t> d16;
    DevBuf<uint32_t> dbase, ovf, pool;
    uint32_t pool_cap = 0;
    NarrowRows narrow_rows(bool on) {
        if (!on) return NarrowRows{nullptr, nullptr, n, nullptr, nullptr, 0};
        return NarrowRows{d16.p, dbase.p, n, ovf.p, pool.p, pool_cap};
    }
    double n_leaf = 0, m_leaf = 0;    // leaves, their out-edges
    std::vector<double> dsc_lvl_leaves;
    // Per-batch state, two slots (batches alternate): a batch's up-sweep runs
    // (on ustream) while the previous batch's down-sweep reads the other
    // slot's up store.  tgt: the batch's target columns by lane; pos_of[i] =
    // lane of the caller's target i; stat: per-level sweep counters (timing
    // runs; 2 per launch: stored / own rows, gathered rows), stat_h its host
    // copy; up_late: (level, arcs, nodes) of the up levels whose bytes wait
    // for it.  ev_fm[slot] marks the end of the slot's batch (its first
    // moves); its down-sweep is the last reader of its up store, live and
    // target masks and stats, and first moves read the targets from fm_tgt.
    struct BatchSlot {
        DevBuf<uint32_t> tgt;
        std::vector<uint32_t> pos_of, tgt_col;
        HostBuf<uint32_t> tgt_h;  // upload staging
        DevBuf<unsigned int> stat;
        HostBuf<unsigned int> stat_h;
        std::vector<std::array<double, 3>> up_late;
    };
    BatchSlot bs[2];
    DevBuf<uint32_t> fm_tgt;  // the targets of the batch whose first moves are queued
    // Timing runs: a batch's sweep bytes that depend on its live-row counts
    // (stat_h, copied out after its first moves), folded into agg once those
    // have landed — at the end of the next batch, or at timing_get / reset.
    // up: (level, arcs, nodes) per up level; down: (stat index, known bytes).
    struct LateRec {
        uint32_t slot = 0;
        std::vector<std::array<double, 3>> up;
        std::vector<std::array<double, 2>> down;
    };
    std::vector<LateRec> late_q;
    uint32_t next_slot = 0;
    // Early up-sweep of the next batch:
    // build_batch launches it on ustream right after queueing the current
    // batch's down-sweep, into the other slot's up store, so it runs beside
    // that down-sweep.  prep: the slot and targets it was launched for, ev_up
    // its end.
    hipStream_t ustream = nullptr;
    hipEvent_t ev_up = nullptr, ev_down = nullptr, ev_fm[2] = {nullptr, nullptr};
    bool prepped = false;
    uint32_t prep_slot = 0;
    std::vector<uint32_t> prep_targets, hint;
    void drop_prep() {  // wait for an early up-sweep nobody will use
        if (ustream) HIP_CHECK(hipStreamSynchronize(ustream));
        prepped = false;
    }
    DevBuf<uint32_t> asc_lvl_of, dsc_lvl_of;  // slot -> level
    // narrow upward levels (<= kNarrow nodes) run chunked: per level l,
    // items [up_item_first[l], up_item_first[l+1]) of (slot, a0, a1, 0);
    // up_init_slots = the ascending slots of all their nodes (leaf-form init)
    std::vector<uint32_t> up_item_first;
    DevBuf<uint32_t> up_items, up_init_slots;
    uint32_t n_init_slots = 0;
    // lane position of each caller target in the current batch (sorted by
    // lane_key when the caller gave coordinates, else by column)
    std::vector<uint32_t> lane_key;  // node -> Hilbert key of its coordinates (may be empty)
    // first_moves' segment order: the 32-column segments by the Hilbert key
    // of their middle column's node (empty: column order)
    DevBuf<uint32_t> seg_order;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<Pending> pending;
    std::map<std::string, Agg> agg;

    ~cpd_graph() {
        if (hipSetDevice(device) == hipSuccess) {
            if (estream) (void)hipStreamSynchronize(estream);
            for (auto e : ev_emit)
                if (e) (void)hipEventDestroy(e);
            if (estream) (void)hipStreamDestroy(estream);
            if (ustream) (void)hipStreamSynchronize(ustream);
            for (auto e : {ev_up, ev_down, ev_fm[0], ev_fm[1]})
                if (e) (void)hipEventDestroy(e);
            if (ustream) (void)hipStreamDestroy(ustream);
            if (stream) (void)hipStreamSynchronize(stream);
            for (auto& p : pending) {
                (void)hipEventDestroy(p.a);
                (void)hipEventDestroy(p.b);
            }
            for (auto e : ev_pool) (void)hipEventDestroy(e);
            if (stream) (void)hipStreamDestroy(stream);
        }
    }

    hipEvent_t get_event() {
        if (ev_pool.empty()) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            return e;
        }
        hipEvent_t e = ev_pool.back();
        ev_pool.pop_back();
        return e;
    }
    // Time one launch when timing is on: the events are attached to the
    // kernel's own dispatch packet (hipExtLaunchKernelGGL, see launchers).
    // Inside group_begin(name) / group_end() the launches of `name` carry no
    // events: one pair recorded around the whole run of launches times them
    // (per-packet profiling signals cost ~7 us per launch, ~3 % of a batch's
    // ~580 sweep launches; the group interval also counts the inter-kernel
    // gaps, so its per-launch average is a slight over-estimate).
    // Every launch is checked: hipGetLastError() is cleared first, so an
    // error left behind by an unrelated earlier runtime call on this thread
    // (it is sticky until read) is not blamed on the launch.
    template <class F>
    void timed(const char* name, double bytes, F&& launch,
               std::function<double()> late_bytes = nullptr) {
        (void)hipGetLastError();
        if (!timing) {
            launch();
            HIP_CHECK(hipGetLastError());
            return;
        }
        if (group_open && std::strcmp(group.name, name) == 0) {
            launch();
            HIP_CHECK(hipGetLastError());
            if (late_bytes) group.late.push_back(std::move(late_bytes));
            else group.bytes += bytes;
            group.launches++;
            return;
        }
        hipEvent_t a = get_event(), b = get_event();
        set_launch_events(a, b);
        launch();
        HIP_CHECK(hipGetLastError());
        Pending p{name, a, b, late_bytes ? 0.0 : bytes, {}, 1};
        if (late_bytes) p.late.push_back(std::move(late_bytes));
        pending.push_back(std::move(p));
    }
    Pending group;
    bool group_open = false;
    hipStream_t group_stream = nullptr;
    void group_begin(const char* name, hipStream_t st) {
        if (!timing) return;
        group = Pending{name, get_event(), nullptr, 0.0, {}, 0};
        group_stream = st;
        HIP_CHECK(hipEventRecord(group.a, st));
        group_open = true;
    }
    void group_end() {
        if (!group_open) return;
        group_open = false;
        group.b = get_event();
        HIP_CHECK(hipEventRecord(group.b, group_stream));
        if (group.launches) {
            pending.push_back(std::move(group));
        } else {
            ev_pool.push_back(group.a);
            ev_pool.push_back(group.b);
        }
        group = Pending{};
    }
    // Wait for `stream` (all = also the emit stream), then fold the timed
    // intervals that have completed into agg; intervals of an emit still
    // running on estream stay pending until a later sync.
    void sync(bool all = false) {
        HIP_CHECK(hipStreamSynchronize(stream));
        if (all) {
            drain_emits();
            if (ustream) HIP_CHECK(hipStreamSynchronize(ustream));
        }
        std::vector<Pending> keep;
        for (auto& p : pending) {
            if (hipEventQuery(p.b) != hipSuccess) {
                keep.push_back(std::move(p));
                continue;
            }
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
            Agg& g = agg[p.name];
            g.launches += p.launches;
            g.ms += ms;
            g.bytes += p.bytes;
            for (auto& f : p.late) g.bytes += f();
            ev_pool.push_back(p.a);
            ev_pool.push_back(p.b);
        }
        pending.swap(keep);
    }
    void select() const { HIP_CHECK(hipSetDevice(device)); }
    uint32_t wpr() const { return npad >> (5u - tlb); }  // words per move-table row

    uint64_t hbm_reserve = 0;  // cpd_graph_set_hbm_reserve
    void reserve_batch(uint32_t want) {
        ArenaScope carve;  // the batch's buffers: what an arena is committed for
        if (want == 0) {
            size_t free_b = 0, total_b = 0;
            HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
            // per target (batch_bytes_per_row), in 85% of free HBM; at most
            // 24 slabs.  Larger batches amortise the latency-bound
            // narrow levels: at 1M nodes 20480 rows per batch measured 310.5k
            // rows/s against 296.1k for 16384 (round 2).
            const double per = batch_bytes_per_row(n, n_up, npad, fmb, narrow, leaf_fm,
                                                   1u << tlb);
            const double fixed = narrow ? 4096.0 * n : 0.0;  // the pool's floor (pool_rows)
            const double avail = free_b > hbm_reserve + fixed ? (double)free_b - hbm_reserve - fixed
                                                              : 0.0;
            const double fit = 0.85 * avail / per;
            CPD_REQUIRE(hbm_reserve == 0 || fit >= 1024.0, CPD_E_OOM,
                        "HBM reserve of " + std::to_string(hbm_reserve >> 20) + " MiB leaves " +
                            std::to_string((size_t)avail >> 20) + " MiB: too little for a 1024-row batch");
            want = (uint32_t)std::min((double)batch_max(), std::max(1024.0, std::floor(fit / 1024) * 1024));
        }
        want = (want + 1023u) / 1024u * 1024u;
        if (want == B && upx[0].p) return;
        drain_emits();
        drop_prep();
        B = want;
        for (int s = 0; s < 2; ++s) {
            upx[s].alloc(std::max<size_t>((size_t)n_up * B, 1));
            livex[s].alloc(std::max<uint32_t>(n_up, 1u));
            tmaskx[s].alloc(n);
        }
        alloc_final_rows();
        // each further buffer set when it takes under an eighth of the HBM
        // still free after the batch's own buffers (one set: emits do not
        // overlap)
        const bool fused = rle_fused(fmb);
        const size_t set_bytes = (size_t)B * (npad / (32u / fmb)) * 4u +
                                 (fused ? 0u : (size_t)B * (npad / 32u) * 5u) + 4u * B;
        nsets = 1;
        for (uint32_t x = 0; x < kSets; ++x) {
            if (x >= 1) {
                size_t free_b = 0, total_b = 0;
                HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
                if (!(async_on() && set_bytes * 8 < (free_b > hbm_reserve ? free_b - hbm_reserve : 0))) {
                    for (uint32_t y = x; y < kSets; ++y) {
                        fmx[y].release();
                        rle_stx[y].release();
                        rle_rcx[y].release();
                        lane_rowx[y].release();
                    }
                    break;
                }
                nsets = x + 1;
            }
            fmx[x].alloc((size_t)B * (npad / (32u / fmb)));
            if (fused) {
                rle_stx[x].release();
                rle_rcx[x].release();
            } else {
                rle_stx[x].alloc((size_t)B * (npad / 32u));
                rle_rcx[x].alloc((size_t)B * (npad / 32u));
            }
            lane_rowx[x].alloc(B);
        }
        async = nsets > 1;
        cur = 0;
        if (fused) {
            emit_ck.alloc(3ull * B * rle_emit_chunks(npad));
        } else if (fmb == 4 && rle_count_chunks(npad)) {
            rle_xs.alloc(2ull * B * rle_count_chunks(npad));
            rle_cc.alloc((size_t)B * rle_count_chunks(npad));
            rle_hard.alloc(1);
        }
        if (leaf_fm) fmleaf.alloc((size_t)n * (B / 4u));
        for (auto& b : bs) {
            b.tgt.alloc(B);
            b.tgt_h.alloc(B);
        }
        fm_tgt.alloc(B);
        counts.alloc(B);
        rle_hard_h.alloc(1);
        ovf_hb.alloc(1);
        ovf_hb.p[0] = 0;
    }
    // The final rows of a batch of B: narrow (u16 offsets, bases, the pool of
    // wide group rows) or the dense 32-bit rows.
    void alloc_final_rows() {
        ArenaScope carve;
        if (narrow) {
            dist.release();
            d16.alloc((size_t)n * B);
            dbase.alloc((size_t)n * (B / 256u));
            pool_cap = (uint32_t)std::min<uint64_t>(pool_rows(n, B), 0xFFFFFFFEull);
            pool.alloc((size_t)pool_cap * 256u);
            ovf.alloc(1);
        } else {
            d16.release();
            dbase.release();
            pool.release();
            pool_cap = 0;
            dist.alloc((size_t)n * B);
        }
    }
};

struct cpd_rows {
    int device = 0;
    uint32_t nrows = 0;
    mutable uint64_t total = 0;  // runs of all rows (valid after settle())
    hipEvent_t done = nullptr;   // after the last batch's count + emit (emit stream)
    void wait() const {
        if (done) HIP_CHECK(hipEventSynchronize(done));
    }
    ~cpd_rows() {
        if (done) {
            (void)hipEventSynchronize(done);
            (void)hipEventDestroy(done);
        }
    }
    // A batch's run counts arrive after its rows are queued: the count pass
    // runs on the emit stream, beside the next batch's sweeps.  Per batch:
    // its rows' lanes and two page-locked buffers — the lane -> table row map
    // the emit reads and the per-lane run counts it lands — turned into run
    // offsets by settle() once `done` has passed.  A rebuild into these rows
    // retires the unsettled batches (their copies may still be in flight).
    struct Batch {
        uint32_t k = 0;
        std::vector<uint32_t> pos_of;
        HostBuf<uint32_t> lane_rows, counts;
        hipEvent_t ev = nullptr;  // after the batch's last copy (emit stream)
        ~Batch() {
            if (ev) (void)hipEventDestroy(ev);
        }
    };
    mutable std::mutex settle_mu;
    mutable std::vector<std::unique_ptr<Batch>> pending, retired, spare;
    Batch* new_batch(uint32_t B) {
        for (size_t i = 0; i < retired.size();) {  // recycle what the device is done with
            if (hipEventQuery(retired[i]->ev) == hipSuccess) {
                spare.push_back(std::move(retired[i]));
                retired.erase(retired.begin() + (long)i);
            } else {
                ++i;
            }
        }
        std::unique_ptr<Batch> b;
        if (!spare.empty()) {
            b = std::move(spare.back());
            spare.pop_back();
        } else {
            b = std::make_unique<Batch>();
        }
        b->lane_rows.alloc(B);
        b->counts.alloc(B);
        if (!b->ev) HIP_CHECK(hipEventCreateWithFlags(&b->ev, hipEventDisableTiming));
        pending.push_back(std::move(b));
        return pending.back().get();
    }
    void retire() {
        for (auto& b : pending) retired.push_back(std::move(b));
        pending.clear();
    }
    void settle() const;
    std::vector<uint32_t> targets;   // node ids, row order
    std::vector<uint32_t> lanes;     // batch lane of each row
    mutable std::vector<uint64_t> offsets;  // run offsets (host), nrows+1 (after settle())
    // The rows in their compact form: move tables at 2^tlb bits per column,
    // wpr = npad * 2^tlb / 32 words per row (rle_moves) — the RLE row
    // expanded, 10x smaller than its runs on the bench graph (2 bits).  Run
    // words are decoded from them on demand (moves_runs, at `off`).
    uint32_t n = 0, wpr = 0, bits = 4, tlb = 2;  // bits: per move in the exported form
    DevBuf<uint32_t> moves;
    mutable DevBuf<uint64_t> off;
    uint32_t packed_words() const { return (uint32_t)(((uint64_t)n * bits + 31u) / 32u); }
    // device staging for decoded runs, one buffer per concurrent exporter
    // (make_cpd_auto's writer threads), kept until the rows are freed
    mutable std::mutex stage_mu;
    mutable std::vector<std::unique_ptr<DevBuf<uint32_t>>> stages;
    std::unique_ptr<DevBuf<uint32_t>> acquire_stage() const {
        std::lock_guard<std::mutex> l(stage_mu);
        if (stages.empty()) return std::make_unique<DevBuf<uint32_t>>();
        auto b = std::move(stages.back());
        stages.pop_back();
        return b;
    }
    void release_stage(std::unique_ptr<DevBuf<uint32_t>> b) const {
        std::lock_guard<std::mutex> l(stage_mu);
        stages.push_back(std::move(b));
    }
};

// A table-search index: nrows rows (row i = target row_targets[i]) that arrive
// in append order — all at once (cpd_index_create / _from_rows) or streamed
// (cpd_index_create_empty + cpd_index_append_*).  Two HBM forms:
//   keep_rle      the RLE runs stay resident (offsets + runs); dense tables,
//                 if asked for, are expanded from them on first use;
//   stream_dense  each appended chunk is expanded into the 4-bit move tables
//                 straight away and its runs are dropped, so a worker whose
//                 runs outgrow HBM (1M nodes div 8: ~312 GB of runs, 62.5 GB
//                 of tables) is still served.
struct cpd_index {
    cpd_graph* g = nullptr;
    uint32_t nrows = 0;   // rows when complete
    uint32_t added = 0;   // rows appended so far
    uint64_t total = 0;   // runs resident so far (keep_rle)
    uint64_t cap = 0;     // run capacity of `runs` (keep_rle)
    uint64_t declared = 0;  // total runs of all rows (from the caller or the rows)
    std::vector<uint32_t> row_of_col;   // host copy
    std::vector<uint32_t> row_targets;  // declared targets, row order
    std::vector<uint64_t> offsets;      // host copy, added + 1 (keep_rle)
    DevBuf<uint32_t> d_row_of_col, runs, adj_sel;  // adj_sel: packed adjacency, custom weights
    DevBuf<uint64_t> off;
    bool custom_w = false;
    // CPD_INDEX_AUTO / _RLE / _DENSE; dense = 4-bit move tables expanded from
    // the RLE rows (built on first use, or as rows stream in)
    int mode = CPD_INDEX_AUTO;
    bool keep_rle = true;
    bool stream_dense = false;
    DevBuf<uint32_t> dense;
    bool dense_ready = false;
    // staging of host-appended chunks (stream_dense), format flag
    DevBuf<uint32_t> stage, pstage;  // pstage: packed compact rows before unpacking
    DevBuf<uint32_t> xstage, lost;   // nibble rows before narrowing; repack's flag
    DevBuf<uint64_t> stage_off;
    DevBuf<uint32_t> flag;
    // expand_rows work split: first run-chunk of each row being expanded
    std::vector<uint32_t> chunk_first_h;
    DevBuf<uint32_t> chunk_first;

    bool use_dense() const {
        if (stream_dense) return true;
        if (mode == CPD_INDEX_DENSE) return true;
        if (mode == CPD_INDEX_RLE) return false;
        // auto: the table whose bytes are fewer (4 B per run vs npad * bits / 8
        // B per row)
        return nrows > 0 && 4.0 * (double)declared > 4.0 * (double)g->wpr() * nrows;
    }
    // CPD-search: per-row tables when they fit (hrow free-flow heuristic,
    // crow / lrow incumbent cost and moves under the current weights; rebuilt
    // for new weights), row target columns, workspace (per lane slot),
    // per-query counters, sums
    DevBuf<uint64_t> hrow, crow;
    DevBuf<uint32_t> lrow, tcol, qstats;
    DevBuf<uint8_t> sws;
    DevBuf<unsigned long long> sagg;
    // resumable overflow: the two spill pools (records of the pass that just
    // ran / of the one running), their bump counters, record offsets
    DevBuf<uint32_t> spool[2];
    DevBuf<unsigned long long> stop, sat;
    bool h_ready = false, c_ready = false;
    bool searched = false;  // qstats hold the counters of the prepared queries
    // query workspace; queries run sorted by target row (qperm[i] = caller
    // index of sorted query i), all of it prepared on the GPU
    uint32_t nq = 0;
    DevBuf<uint32_t> qin_s, qin_t, qkey, qkey2, qval, qperm, qbad;
    DevBuf<uint8_t> qsort_tmp, qout;
    DevBuf<uint32_t> qs, qt, qrow, hops;
    DevBuf<uint64_t> cost;
    DevBuf<uint8_t> fin;
    DevBuf<unsigned long long> agg;
};

void cpd_rows::settle() const {
    std::lock_guard<std::mutex> l(settle_mu);
    HIP_CHECK(hipSetDevice(device));
    wait();
    for (auto& b : retired) spare.push_back(std::move(b));
    retired.clear();
    if (pending.empty()) return;
    for (auto& b : pending) {
        for (uint32_t i = 0; i < b->k; ++i)
            offsets.push_back(offsets.back() + b->counts.p[b->pos_of[i]]);
        spare.push_back(std::move(b));
    }
    pending.clear();
    total = offsets.back();
    hipStream_t st = thread_stream(device);
    off.upload(offsets.data(), offsets.size(), st);
    HIP_CHECK(hipStreamSynchronize(st));
}

namespace {

// Closed-form encodings of the two lowest upward levels (cpd_kernels.hip).
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kL1Bit = 0x40000000u;

// Optimisation switches for A/B runs: CPD_<NAME>=0 turns one off (CPD_LIVE,
// CPD_SORT, CPD_LEAFFM here, CPD_XCD in the launchers); results are identical
// either way.
bool env_on(const char* name) {
    const char* e = std::getenv(name);
    return !(e && *e == '0');
}

// One non-blocking stream per (host thread, device), kept for the thread's
// lifetime: exports from several host threads never queue behind a build's
// stream or each other.
hipStream_t thread_stream(int device) {
    thread_local std::vector<hipStream_t> streams;
    if (streams.size() <= (size_t)device) streams.resize(device + 1, nullptr);
    hipStream_t& st = streams[device];
    if (!st) HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
}

// Runs decoded per export piece (a longer row alone): 256 MB of staging.
constexpr uint64_t kDecodeRuns = 64ull << 20;

void require_device() {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0)
        throw Error(CPD_E_HIP, "no HIP device available (libcpd has no CPU fallback)");
}

// Nodes ordered by (level, column): node_of_slot, and lvl_first[l] = first slot.
std::vector<uint32_t> level_order(const cpd_plan& p, const std::vector<uint32_t>& level,
                                  uint32_t nlev, std::vector<uint32_t>& lvl_first) {
    const uint32_t n = p.n;
    std::vector<uint32_t> cnt(nlev + 1, 0);
    for (uint32_t v = 0; v < n; ++v) cnt[level[v] + 1]++;
    for (uint32_t l = 0; l < nlev; ++l) cnt[l + 1] += cnt[l];
    lvl_first.assign(cnt.begin(), cnt.end());
    std::vector<uint32_t> node_of_slot(n), pos(cnt.begin(), cnt.end() - 1);
    for (uint32_t c = 0; c < n; ++c) {  // columns ascending inside a level
        uint32_t v = p.inv[c];
        node_of_slot[pos[level[v]]++] = v;
    }
    return node_of_slot;
}

// Build the level-ordered sweep arrays in column space, with the closed-form
// encodings of cpd_kernels.hip (kLeafBit: upward level 0, kL1Bit: level 1,
// referenced by its slot in the ASCENDING list, asc_slot[node]).
// lvl_arcs: gathered arcs per level; lvl_reads: nodes reading their own row.
// leaf_edges (descending only): a leaf's list is its out-edges in file order
// (self loops and parallel edges included) instead of its up-arcs — the same
// minimum, and the list position is the move index for the leaf's first-move
// set (the down-sweep computes leaf sets, cpd_kernels.hip sweep_down8c).
// Nodes of up-level >= 2 own a row of the compact up store, u = ascending
// slot - ubase: ascending arcs into them carry u; uidx (descending only)
// gets each slot's u (~0 for the closed forms).
void build_sweep(const cpd_plan& p, bool ascend, const std::vector<uint32_t>& asc_slot,
                 uint32_t ubase, std::vector<uint32_t>& nodes, std::vector<uint32_t>& off,
                 std::vector<uint32_t>& arcs, std::vector<uint32_t>& lvl_first,
                 std::vector<double>& lvl_arcs, std::vector<double>& lvl_reads,
                 bool leaf_edges = false, std::vector<uint32_t>* uidx = nullptr) {
    const Hierarchy& H = p.ch;
    const uint32_t n = p.n;
    const std::vector<uint32_t>& level = ascend ? H.level_up : H.level_dn;
    const uint32_t nlev = ascend ? H.nlev_up : H.nlev_dn;
    // ascend reads each node's DOWN arcs; descend reads its UP arcs
    const std::vector<uint64_t>& aoff = ascend ? H.dn_off : H.up_off;
    const std::vector<uint32_t>& adst = ascend ? H.dn_dst : H.up_dst;
    const std::vector<uint32_t>& aw = ascend ? H.dn_w : H.up_w;
    const std::vector<uint32_t>& lup = H.level_up;
    CPD_REQUIRE(aoff[n] < 0xFFFFFFFFull, CPD_E_RANGE, "hierarchy has >= 2^32 arcs");
    // (ordering a level's nodes by their lowest up-arc head instead, so that
    // nodes gathering the same rows run side by side, measured no faster)
    std::vector<uint32_t> node_of_slot = level_order(p, level, nlev, lvl_first);
    // how a node is referenced: closed form (level 0 / 1 of the up sweep) or row
    auto ref = [&](uint32_t v) -> uint32_t {
        if (lup[v] == 0) return p.order[v] | kLeafBit;
        if (lup[v] == 1) return asc_slot[v] | kL1Bit;
        return p.order[v];
    };
    nodes.assign(n, 0);
    if (uidx) uidx->assign(n, 0xFFFFFFFFu);
    for (uint32_t s = 0; s < n; ++s) {
        uint32_t v = node_of_slot[s];
        nodes[s] = ascend ? p.order[v] : ref(v);  // descending: closed-form init
        if (uidx && lup[v] >= 2) (*uidx)[s] = asc_slot[v] - ubase;
    }
    const bool leaf_rows = !ascend && leaf_edges;  // a leaf's arcs: its out-edges
    off.assign(n + 1, 0);
    for (uint32_t s = 0; s < n; ++s) {
        const uint32_t v = node_of_slot[s];
        off[s + 1] = off[s] + (leaf_rows && lup[v] == 0 ? p.row_ptr[v + 1] - p.row_ptr[v]
                                                        : (uint32_t)(aoff[v + 1] - aoff[v]));
    }
    arcs.assign(2ull * off[n], 0u);
    // slots filled by 8 host threads (each writes its slots' arcs; level
    // counts per thread, summed after)
    constexpr uint32_t kThreads = 8;
    std::vector<std::vector<double>> la(kThreads, std::vector<double>(nlev, 0.0)),
        lr(kThreads, std::vector<double>(nlev, 0.0));
    auto fill = [&](uint32_t t, uint32_t s0, uint32_t s1) {
        std::vector<std::pair<uint32_t, uint32_t>> tmp;
        for (uint32_t s = s0; s < s1; ++s) {
            const uint32_t v = node_of_slot[s];
            uint32_t* out = arcs.data() + 2ull * off[s];
            if (leaf_rows && lup[v] == 0) {
                for (uint32_t e = p.row_ptr[v]; e < p.row_ptr[v + 1]; ++e) {
                    *out++ = p.order[p.dst[e]];
                    *out++ = p.w[e];
                    if (p.dst[e] != v) la[t][level[v]] += 1.0;
                }
                continue;
            }
            tmp.clear();
            for (uint64_t e = aoff[v]; e < aoff[v + 1]; ++e) tmp.push_back({p.order[adst[e]], aw[e]});
            std::sort(tmp.begin(), tmp.end());
            for (auto& a : tmp) {
                // ascending arcs into upward levels 0/1 use the closed forms,
                // the others the head's up-store row
                const uint32_t h = p.inv[a.first];
                const uint32_t r = !ascend ? a.first : lup[h] >= 2 ? asc_slot[h] - ubase : ref(h);
                *out++ = r;
                *out++ = a.second;
                if (!(r & (kLeafBit | kL1Bit))) la[t][level[v]] += 1.0;
            }
            if (!ascend && !(nodes[s] & (kLeafBit | kL1Bit))) lr[t][level[v]] += 1.0;
        }
    };
    {
        std::vector<std::thread> th;
        const uint32_t per = (n + kThreads - 1u) / kThreads;
        for (uint32_t t = 0; t < kThreads; ++t)
            th.emplace_back(fill, t, std::min(n, t * per), std::min(n, (t + 1u) * per));
        for (auto& x : th) x.join();
    }
    lvl_arcs.assign(nlev, 0.0);
    lvl_reads.assign(nlev, 0.0);
    for (uint32_t t = 0; t < kThreads; ++t)
        for (uint32_t l = 0; l < nlev; ++l) {
            lvl_arcs[l] += la[t][l];
            lvl_reads[l] += lr[t][l];
        }
}


}  // namespace

extern "C" {

int cpd_device_count(int* count) {
    return guarded([&] {
        CPD_REQUIRE(count, CPD_E_ARG, "null count");
        hipError_t e = hipGetDeviceCount(count);
        if (e != hipSuccess) *count = 0;
    });
}

int cpd_device_mem_info(int device, uint64_t* free_bytes, uint64_t* total_bytes) {
    return guarded([&] {
        CPD_REQUIRE(free_bytes && total_bytes, CPD_E_ARG, "null argument");
        require_device();
        int count = 0;
        HIP_CHECK(hipGetDeviceCount(&count));
        CPD_REQUIRE(device >= 0 && device < count, CPD_E_ARG, "no such device");
        HIP_CHECK(hipSetDevice(device));
        size_t f = 0, t = 0;
        HIP_CHECK(hipMemGetInfo(&f, &t));
        *free_bytes = f;
        *total_bytes = t;
    });
}

int cpd_device_arena(int device, uint64_t bytes, int touch) {
    return guarded([&] {
        require_device();
        int count = 0;
        HIP_CHECK(hipGetDeviceCount(&count));
        CPD_REQUIRE(device >= 0 && device < count, CPD_E_ARG, "no such device");
        HIP_CHECK(hipSetDevice(device));
        {
            std::lock_guard<std::mutex> l(g_arena_mu);
            CPD_REQUIRE(!g_arena[device].base, CPD_E_ARG, "device arena already committed");
        }
        void* p = nullptr;
        HIP_CHECK(hipMalloc(&p, std::max<uint64_t>(bytes, 256)));
        if (touch) {  // first-touch costs paid here, off the build's path
            HIP_CHECK(hipMemset(p, 0, std::max<uint64_t>(bytes, 256)));
            HIP_CHECK(hipDeviceSynchronize());
        }
        std::lock_guard<std::mutex> l(g_arena_mu);
        g_arena[device] = Arena{static_cast<char*>(p), (size_t)std::max<uint64_t>(bytes, 256), 0};
    });
}

int cpd_device_arena_release(int device) {
    return guarded([&] {
        char* p = nullptr;
        {
            std::lock_guard<std::mutex> l(g_arena_mu);
            auto it = g_arena.find(device);
            if (it == g_arena.end()) return;
            CPD_REQUIRE(it->second.live == 0, CPD_E_ARG,
                        "device arena still holds " + std::to_string(it->second.live) +
                            " live buffers: free the graphs, row sets and indexes first");
            p = it->second.base;
            g_arena.erase(it);
        }
        if (p) {
            HIP_CHECK(hipSetDevice(device));
            HIP_CHECK(hipFree(p));
        }
    });
}

int cpd_batch_bytes(uint32_t n, uint32_t max_degree, uint32_t batch, uint64_t* bytes) {
    return guarded([&] {
        CPD_REQUIRE(bytes && batch % 1024u == 0 && batch > 0, CPD_E_ARG,
                    "batch_bytes: batch must be a positive multiple of 1024");
        uint32_t shift = 0;
        while ((1u << shift) < std::max(1u, max_degree)) ++shift;
        const uint32_t fmb = fm_bits(shift);
        const uint32_t npad = (n + kFmTile - 1u) / kFmTile * kFmTile;
        // narrow rows and leaf sets assumed, every node with a row in the up
        // stores (their upper bounds: the hierarchy is not known yet), plus the
        // pool's floor, the per-column arrays and the lane tables
        const uint32_t mbits = max_degree <= 2u ? 1u : max_degree <= 4u ? 2u : 4u;
        *bytes = (uint64_t)(batch_bytes_per_row(n, n, npad, fmb, true, fmb == 4, mbits) * batch) +
                 (uint64_t)batch * (n / 256u + 1u) * 4u + 4096ull * n + 512ull * n + (64ull << 20);
    });
}

namespace {
bool trace_on();
}  // namespace

int cpd_graph_create(const cpd_plan* p, int device, cpd_graph** out) {
    return guarded([&] {
        CPD_REQUIRE(p && out, CPD_E_ARG, "graph: null argument");
        *out = nullptr;
        require_device();
        const double tg0 = now_seconds();
        auto g = std::make_unique<cpd_graph>();
        g->device = device;
        g->select();
        // Three streams: the main one (down-sweep, first moves), the emit
        // stream and the up-sweep stream, where the next batch's up-sweep runs
        // beside the previous batch's first moves.  CU masks were measured and
        // removed: the up-sweep given q of every 8 CUs and the other streams
        // the rest (rounds 4-6: 350.6k / 324.2k against 366.7k rows/s; r06d:
        // 355.9k / 310.6k against 380.1k), or the up-sweep alone confined to
        // q of 8 (397.3-420.4k against 420.0-421.5k, profiles/up_store_ab/r06s_*).
        HIP_CHECK(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
        // (a lowest-priority emit stream measured the same: 65.2-65.7 ms/step
        // in round 5, 374.6-375.9k against 375.2-375.9k rows/s with the
        // one-wave emit, profiles/up_store_ab/r06k_*)
        HIP_CHECK(hipStreamCreateWithFlags(&g->estream, hipStreamNonBlocking));
        {
            // the highest priority: its small, latency-bound level kernels
            // must get CUs while the other streams' workgroups are queued (at
            // equal priority they waited for all of them to be dispatched:
            // 15 ms for a 0.7-ms init kernel; beside the first moves, as now,
            // normal priority measured the same: 419.1k against 413.2-419.1k
            // rows/s, profiles/up_store_ab/r06o_*)
            int least = 0, greatest = 0;
            HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIP_CHECK(hipStreamCreateWithPriority(&g->ustream, hipStreamNonBlocking, greatest));
        }
        for (hipEvent_t* e : {&g->ev_up, &g->ev_down, &g->ev_fm[0], &g->ev_fm[1]})
            HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        for (auto& e : g->ev_emit) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (trace_on()) std::fprintf(stderr, "[cpd] graph streams %.3f s\n", now_seconds() - tg0);
        const uint32_t n = p->n, m = p->m;
        g->n = n;
        g->m = m;
        g->npad = (n + kFmTile - 1u) / kFmTile * kFmTile;
        g->order = p->order;
        g->inv = p->inv;
        // column-space CSR, per-node out-edge order preserved (moves = file order)
        g->rowc_host.assign(n + 1, 0);
        for (uint32_t c = 0; c < n; ++c) {
            uint32_t v = p->inv[c];
            g->rowc_host[c + 1] = g->rowc_host[c] + (p->row_ptr[v + 1] - p->row_ptr[v]);
        }
        std::vector<uint32_t>& dstc = g->dst_col_host;
        dstc.resize(m);
        g->edge_perm.resize(m);
        g->w_free_col.resize(m);
        uint32_t maxdeg = 1;
        for (uint32_t c = 0; c < n; ++c) {
            uint32_t v = p->inv[c];
            uint32_t b = p->row_ptr[v], k = p->row_ptr[v + 1] - b;
            maxdeg = std::max(maxdeg, k);
            for (uint32_t i = 0; i < k; ++i) {
                uint32_t e = g->rowc_host[c] + i;
                g->edge_perm[e] = b + i;
                dstc[e] = p->order[p->dst[b + i]];
                g->w_free_col[e] = p->w[b + i];
            }
        }
        while ((1u << g->adj_shift) < maxdeg) ++g->adj_shift;
        g->fmb = fm_bits(g->adj_shift);
        g->move_bits = maxdeg <= 2 ? 1u : maxdeg <= 4 ? 2u : 4u;
        g->tlb = g->move_bits == 1u ? 0u : g->move_bits == 2u ? 1u : 2u;
        hipStream_t s = g->stream;
        g->order_d.upload(g->order.data(), n, s);
        g->row_ptr.upload(g->rowc_host.data(), n + 1, s);
        g->dst.upload(dstc.data(), m, s);
        g->w.upload(g->w_free_col.data(), m, s);
        std::vector<uint32_t> adj = g->packed_adjacency(g->w_free_col);
        g->adj.upload(adj.data(), adj.size(), s);
        HIP_CHECK(hipStreamSynchronize(s));
        if (trace_on()) std::fprintf(stderr, "[cpd] graph csr+adjacency %.3f s\n", now_seconds() - tg0);
        g->has_ch = !p->ch.rank.empty();
        if (!g->has_ch) {  // query-only graph (fifo_auto)
            *out = g.release();
            return;
        }
        std::vector<uint32_t> nodes, off, arcs, lvl;
        std::vector<double> unused;
        std::vector<uint32_t> asc_slot(n);
        {
            std::vector<uint32_t> node_of_slot =
                level_order(*p, p->ch.level_up, p->ch.nlev_up, lvl);
            for (uint32_t s2 = 0; s2 < n; ++s2) asc_slot[node_of_slot[s2]] = s2;
        }
        // the up store's rows: the nodes of up-level >= 2, in ascending slot order
        g->ubase = lvl.size() > 2 ? lvl[2] : n;
        g->n_up = n - g->ubase;
        // the two sweeps' lists are independent host work (~0.1 s each at 1M
        // nodes): the down-sweep's is built on a second thread meanwhile
        g->leaf_fm = g->fmb == 4 && env_on("CPD_LEAFFM");
        std::vector<uint32_t> dnodes, doff, darcs, dup;
        std::exception_ptr derr;
        std::thread dthr([&] {
            try {
                build_sweep(*p, false, asc_slot, g->ubase, dnodes, doff, darcs, g->dsc_lvl,
                            g->dsc_lvl_arcs, g->dsc_lvl_reads, g->leaf_fm, &dup);
            } catch (...) {
                derr = std::current_exception();
            }
        });
        struct Join {
            std::thread& t;
            ~Join() {
                if (t.joinable()) t.join();
            }
        } djoin{dthr};
        build_sweep(*p, true, asc_slot, g->ubase, nodes, off, arcs, g->asc_lvl, g->asc_lvl_arcs,
                    unused);
        g->asc_off_host = off;
        const std::vector<uint32_t> nodes_asc_host = nodes, asc_arcs_host = arcs;
        g->asc_nodes.upload(nodes.data(), nodes.size(), s);
        g->asc_off.upload(off.data(), off.size(), s);
        g->asc_arcs.upload(arcs.data(), arcs.size(), s);
        HIP_CHECK(hipStreamSynchronize(s));
        if (trace_on()) std::fprintf(stderr, "[cpd] graph up lists %.3f s\n", now_seconds() - tg0);
        g->ch_arcs = arcs.size() / 2;
        // leaf first moves in the down-sweep: 4-bit sets only (<= 4 slots)
        dthr.join();
        if (derr) std::rethrow_exception(derr);
        nodes.swap(dnodes);
        off.swap(doff);
        arcs.swap(darcs);
        g->dsc_nodes.upload(nodes.data(), nodes.size(), s);
        g->dsc_off.upload(off.data(), off.size(), s);
        g->dsc_arcs.upload(arcs.data(), arcs.size(), s);
        g->dsc_up.upload(dup.data(), dup.size(), s);
        {
            const uint32_t na = down_desc_arcs();
            std::vector<uint32_t> desc((size_t)n * 32u, 0u);
            const std::vector<uint32_t>& aoff = g->asc_off_host;
            // 128 B per node written by 8 host threads (each node's own slots)
            auto fill = [&](uint32_t x0, uint32_t x1) {
            for (uint32_t x = x0; x < x1; ++x) {
                uint32_t* d = desc.data() + (size_t)x * 32u;
                d[0] = nodes[x];
                d[1] = off[x];
                d[2] = off[x + 1];
                d[3] = dup[x];
                for (uint32_t i = 0; i < na; ++i) {
                    const bool in = off[x] + i < off[x + 1];
                    d[4 + 2 * i] = in ? arcs[2 * (size_t)(off[x] + i)] : 0xFFFFFFFFu;
                    d[5 + 2 * i] = in ? arcs[2 * (size_t)(off[x] + i) + 1] : 0u;
                }
                if (nodes[x] & kL1Bit) {  // level-1 closed form inputs
                    const uint32_t s1 = nodes[x] & ~kL1Bit;
                    d[16] = nodes_asc_host[s1];
                    d[17] = aoff[s1 + 1] - aoff[s1];
                    for (uint32_t i = 0; i < 4 && aoff[s1] + i < aoff[s1 + 1]; ++i) {
                        d[18 + 2 * i] = asc_arcs_host[2 * (size_t)(aoff[s1] + i)] & ~kLeafBit;
                        d[19 + 2 * i] = asc_arcs_host[2 * (size_t)(aoff[s1] + i) + 1];
                    }
                }
            }
            };
            {
                constexpr uint32_t kFillThreads = 8;
                const uint32_t per = (n + kFillThreads - 1u) / kFillThreads;
                std::vector<std::thread> ft;
                for (uint32_t t = 0; t < kFillThreads; ++t)
                    ft.emplace_back(fill, std::min(n, t * per), std::min(n, (t + 1u) * per));
                for (auto& t : ft) t.join();
            }
            g->dsc_desc.upload(desc.data(), desc.size(), s);
        }
        HIP_CHECK(hipStreamSynchronize(s));
        if (trace_on()) std::fprintf(stderr, "[cpd] graph down lists+desc %.3f s\n", now_seconds() - tg0);
        g->ch_arcs += arcs.size() / 2;
        g->narrow = env_on("CPD_NARROW") && p->dist_bound < 0xFFFFFFFEull;
        {
            std::vector<uint32_t> lb(g->npad / 32u, 0u);
            g->dsc_lvl_leaves.assign(g->dsc_lvl.size(), 0.0);
            for (uint32_t v = 0; v < n; ++v)
                if (p->ch.level_up[v] == 0) {
                    const uint32_t c = p->order[v];
                    lb[c >> 5] |= 1u << (c & 31u);
                    g->n_leaf += 1;
                    g->m_leaf += p->row_ptr[v + 1] - p->row_ptr[v];
                    g->dsc_lvl_leaves[p->ch.level_dn[v]] += 1;
                }
            g->leafbits.upload(lb.data(), lb.size(), s);
        }
        for (auto& b : g->bs) {
            b.stat.alloc(2 * (g->asc_lvl.size() + g->dsc_lvl.size()));
            b.stat_h.alloc(b.stat.n);
            std::fill(b.stat_h.p, b.stat_h.p + b.stat.n, 0u);
        }
        auto lvl_of = [n](const std::vector<uint32_t>& first) {
            std::vector<uint32_t> v(n, 0);
            for (size_t l = 0; l + 1 < first.size(); ++l)
                for (uint32_t x = first[l]; x < first[l + 1]; ++x) v[x] = (uint32_t)l;
            return v;
        };
        {
            // up levels of at most kNarrow nodes run chunked (CPD_UP_NARROW: A/B)
            static const uint32_t kNarrow = [] {
                const char* e = std::getenv("CPD_UP_NARROW");
                return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : 1024u;
            }();
            const uint32_t C = sweep_chunk_arcs();
            std::vector<uint32_t> items, slots;
            g->up_item_first.assign(g->asc_lvl.size(), 0);
            for (size_t l = 0; l + 1 < g->asc_lvl.size(); ++l) {
                g->up_item_first[l] = (uint32_t)(items.size() / 4);
                const uint32_t s0 = g->asc_lvl[l], s1 = g->asc_lvl[l + 1];
                if (l < 2 || s1 - s0 > kNarrow) continue;
                for (uint32_t x = s0; x < s1; ++x) {
                    slots.push_back(x);
                    for (uint32_t a = g->asc_off_host[x]; a < g->asc_off_host[x + 1]; a += C)
                        items.insert(items.end(),
                                     {x, a, std::min(a + C, g->asc_off_host[x + 1]), 0u});
                }
            }
            g->up_item_first.back() = (uint32_t)(items.size() / 4);
            g->up_items.upload(items.data(), items.size(), s);
            g->up_init_slots.upload(slots.data(), slots.size(), s);
            g->n_init_slots = (uint32_t)slots.size();
        }
        std::vector<uint32_t> la = lvl_of(g->asc_lvl), ld = lvl_of(g->dsc_lvl);
        g->asc_lvl_of.upload(la.data(), n, s);
        g->dsc_lvl_of.upload(ld.data(), n, s);
        HIP_CHECK(hipStreamSynchronize(s));
        if (trace_on()) std::fprintf(stderr, "[cpd] graph levels %.3f s\n", now_seconds() - tg0);
        *out = g.release();
    });
}

int cpd_graph_set_batch(cpd_graph* g, uint32_t batch) {
    return guarded([&] {
        CPD_REQUIRE(g, CPD_E_ARG, "null graph");
        CPD_REQUIRE(batch % 1024u == 0 && batch <= 32768u, CPD_E_ARG,
                    "batch must be a multiple of 1024, at most 32768");
        g->select();
        HIP_CHECK(hipStreamSynchronize(g->stream));
        g->reserve_batch(batch);
    });
}

int cpd_graph_set_hbm_reserve(cpd_graph* g, uint64_t bytes) {
    return guarded([&] {
        CPD_REQUIRE(g, CPD_E_ARG, "null graph");
        g->hbm_reserve = bytes;
    });
}

int cpd_graph_set_coords(cpd_graph* g, const int32_t* x, const int32_t* y) {
    return guarded([&] {
        CPD_REQUIRE(g, CPD_E_ARG, "null graph");
        if (!x || !y) {
            g->lane_key.clear();
            g->seg_order.release();
            return;
        }
        g->lane_key = hilbert_keys(x, y, g->n);
        if (seg_order_on()) {
            // first_moves gathers each column's out-neighbours' rows: with the
            // segments handed out in Hilbert order, the blocks one XCD runs at
            // once cover a compact patch of the graph and gather overlapping
            // rows (in DFS order a lattice node's cross neighbours are far)
            const uint32_t nseg = g->npad / 32u;
            std::vector<uint32_t> node_of(g->n);
            for (uint32_t v = 0; v < g->n; ++v) node_of[g->order[v]] = v;
            std::vector<uint64_t> kv(nseg);
            for (uint32_t sg = 0; sg < nseg; ++sg) {
                const uint32_t c = std::min(g->n - 1u, sg * 32u + 16u);
                kv[sg] = ((uint64_t)g->lane_key[node_of[c]] << 32) | sg;
            }
            std::sort(kv.begin(), kv.end());
            std::vector<uint32_t> so(nseg);
            for (uint32_t i = 0; i < nseg; ++i) so[i] = (uint32_t)kv[i];
            g->select();
            g->seg_order.upload(so.data(), nseg, g->stream);
            HIP_CHECK(hipStreamSynchronize(g->stream));
        }
    });
}

int cpd_graph_move_bits(const cpd_graph* g, uint32_t* bits) {
    return guarded([&] {
        CPD_REQUIRE(g && bits, CPD_E_ARG, "null argument");
        *bits = g->move_bits;
    });
}

int cpd_graph_get_batch(const cpd_graph* g, uint32_t* batch) {
    return guarded([&] {
        CPD_REQUIRE(g && batch, CPD_E_ARG, "null argument");
        *batch = g->B;
    });
}

void cpd_graph_free(cpd_graph* g) { delete g; }

}  // extern "C"

namespace {

// CPD_LIVE=0: no up-sweep row skipping; CPD_SORT=0: batches keep the caller's
// target order (A/B measurements; results are identical either way).
bool live_on() {
    static const bool on = env_on("CPD_LIVE");
    return on;
}
bool lane_key_on() {  // CPD_LANE_KEY=0: ignore cpd_graph_set_coords (A/B)
    static const bool on = env_on("CPD_LANE_KEY");
    return on;
}
bool seg_order_on() {  // CPD_FM_ORDER=0: first_moves takes segments in column order (A/B)
    static const bool on = env_on("CPD_FM_ORDER");
    return on;
}

// Hilbert-curve index of each node's (x, y), scaled to a 2^16 x 2^16 grid over
// the bounding box: nearby keys are nearby points, and any run of keys covers
// a compact region (the DFS column order follows the DFS tree, whose long
// branches and back-jumps spread a run of columns out).
std::vector<uint32_t> hilbert_keys(const int32_t* x, const int32_t* y, uint32_t n) {
    std::vector<uint32_t> key(n, 0);
    if (!n) return key;
    const int64_t x0 = *std::min_element(x, x + n), y0 = *std::min_element(y, y + n);
    const int64_t ext = std::max<int64_t>(*std::max_element(x, x + n) - x0,
                                          *std::max_element(y, y + n) - y0) + 1;
    constexpr uint32_t kSide = 1u << 16;
    for (uint32_t v = 0; v < n; ++v) {
        uint32_t px = (uint32_t)(((int64_t)x[v] - x0) * (kSide - 1) / ext);
        uint32_t py = (uint32_t)(((int64_t)y[v] - y0) * (kSide - 1) / ext);
        uint64_t d = 0;
        for (uint32_t s = kSide / 2; s > 0; s /= 2) {
            const uint32_t rx = (px & s) ? 1u : 0u, ry = (py & s) ? 1u : 0u;
            d += (uint64_t)s * s * ((3u * rx) ^ ry);
            if (ry == 0) {  // rotate the quadrant (only the lower bits matter from here)
                if (rx == 1) {
                    px = kSide - 1 - px;
                    py = kSide - 1 - py;
                }
                std::swap(px, py);
            }
        }
        key[v] = (uint32_t)d;
    }
    return key;
}

bool sort_on() {
    static const bool on = env_on("CPD_SORT");
    return on;
}
bool async_on() {  // CPD_ASYNC=0: every emit finishes before its batch returns
    static const bool on = env_on("CPD_ASYNC");
    return on;
}


// Distances + first-move sets for `k` targets (columns already in g->tgt,
// padded to a multiple of 1024 with valid columns).
bool trace_on();

// After a full narrow batch (g->ovf_h = its wide group rows): switch narrow
// rows off for good when most group rows had to be kept wide — the dense
// final rows replace the narrow rows and the pool (nothing may still read
// them: the caller has synchronised the main stream).  True if switched.
bool narrow_decide(cpd_graph* g) {
    const uint64_t groups = (uint64_t)g->n * (g->B / 256u);
    if (2ull * g->ovf_h() <= groups) return false;
    g->narrow = false;
    g->narrow_probe = 0;
    g->alloc_final_rows();
    if (trace_on())
        std::fprintf(stderr, "[cpd] narrow rows off: %u of %llu group rows wide\n", g->ovf_h(),
                     (unsigned long long)groups);
    return true;
}

// Phase U of a batch of k targets (slot's columns already uploaded), on
// stream st: the target mask, the leaf-form init of the chunked levels and the
// up-sweep levels, into the slot's up store, live and target masks — which
// only this slot's down-sweep reads: the caller orders st after the slot's
// previous batch (its first moves, ev_fm[slot]).
void launch_up(cpd_graph* g, uint32_t k, uint32_t slot, hipStream_t st) {
    const uint32_t B = g->B;
    auto& S = g->bs[slot];
    const uint32_t slabs = (k + 1023u) / 1024u;  // active 1024-target slabs
    const uint32_t active = slabs * 1024u;
    uint32_t* up = g->upx[slot].p;
    uint32_t* tmask = g->tmaskx[slot].p;
    uint32_t* live = live_on() ? g->livex[slot].p : nullptr;
    unsigned int* stat = g->timing ? S.stat.p : nullptr;
    const size_t nasc = g->asc_lvl.size();
    S.up_late.clear();
    if (stat) HIP_CHECK(hipMemsetAsync(stat, 0, S.stat.n * sizeof(unsigned int), st));
    if (live) {
        HIP_CHECK(hipMemsetAsync(tmask, 0, (size_t)g->n * sizeof(uint32_t), st));
        launch_target_mask(S.tgt.p, active, tmask, st);
        g->timed("sweep_up_init", 4.0 * g->n_init_slots * active, [&] {
            launch_sweep_up_init(g->up_init_slots.p, g->n_init_slots, g->asc_nodes.p, up, g->ubase,
                                 S.tgt.p, B, slabs, live, tmask, st);
        });
    }
    // ascending sweep: each level reads lower levels' rows.  Levels 0 and 1
    // are never materialised (closed forms, kLeafBit / kL1Bit): not launched.
    // Dense bytes per level: gathered rows 4 B x target, row writes 4 B x
    // target, arcs 8 B and node slot 12 B per 1024-target slab.  Sparse: 4 KiB
    // per live (row, slab) stored and per live row gathered, arcs 8 B + their
    // masks 4 B, node slot 12 B + masks 8 B, once per node — known once the
    // batch's live_stats have run (added by build_batch from S.up_late).
    g->group_begin("sweep_up", st);
    // bytes of level l (0 when they wait for the batch's stats)
    auto level_bytes = [&](size_t l) {
        const uint32_t s0 = g->asc_lvl[l], cnt = g->asc_lvl[l + 1] - s0;
        const double arcs_l = (double)(g->asc_off_host[g->asc_lvl[l + 1]] - g->asc_off_host[s0]);
        if (live && stat) {
            S.up_late.push_back({(double)l, arcs_l, (double)cnt});
            return 0.0;
        }
        return (4.0 * g->asc_lvl_arcs[l] + 4.0 * cnt) * active + 8.0 * arcs_l * slabs +
               12.0 * cnt * slabs;
    };
    auto items_of = [&](size_t l) { return g->up_item_first[l + 1] - g->up_item_first[l]; };
    for (size_t l = 2; l + 1 < nasc; ++l) {
        uint32_t s0 = g->asc_lvl[l], cnt = g->asc_lvl[l + 1] - s0;
        if (!cnt) continue;
        const uint32_t i0 = g->up_item_first[l], ni = items_of(l);
        const double dense = level_bytes(l);
        g->timed("sweep_up", dense, [&] {
            if (live && ni)
                launch_sweep_up_chunks(g->up_items.p + 4 * (size_t)i0, ni, g->asc_arcs.p, up,
                                       g->ubase, S.tgt.p, B, slabs, g->asc_nodes.p,
                                       g->asc_off.p, g->asc_arcs.p, live, tmask, st);
            else
                launch_sweep(true, g->asc_nodes.p, g->asc_off.p, g->asc_arcs.p, s0, cnt, nullptr,
                             up, g->ubase, nullptr, S.tgt.p, B, slabs, g->asc_nodes.p,
                             g->asc_off.p, g->asc_arcs.p, live, tmask, g->adj.p, g->adj_shift,
                             nullptr, g->narrow_rows(false), nullptr, st);
        });
    }
    g->group_end();
}

// Fold the late bytes of all but the newest `keep` batches: their stats
// (stat_h of their slot) have landed — the caller has seen a later point of
// the main stream (the next batch's down-sweep end, or a full sync).
void fold_late(cpd_graph* g, size_t keep) {
    while (g->late_q.size() > keep) {
        const auto& rec = g->late_q.front();
        const unsigned int* sh = g->bs[rec.slot].stat_h.p;
        double up = 0.0, down = 0.0;
        for (const auto& u : rec.up) {
            const size_t l = (size_t)u[0];
            up += 4096.0 * ((double)sh[2 * l] + (double)sh[2 * l + 1]) + 12.0 * u[1] + 20.0 * u[2];
        }
        for (const auto& d : rec.down) down += 4096.0 * (double)sh[(size_t)d[0]] + d[1];
        g->agg["sweep_up"].bytes += up;
        g->agg["sweep_down"].bytes += down;
        g->late_q.erase(g->late_q.begin());
    }
}

// Phase D of the batch in `slot` (its up-sweep done or ordered before), on
// g->stream: the down-sweep (own rows from the slot's up store), the pool
// rows it took (narrow; the count lands in g->ovf_h), the live stats
// (timing runs), then ev_down.
void launch_down(cpd_graph* g, uint32_t k, bool narrow, uint32_t slot) {
    const uint32_t B = g->B, n = g->n;
    auto& S = g->bs[slot];
    const NarrowRows nr = g->narrow_rows(narrow);
    if (narrow) HIP_CHECK(hipMemsetAsync(g->ovf.p, 0, sizeof(uint32_t), g->stream));
    // bytes per target of a final-distance row access: 4 wide; 2 + a 4-B base
    // per 256 targets narrow
    const double drow = narrow ? 2.0 + 4.0 / 256.0 : 4.0;
    const uint32_t slabs = (k + 1023u) / 1024u;  // active 1024-target slabs
    const uint32_t active = slabs * 1024u;
    uint32_t* live = live_on() ? g->livex[slot].p : nullptr;
    unsigned int* stat = g->timing ? S.stat.p : nullptr;
    const size_t nasc = g->asc_lvl.size();
    cpd_graph::LateRec rec;
    rec.slot = slot;
    rec.up.swap(S.up_late);  // this batch's up levels (launch_up)
    g->group_begin("sweep_down", g->stream);
    for (size_t l = 0; l + 1 < g->dsc_lvl.size(); ++l) {
        uint32_t s0 = g->dsc_lvl[l], cnt = g->dsc_lvl[l + 1] - s0;
        if (!cnt) continue;
        const size_t si = 2 * (nasc + l);
        double base = (drow * g->dsc_lvl_arcs[l] + drow * cnt) * active +
                      8.0 * g->dsc_lvl_arcs[l] * slabs + 12.0 * cnt * slabs;
        if (g->leaf_fm) base += 0.5 * g->dsc_lvl_leaves[l] * active;  // leaf sets
        double dense = base + 4.0 * g->dsc_lvl_reads[l] * active;
        if (live && stat) {  // own rows: 4 KiB per live (row, slab), counted by live_stats
            rec.down.push_back({(double)si, 4.0 * g->dsc_lvl_reads[l] * slabs});
            dense = base;
        }
        g->timed("sweep_down", dense, [&] {
            launch_sweep(false, g->dsc_nodes.p, g->dsc_off.p, g->dsc_arcs.p, s0, cnt, g->dist.p,
                         g->upx[slot].p, g->ubase, g->dsc_up.p, S.tgt.p, B, slabs, g->asc_nodes.p,
                         g->asc_off.p, g->asc_arcs.p, live, g->tmaskx[slot].p, g->adj.p,
                         g->adj_shift, g->leaf_fm ? g->fmleaf.p : nullptr, nr, g->dsc_desc.p,
                         g->stream);
        });
    }
    g->group_end();
    if (stat) g->late_q.push_back(std::move(rec));
    if (narrow)
        HIP_CHECK(hipMemcpyAsync(g->ovf_hb.p, g->ovf.p, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                 g->stream));
    if (live && stat && nasc > 2) {  // row counts behind the late byte counts
        g->timed("live_stats", 0.0, [&] {
            launch_live_stats(true, g->asc_nodes.p, g->asc_off.p, g->asc_arcs.p,
                              g->asc_lvl_of.p, g->asc_lvl[2], n, g->ubase, g->dsc_up.p, live,
                              stat, g->stream);
        });
        g->timed("live_stats", 0.0, [&] {
            launch_live_stats(false, g->dsc_nodes.p, g->dsc_off.p, g->dsc_arcs.p,
                              g->dsc_lvl_of.p, 0, n, g->ubase, g->dsc_up.p, live,
                              stat + 2 * nasc, g->stream);
        });
    }
    // the slot is free for the batch after next once these land: its targets
    // copied for the first moves, the stats copied out
    HIP_CHECK(hipMemcpyAsync(g->fm_tgt.p, S.tgt.p, (size_t)B * sizeof(uint32_t),
                             hipMemcpyDeviceToDevice, g->stream));
    if (stat)
        HIP_CHECK(hipMemcpyAsync(S.stat_h.p, stat, S.stat.n * sizeof(unsigned int),
                                 hipMemcpyDeviceToHost, g->stream));
    HIP_CHECK(hipEventRecord(g->ev_down, g->stream));
}

// Phase F: the first moves of the batch in `slot` into fm (after its
// down-sweep on g->stream), then ev_fm[slot]; the timing stats' copy.
void launch_fm(cpd_graph* g, uint32_t k, bool narrow, uint32_t* fm, uint32_t slot) {
    const uint32_t B = g->B, n = g->n;
    const NarrowRows nr = g->narrow_rows(narrow);
    const double drow = narrow ? 2.0 + 4.0 / 256.0 : 4.0;
    // per row: own distance 4n (kernels that read it) + neighbour distances
    // 4m + first-move write npad * fmb / 8; the packed adjacency (8 B per
    // slot) is read once per 1024-target slab.  Leaf columns (leaf_fm) read
    // 0.5 B of sets instead of their own and neighbour distances.
    const uint32_t fslabs = (k + 1023u) / 1024u;
    const double nl = g->leaf_fm ? g->n_leaf : 0.0, ml = g->leaf_fm ? g->m_leaf : 0.0;
    const double own = first_moves_reads_own(g->adj_shift, narrow) ? drow * (n - nl) : 0.0;
    double fbytes =
        (own + drow * (g->m - ml) + 0.5 * nl + g->fmb / 8.0 * g->npad) *
            (fslabs * 1024.0) +
        8.0 * (double)(n - nl) * (double)(1u << g->adj_shift) * fslabs + 4.0 * g->npad / 32.0;
    g->timed("first_moves", fbytes, [&] {
        launch_first_moves(g->adj.p, g->adj_shift, g->dist.p, g->fm_tgt.p, B, k, n, g->npad,
                           fm, g->leaf_fm ? g->leafbits.p : nullptr,
                           g->leaf_fm ? g->fmleaf.p : nullptr, nr, g->stream, g->seg_order.p);
    });
    HIP_CHECK(hipEventRecord(g->ev_fm[slot], g->stream));
}

void launch_down_fm(cpd_graph* g, uint32_t k, bool narrow, uint32_t* fm, uint32_t slot) {
    launch_down(g, k, narrow, slot);
    launch_fm(g, k, narrow, fm, slot);
}

// Upload a batch's targets as columns into `slot`, on stream st.  With
// sorting on, lanes hold the targets in column order (DFS preorder is
// spatially coherent, so a 1024-lane slab covers one compact region and the
// up-sweep skips most rows); pos_of[i] = lane of the caller's target i.
// The batch's lane order and columns into the slot's host buffers (host
// work only; upload_targets copies them to the device).
void prepare_targets(cpd_graph* g, const uint32_t* targets, uint32_t k, uint32_t slot) {
    auto& S = g->bs[slot];
    CPD_REQUIRE(g->has_ch, CPD_E_ARG,
                "graph was created from a plan without hierarchy: it can serve queries "
                "but not build rows");
    std::vector<uint32_t> cols(g->B), idx(k);
    for (uint32_t i = 0; i < k; ++i) {
        CPD_REQUIRE(targets[i] < g->n, CPD_E_ARG,
                    "target " + std::to_string(targets[i]) + " out of range");
        idx[i] = i;
    }
    if (sort_on() && k > 0) {
        // lanes by (Hilbert key, column), or by column without coordinates:
        // compact 2-D groups — a 256-lane group spans a small square, so its
        // final distances fit the narrow rows' 16-bit offsets (column order:
        // 5.5% of group rows wide on the 1M-node bench batch).
        // A stable LSD radix sort of the 64-bit keys (a comparison sort of a
        // 16k batch took ~1.7 ms of host time between two batches' kernels).
        const bool hk = !g->lane_key.empty() && lane_key_on();
        std::vector<uint64_t> kv(k), kt(k);
        std::vector<uint32_t> it(k);
        for (uint32_t i = 0; i < k; ++i)
            kv[i] = ((hk ? (uint64_t)g->lane_key[targets[i]] : 0ull) << 32) |
                    g->order[targets[i]];
        for (int pass = 0; pass < (hk ? 8 : 4); ++pass) {
            const int sh = 8 * pass;
            uint32_t cnt[257] = {0};
            for (uint32_t i = 0; i < k; ++i) ++cnt[((kv[i] >> sh) & 0xFFu) + 1];
            if (cnt[((kv[0] >> sh) & 0xFFu) + 1] == k) continue;  // one digit value: no-op
            for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
            for (uint32_t i = 0; i < k; ++i) {
                const uint32_t pos = cnt[(kv[i] >> sh) & 0xFFu]++;
                kt[pos] = kv[i];
                it[pos] = idx[i];
            }
            kv.swap(kt);
            idx.swap(it);
        }
    }
    S.pos_of.resize(k);
    for (uint32_t p = 0; p < k; ++p) {
        cols[p] = g->order[targets[idx[p]]];
        S.pos_of[idx[p]] = p;
    }
    for (uint32_t i = k; i < g->B; ++i) cols[i] = cols[0];  // padding lanes
    S.tgt_col = cols;
    std::copy(cols.begin(), cols.end(), S.tgt_h.p);
}

void upload_targets(cpd_graph* g, const uint32_t* targets, uint32_t k, uint32_t slot,
                    hipStream_t st, bool prepared = false) {
    if (!prepared) prepare_targets(g, targets, k, slot);
    auto& S = g->bs[slot];
    HIP_CHECK(hipMemcpyAsync(S.tgt.p, S.tgt_h.p, (size_t)g->B * sizeof(uint32_t),
                             hipMemcpyHostToDevice, st));
}


// CPD_OVERLAP=0: no early up-sweep of the next batch (A/B; identical rows).
bool overlap_on() {
    static const bool on = env_on("CPD_OVERLAP");
    return on;
}

// CPD_TRACE=1: host-side phase times of every batch on stderr.
bool trace_on() {
    static const bool on = [] {
        const char* e = std::getenv("CPD_TRACE");
        return e && *e && *e != '0';
    }();
    return on;
}

// Build rows for one batch of k <= B targets; append to r (device).  next /
// next_k (may be null / 0): the targets of the batch that follows; its
// up-sweep is queued first, on ustream behind this batch's own: it writes
// the other slot's up store, so it starts as soon as this batch's up-sweep
// ends — with this batch's down-sweep — and runs beside it.
void build_batch(cpd_graph* g, const uint32_t* targets, uint32_t k, cpd_rows* r,
                 const uint32_t* next, uint32_t next_k) {
    const double t0 = now_seconds();
    uint32_t slot;
    if (g->prepped && g->prep_targets.size() == k &&
        std::equal(targets, targets + k, g->prep_targets.begin())) {
        slot = g->prep_slot;  // up-sweep launched by the previous batch
        HIP_CHECK(hipStreamWaitEvent(g->stream, g->ev_up, 0));
        g->prepped = false;
    } else {
        if (g->prepped) g->drop_prep();
        slot = g->next_slot;
        upload_targets(g, targets, k, slot, g->stream);
        launch_up(g, k, slot, g->stream);
    }
    g->next_slot = slot ^ 1u;
    const uint32_t npad = g->npad;
    const double fm_row = g->fmb / 8.0 * npad;  // first-move bytes per row
    // + per 32-column segment a 4-B entry state and a 1-B count (fmb == 4)
    const double st_row = 5.0 * npad / 32.0;
    const bool narrow = g->narrow;
    // The next batch's up-sweep (ustream, high priority) into the other slot,
    // after that slot's last batch's down-sweep (the last reader of the
    // slot's targets, up store, masks and stats; its first moves read the
    // targets from fm_tgt).  The host queues it as soon as this batch starts:
    // it runs beside the previous batch's first moves, ahead of this
    // down-sweep, which the host's launch latency then never delays.
    const uint32_t ns = slot ^ 1u;
    if (next && next_k && overlap_on()) {
        prepare_targets(g, next, next_k, ns);
        // after the other slot's last batch: its down-sweep (ev_down, not yet
        // re-recorded for this batch), so this up-sweep runs beside its first
        // moves (after them, ev_fm[ns], it ran beside this down-sweep: with
        // the one-row emit the same rows/s within noise, 371.9-376.9k against
        // 374.6-377.1k, profiles/up_store_ab/r06k_*; with the eight-row emit
        // 414.2-415.1k against 413.2-423.4k, the down-sweep's launches 12%
        // longer, r06o_*; with first_moves at 8 waves per SIMD 419.0-420.5k
        // against 425.2-431.7k, r06z_*)
        HIP_CHECK(hipStreamWaitEvent(g->ustream, g->ev_down, 0));
        upload_targets(g, next, next_k, ns, g->ustream, true);
        launch_up(g, next_k, ns, g->ustream);
        HIP_CHECK(hipEventRecord(g->ev_up, g->ustream));
        g->prepped = true;
        g->prep_slot = ns;
        g->prep_targets.assign(next, next + next_k);
    }
    launch_down(g, k, narrow, slot);
    // the first moves' buffer set, once the emit that last read it is done
    const uint32_t x = g->acquire_set();
    uint32_t* fm = g->fmx[x].p;
    uint32_t* rst = g->rle_stx[x].p;
    uint8_t* rrc = g->rle_rcx[x].p;
    launch_fm(g, k, narrow, fm, slot);
    const double t1 = now_seconds();
    // Narrow rows: the pool rows the down-sweep took (wide group rows).  Past
    // the pool the batch is rebuilt below; the first full batches decide
    // whether narrow rows pay at all (narrow_decide).
    // (The host waits for this down-sweep in any case: the next batch's
    // target staging buffers are then free.)
    HIP_CHECK(hipEventSynchronize(g->ev_down));  // g->ovf_h has landed
    bool rebuild = false;
    if (narrow) {
        const uint64_t groups = (uint64_t)g->n * (g->B / 256u);
        if (g->timing) {  // group rows kept wide / all group rows
            g->agg["wide_rows"].launches += g->ovf_h();
            g->agg["group_rows"].launches += groups;
        }
        if (g->timing) g->agg["emit_sets"].launches = g->nsets;  // the emit overlap's depth
        rebuild = g->ovf_h() > g->pool_cap;
        if (g->narrow_probe && k == g->B) {
            --g->narrow_probe;
            if (2ull * g->ovf_h() > groups) {
                HIP_CHECK(hipStreamSynchronize(g->stream));  // nothing reads the narrow rows
                narrow_decide(g);
            }
        }
    }
    if (rebuild) {
        // This batch's rows are not emitted: they are built again, with the
        // dense rows when narrow rows were just switched off, else in pieces
        // of pool_cap / (4 n) slabs, whose group rows all fit the pool.
        HIP_CHECK(hipStreamSynchronize(g->stream));
        g->drop_prep();
        if (g->timing) g->agg["pool_rebuilds"].launches += 1;
        if (trace_on())
            std::fprintf(stderr, "[cpd] batch of %u rows: %u wide group rows past the pool's %u, rebuilt\n",
                         k, g->ovf_h(), g->pool_cap);
        const uint32_t piece =
            g->narrow ? std::min(g->B, std::max(1024u, (uint32_t)(g->pool_cap / (4ull * g->n)) * 1024u))
                      : g->B;
        for (uint32_t b = 0; b < k; b += piece) {
            const uint32_t kk = std::min(piece, k - b);
            const bool last = b + kk >= k;
            build_batch(g, targets + b, kk, r, last ? next : targets + b + kk,
                        last ? next_k : std::min(piece, k - b - kk));
        }
        return;
    }
    const double t2 = now_seconds();
    // The count, the seam repair and the move-table emit of this batch go to
    // the emit stream (estream; `stream` when the overlap is off), after its
    // first moves (ev_fm): they run beside the next batch's sweeps, and the
    // run counts land in a page-locked buffer the rows settle from later
    // (cpd_rows::settle) — the host waits for none of it here.
    hipStream_t es = g->async ? g->estream : g->stream;
    if (es != g->stream) HIP_CHECK(hipStreamWaitEvent(es, g->ev_fm[slot], 0));
    // the batch's rows become table rows r->nrows + i, written by lane pos_of[i]
    const std::vector<uint32_t>& pos_of = g->bs[slot].pos_of;
    CPD_REQUIRE(r->moves.n >= (size_t)(r->nrows + k) * r->wpr, CPD_E_ARG,
                "rows: move table capacity");
    cpd_rows::Batch* rb = r->new_batch(g->B);
    rb->k = k;
    rb->pos_of.assign(pos_of.begin(), pos_of.begin() + k);
    for (uint32_t i = 0; i < k; ++i) rb->lane_rows.p[pos_of[i]] = r->nrows + i;
    auto emit = [=]() {
        HIP_CHECK(hipMemcpyAsync(g->lane_rowx[x].p, rb->lane_rows.p, k * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, es));
        const uint32_t nch = g->fmb == 4 ? rle_count_chunks(npad) : 0u;
        if (rle_fused(g->fmb)) {
            // one pass: each set read once, the tables written, the run counts
            // summed from the chunks (rle_emit4 + the seam check rle_emit_fix)
            const uint32_t ec = rle_emit_chunks(npad);
            const size_t cks = (size_t)k * ec;
            g->timed("rle_emit", (fm_row + 4.0 * r->wpr) * k + 24.0 * cks + 8.0 * k, [&] {
                launch_rle_emit(fm, npad, k, g->lane_rowx[x].p, r->tlb, r->moves.p, g->emit_ck.p,
                                g->emit_ck.p + cks, g->emit_ck.p + 2 * cks, g->counts.p, es);
            });
            HIP_CHECK(hipMemcpyAsync(rb->counts.p, g->counts.p, k * sizeof(uint32_t),
                                     hipMemcpyDeviceToHost, es));
            HIP_CHECK(hipEventRecord(rb->ev, es));
        } else {  // the count, the seam repair and the emit (8/16-bit sets, or CPD_RLE_FUSED=0)
            if (nch) {  // chunked count + seam repair (rescans are rare and not counted)
                HIP_CHECK(hipMemsetAsync(g->rle_hard.p, 0, sizeof(uint32_t), es));
                g->timed("rle_count", (fm_row + st_row + 12.0 * nch) * k, [&] {
                    launch_rle_count_ch(fm, npad, k, rst, rrc, g->rle_xs.p, g->rle_cc.p, es);
                });
                g->timed("rle_fix", (12.0 * nch + 4.0) * k, [&] {
                    launch_rle_fix(fm, npad, k, rst, rrc, g->rle_xs.p, g->rle_cc.p, g->counts.p,
                                   g->rle_hard.p, es);
                });
                // runs too long for the seam repair: the bounded pass, which does
                // nothing unless rle_fix raised rle_hard
                g->timed("rle_recount", 0.0, [&] {
                    launch_rle_count(fm, g->fmb, npad, k, g->counts.p, rst, rrc, es, g->rle_hard.p);
                });
            } else {
                g->timed("rle_count", (fm_row + st_row) * k + 4.0 * k, [&] {
                    launch_rle_count(fm, g->fmb, npad, k, g->counts.p, rst, rrc, es);
                });
            }
            HIP_CHECK(hipMemcpyAsync(rb->counts.p, g->counts.p, k * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                     es));
            HIP_CHECK(hipEventRecord(rb->ev, es));
            // per row: the sets (fm_row), the segment states (4 B per 32 columns;
            // the run counts are read only where the look-ahead needs them), the
            // table (npad * bits / 8)
            const double ebytes = (fm_row + 4.0 * npad / 32.0 + 4.0 * r->wpr) * k + 4.0 * k;
            g->timed("rle_moves", ebytes, [&] {
                launch_rle_moves(fm, g->fmb, npad, k, rst, rrc, g->lane_rowx[x].p, r->tlb, r->moves.p, es);
            });
        }
        if (!r->done) HIP_CHECK(hipEventCreateWithFlags(&r->done, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(r->done, es));
        if (g->async) {
            HIP_CHECK(hipEventRecord(g->ev_emit[x], es));
            g->emit_pending[x] = true;
        }
    };
    emit();
    // the previous batch's sweep bytes: its stats landed before this down-sweep
    if (g->timing) fold_late(g, 1);
    if (trace_on())
        std::fprintf(stderr, "[cpd] batch %u rows: launch sweeps+fm %.2f ms, to down-sweep end %.2f "
                             "ms, count+emit queued %.2f ms\n",
                     k, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (now_seconds() - t2) * 1e3);
    r->targets.insert(r->targets.end(), targets, targets + k);
    r->lanes.insert(r->lanes.end(), pos_of.begin(), pos_of.begin() + k);
    r->nrows += k;
}

}  // namespace

extern "C" {

int cpd_build_rows(cpd_graph* g, const uint32_t* targets, uint32_t ntargets,
                   cpd_rows* reuse, cpd_rows** out) {
    return guarded([&] {
        CPD_REQUIRE(g && out && (targets || ntargets == 0), CPD_E_ARG, "build: null argument");
        *out = nullptr;
        g->select();
        if (!g->B) g->reserve_batch(0);
        cpd_rows* r = reuse ? reuse : new cpd_rows();
        std::unique_ptr<cpd_rows> owned(reuse ? nullptr : r);
        r->device = g->device;
        r->retire();  // an earlier build's unsettled batches (copies may be in flight)
        r->nrows = 0;
        r->total = 0;
        r->targets.clear();
        r->lanes.clear();
        r->offsets.assign(1, 0);
        r->n = g->n;
        // built rows at the graph's packed width (2 bits per column on the
        // bench graph): the register-resident fused emit writes them with
        // 16-B stores, half the bytes of nibble tables (6.2 against 12.3 GB
        // per 24576-row step), and the export and an index take them as
        // they are (round 4 built nibble tables and narrowed them on the way
        // out, when narrowing cost the unfused emit ~0.5 ms)
        r->tlb = g->tlb;
        r->wpr = g->npad >> (5u - r->tlb);
        r->bits = g->move_bits;
        if (r->moves.n < (size_t)ntargets * r->wpr) {
            r->wait();  // an earlier build's emit may still write the old table
            ArenaScope carve;
            r->moves.alloc((size_t)ntargets * r->wpr);
        }
        for (uint32_t b = 0; b < ntargets; b += g->B) {
            uint32_t k = std::min(g->B, ntargets - b);
            const uint32_t* next = nullptr;
            uint32_t next_k = 0;
            if (b + k < ntargets) {  // the call's own next batch
                next = targets + b + k;
                next_k = std::min(g->B, ntargets - b - k);
            } else if (!g->hint.empty()) {  // the next call's first batch
                next = g->hint.data();
                next_k = (uint32_t)std::min<size_t>(g->B, g->hint.size());
            }
            build_batch(g, targets + b, k, r, next, next_k);
        }
        g->hint.clear();
        owned.release();
        *out = r;
    });
}

int cpd_graph_hint_next(cpd_graph* g, const uint32_t* targets, uint32_t ntargets) {
    return guarded([&] {
        CPD_REQUIRE(g && (targets || ntargets == 0), CPD_E_ARG, "hint: null argument");
        for (uint32_t i = 0; i < ntargets; ++i)
            CPD_REQUIRE(targets[i] < g->n, CPD_E_ARG, "hint: target out of range");
        g->hint.assign(targets, targets + ntargets);
    });
}

int cpd_rows_count(const cpd_rows* r, uint32_t* nrows, uint64_t* total_runs) {
    return guarded([&] {
        CPD_REQUIRE(r, CPD_E_ARG, "null rows");
        if (total_runs) r->settle();
        if (nrows) *nrows = r->nrows;
        if (total_runs) *total_runs = r->total;
    });
}

int cpd_rows_wait(const cpd_rows* r) {
    return guarded([&] {
        CPD_REQUIRE(r, CPD_E_ARG, "null rows");
        r->settle();
    });
}

int cpd_rows_export(const cpd_rows* r, uint64_t* offsets, uint32_t* runs) {
    return cpd_rows_export_range(r, 0, r ? r->nrows : 0, offsets, runs);
}

int cpd_rows_export_range(const cpd_rows* r, uint32_t first, uint32_t count, uint64_t* offsets,
                          uint32_t* runs) {
    return guarded([&] {
        CPD_REQUIRE(r, CPD_E_ARG, "null rows");
        CPD_REQUIRE(first <= r->nrows && count <= r->nrows - first, CPD_E_ARG,
                    "export range: rows out of range");
        r->settle();
        const uint64_t base = r->offsets[first], end = r->offsets[first + count];
        if (offsets)
            for (uint32_t i = 0; i <= count; ++i) offsets[i] = r->offsets[first + i] - base;
        if (!runs || end == base) return;
        HIP_CHECK(hipSetDevice(r->device));
        hipStream_t st = thread_stream(r->device);
        // decode piece by piece (<= kDecodeRuns runs, a longer row alone) into
        // a staging buffer of the rows' pool, then copy out
        auto stage = r->acquire_stage();
        for (uint32_t p0 = first; p0 < first + count;) {
            uint32_t p1 = p0 + 1;
            while (p1 < first + count && r->offsets[p1 + 1] - r->offsets[p0] <= kDecodeRuns) ++p1;
            const uint64_t nr = r->offsets[p1] - r->offsets[p0];
            stage->alloc(std::max<uint64_t>(nr, std::min<uint64_t>(end - base, kDecodeRuns)));
            launch_moves_runs(r->moves.p + (size_t)p0 * r->wpr, r->wpr, r->tlb, r->n, p1 - p0,
                              r->off.p + p0, r->offsets[p0], stage->p, st);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyAsync(runs + (r->offsets[p0] - base), stage->p, nr * sizeof(uint32_t),
                                     hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            p0 = p1;
        }
        r->release_stage(std::move(stage));
    });
}

int cpd_rows_move_words(const cpd_rows* r, uint32_t* words) {
    return guarded([&] {
        CPD_REQUIRE(r && words, CPD_E_ARG, "null argument");
        *words = r->packed_words();
    });
}

int cpd_rows_move_bits(const cpd_rows* r, uint32_t* bits) {
    return guarded([&] {
        CPD_REQUIRE(r && bits, CPD_E_ARG, "null argument");
        *bits = r->bits;
    });
}

int cpd_rows_export_moves(const cpd_rows* r, uint32_t first, uint32_t count, uint32_t* moves) {
    return guarded([&] {
        CPD_REQUIRE(r && (moves || count == 0), CPD_E_ARG, "null argument");
        CPD_REQUIRE(first <= r->nrows && count <= r->nrows - first, CPD_E_ARG,
                    "export range: rows out of range");
        if (!count) return;
        HIP_CHECK(hipSetDevice(r->device));
        r->wait();
        hipStream_t st = thread_stream(r->device);
        const size_t w = r->packed_words();
        const uint32_t* src = r->moves.p + (size_t)first * r->wpr;
        if (w == r->wpr && r->bits == (1u << r->tlb)) {  // the tables as they are
            HIP_CHECK(hipMemcpyAsync(moves, src, (size_t)count * w * sizeof(uint32_t),
                                     hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            return;
        }
        // rows made contiguous at the exported width on the GPU (a pitched
        // device copy when the widths agree, else repacked), then one copy out
        auto stage = r->acquire_stage();
        stage->alloc((size_t)count * w);
        if (r->bits == (1u << r->tlb))
            HIP_CHECK(hipMemcpy2DAsync(stage->p, w * sizeof(uint32_t), src,
                                       (size_t)r->wpr * sizeof(uint32_t), w * sizeof(uint32_t),
                                       count, hipMemcpyDeviceToDevice, st));
        else
            launch_repack_moves(src, r->wpr, r->wpr, 1u << r->tlb, count, stage->p, (uint32_t)w,
                                (uint32_t)w, r->bits, st);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(moves, stage->p, (size_t)count * w * sizeof(uint32_t),
                                 hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        r->release_stage(std::move(stage));
    });
}

int cpd_host_alloc(size_t bytes, void** out) {
    return guarded([&] {
        CPD_REQUIRE(out, CPD_E_ARG, "host alloc: null output");
        *out = nullptr;
        require_device();
        HIP_CHECK(hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault));
    });
}

void cpd_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int cpd_rows_targets(const cpd_rows* r, uint32_t* targets) {
    return guarded([&] {
        CPD_REQUIRE(r && targets, CPD_E_ARG, "null argument");
        std::memcpy(targets, r->targets.data(), r->nrows * sizeof(uint32_t));
    });
}

int cpd_rows_lanes(const cpd_rows* r, uint32_t* lanes) {
    return guarded([&] {
        CPD_REQUIRE(r && lanes, CPD_E_ARG, "null argument");
        std::memcpy(lanes, r->lanes.data(), r->nrows * sizeof(uint32_t));
    });
}

void cpd_rows_free(cpd_rows* r) {
    if (r) (void)hipSetDevice(r->device);
    delete r;
}

int cpd_debug_rows(cpd_graph* g, const uint32_t* targets, uint32_t ntargets, uint32_t* dist,
                   uint16_t* fm) {
    return guarded([&] {
        CPD_REQUIRE(g && targets, CPD_E_ARG, "debug: null argument");
        g->select();
        if (!g->B) g->reserve_batch(0);
        CPD_REQUIRE(ntargets > 0 && ntargets <= g->B, CPD_E_ARG, "debug: 0 < ntargets <= batch");
        if (g->prepped) g->drop_prep();
        const uint32_t slot = g->next_slot;
        upload_targets(g, targets, ntargets, slot, g->stream);
        launch_up(g, ntargets, slot, g->stream);
        uint32_t x = 0;
        for (;;) {
            x = g->acquire_set();
            const bool narrow = g->narrow;
            launch_down_fm(g, ntargets, narrow, g->fmx[x].p, slot);
            g->sync();
            // wide group rows past the pool: again with the dense rows
            if (!narrow || g->ovf_h() <= g->pool_cap) break;
            g->ovf_hb.p[0] = 2u * g->n * (g->B / 256u);
            narrow_decide(g);
        }
        fold_late(g, 0);
        const std::vector<uint32_t>& pos_of = g->bs[slot].pos_of;
        const std::vector<uint32_t>& tgt_col = g->bs[slot].tgt_col;
        const uint32_t n = g->n, B = g->B;
        // lane p holds the caller's target i = pos_of^-1(p)
        std::vector<uint32_t> h((size_t)n * B);
        if (!g->narrow) {
            HIP_CHECK(hipMemcpy(h.data(), g->dist.p, h.size() * sizeof(uint32_t),
                                hipMemcpyDeviceToHost));
        } else {  // base + u16 offset (0xFFFF = unreachable), or a pool row
            std::vector<uint16_t> q((size_t)n * B);
            std::vector<uint32_t> b((size_t)n * (B / 256u));
            std::vector<uint32_t> pr((size_t)std::min(g->ovf_h(), g->pool_cap) * 256u);
            HIP_CHECK(hipMemcpy(q.data(), g->d16.p, q.size() * sizeof(uint16_t),
                                hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(b.data(), g->dbase.p, b.size() * sizeof(uint32_t),
                                hipMemcpyDeviceToHost));
            if (!pr.empty())
                HIP_CHECK(hipMemcpy(pr.data(), g->pool.p, pr.size() * sizeof(uint32_t),
                                    hipMemcpyDeviceToHost));
            for (uint32_t c = 0; c < n; ++c)
                for (uint32_t p = 0; p < B; ++p) {
                    const uint32_t base = b[(size_t)(p / 256u) * n + c];
                    if (base == 0xFFFFFFFEu) {  // kept wide: the pool row in its d16 words
                        const size_t w = ((size_t)c * B + (p & ~1u)) / 2u * 2u;
                        const uint32_t idx = (uint32_t)q[w] | ((uint32_t)q[w + 1] << 16);
                        h[(size_t)c * B + p] = pr[(size_t)idx * 256u + (p & 255u)];
                        continue;
                    }
                    const uint16_t d = q[(size_t)c * B + p];
                    h[(size_t)c * B + p] = d == 0xFFFFu ? CPD_INF : base + d;
                }
        }
        if (dist)
            for (uint32_t v = 0; v < n; ++v)
                for (uint32_t i = 0; i < ntargets; ++i)
                    dist[(size_t)v * ntargets + i] = h[(size_t)g->order[v] * B + pos_of[i]];
        if (fm) {
            // unpack fmb-bit sets; a column whose set is the wildcard (the
            // target, unreachable columns) reports CPD_FM_ALL like the oracle
            const uint32_t per = 32u / g->fmb, all = (1u << g->fmb) - 1u;
            const size_t row_words = g->npad / per;
            std::vector<uint32_t> w((size_t)B * row_words);
            HIP_CHECK(hipMemcpy(w.data(), g->fmx[x].p, w.size() * sizeof(uint32_t),
                                hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < ntargets; ++i) {
                const uint32_t p = pos_of[i];
                for (uint32_t v = 0; v < n; ++v) {
                    const uint32_t c = g->order[v];
                    // 4-bit rows are row-group interleaved (cpd_kernels.hip
                    // fm4_piece): 16-B piece (p/4, segment c/32, p%4)
                    const size_t wi =
                        g->fmb == 4 ? ((((size_t)(p >> 2) * (g->npad / 32u) + c / 32u) * 4u +
                                        (p & 3u)) * 4u + (c % 32u) / 8u)
                                    : (size_t)p * row_words + c / per;
                    const uint32_t f = (w[wi] >> (g->fmb * (c % per))) & all;
                    const bool wild = c == tgt_col[p] || h[(size_t)c * B + p] == CPD_INF;
                    fm[(size_t)i * n + v] = wild ? (uint16_t)CPD_FM_ALL : (uint16_t)f;
                }
            }
        }
    });
}

// ---------------------------------------------------------------------------
// Index + queries

}  // extern "C"

namespace {

// Runs staged per host chunk of a streamed dense index (a row larger than
// this is staged alone).
constexpr uint64_t kStageRuns = 1ull << 28;  // 1 GiB

std::unique_ptr<cpd_index> index_init(cpd_graph* g, const uint32_t* row_targets, uint32_t nrows) {
    CPD_REQUIRE(nrows == 0 || row_targets, CPD_E_ARG, "index: null row targets");
    auto ix = std::make_unique<cpd_index>();
    ix->g = g;
    ix->nrows = nrows;
    ix->row_of_col.assign(g->n, CPD_INF);
    if (nrows) ix->row_targets.assign(row_targets, row_targets + nrows);
    for (uint32_t i = 0; i < nrows; ++i) {
        CPD_REQUIRE(row_targets[i] < g->n, CPD_E_ARG, "index: row target out of range");
        ix->row_of_col[g->order[row_targets[i]]] = i;
    }
    ix->offsets.assign(1, 0);
    ix->d_row_of_col.upload(ix->row_of_col.data(), g->n, g->stream);
    ix->agg.alloc(4);
    ix->flag.alloc(1);
    return ix;
}

void index_keep_rle(cpd_index* ix, uint64_t cap) {
    ix->keep_rle = true;
    ix->stream_dense = false;
    ix->cap = cap;
    ix->runs.alloc(cap);
    ix->off.alloc((size_t)ix->nrows + 1);
    HIP_CHECK(hipMemsetAsync(ix->off.p, 0, sizeof(uint64_t), ix->g->stream));
}

void index_stream_dense(cpd_index* ix) {
    cpd_graph* g = ix->g;
    CPD_REQUIRE(g->npad / kFmTile < 65536u, CPD_E_RANGE, "graph too large for dense tables");
    ix->keep_rle = false;
    ix->stream_dense = true;
    ix->mode = CPD_INDEX_DENSE;
    {
        ArenaScope carve;  // an index's move tables (fifo_auto commits them early)
        ix->dense.alloc((size_t)ix->nrows * g->wpr());
    }
    ix->dense_ready = true;
}

// Moves an index's tables can hold: 16 (any 4-bit word) or 2^bits.
uint32_t table_move_limit(const cpd_graph* g) { return g->tlb == 2u ? 16u : 1u << (1u << g->tlb); }

// Host-side checks of a chunk's offsets (relative, offsets[0] == 0).
void check_chunk_offsets(const uint64_t* offsets, uint32_t count) {
    CPD_REQUIRE(offsets[0] == 0, CPD_E_ARG, "index: offsets[0] must be 0");
    for (uint32_t i = 0; i < count; ++i)
        CPD_REQUIRE(offsets[i + 1] > offsets[i], CPD_E_ARG, "index: empty or unsorted row");
}

// expand_rows' / validate_rows' work split for `count` rows whose host
// offsets are h_off (count + 1 values): the first run-chunk of each row,
// uploaded to ix->chunk_first; returns the number of chunks.  Every caller
// syncs the stream before the next call reuses the table.
uint32_t prepare_chunks(cpd_index* ix, const uint64_t* h_off, uint32_t count) {
    const uint64_t per = expand_chunk_runs();
    std::vector<uint32_t>& cf = ix->chunk_first_h;
    cf.assign((size_t)count + 1, 0);
    uint64_t tot = 0;
    for (uint32_t i = 0; i < count; ++i) {
        cf[i] = (uint32_t)tot;
        tot += (h_off[i + 1] - h_off[i] + per - 1) / per;
        CPD_REQUIRE(tot < (1ull << 31), CPD_E_RANGE, "index: too many runs in one append");
    }
    cf[count] = (uint32_t)tot;
    ix->chunk_first.upload(cf.data(), cf.size(), ix->g->stream);
    return (uint32_t)tot;
}

// Format check of `count` device rows (validate_rows); throws on a bad row.
// Leaves the rows' chunk table in ix->chunk_first and returns its size, for
// expand_into.
uint32_t validate_device_rows(cpd_index* ix, const uint64_t* d_off, const uint32_t* d_runs,
                              const uint64_t* h_off, uint32_t count, uint32_t mlimit = 16u) {
    cpd_graph* g = ix->g;
    const uint32_t chunks = prepare_chunks(ix, h_off, count);
    HIP_CHECK(hipMemsetAsync(ix->flag.p, 0, sizeof(uint32_t), g->stream));
    g->timed("validate_rows", 4.0 * (double)(h_off[count] - h_off[0]), [&] {
        launch_validate_rows(d_off, d_runs, ix->chunk_first.p, count, chunks, g->n, mlimit,
                             ix->flag.p, g->stream);
    });
    uint32_t bad = 0;
    HIP_CHECK(hipMemcpyAsync(&bad, ix->flag.p, sizeof bad, hipMemcpyDeviceToHost, g->stream));
    g->sync();
    CPD_REQUIRE(!bad, CPD_E_ARG,
                "index: malformed row (must start at column 0, run columns strictly increasing "
                "and < n" + std::string(mlimit < 16u ? ", moves < " + std::to_string(mlimit) +
                                                           " for this graph's move tables" : "") + ")");
    return chunks;
}

// Expand `count` rows (device offsets into d_runs; h_off = the same count + 1
// offsets on the host) into dense rows starting at index row `first`.
// chunks: the rows' chunk table is already in ix->chunk_first (what
// validate_device_rows returned), or 0 to build it here.
void expand_into(cpd_index* ix, const uint64_t* d_off, const uint32_t* d_runs,
                 const uint64_t* h_off, uint32_t count, uint64_t runs_in_chunk, uint32_t first,
                 uint32_t chunks = 0) {
    cpd_graph* g = ix->g;
    if (g->tlb != 2u) {
        // narrower tables: nibble rows into a stage (<= 256 MiB), then
        // narrowed into the index — rows checked to fit (validate_rows)
        const size_t w4 = g->npad / 8u, wpr = g->wpr();
        const uint32_t piece = (uint32_t)std::max<size_t>(1, ((size_t)1 << 26) / w4);
        ix->xstage.alloc((size_t)std::min(piece, count) * w4);
        for (uint32_t p0 = 0; p0 < count; p0 += piece) {
            const uint32_t p1 = std::min(count, p0 + piece);
            const uint32_t ch = prepare_chunks(ix, h_off + p0, p1 - p0);
            g->timed("expand_rows", 4.0 * (double)(h_off[p1] - h_off[p0]) + 4.0 * (double)w4 * (p1 - p0),
                     [&] {
                         launch_expand_rows(d_off + p0, d_runs, ix->chunk_first.p, p1 - p0, ch,
                                            g->npad, ix->xstage.p, g->stream);
                     });
            launch_repack_moves(ix->xstage.p, (uint32_t)w4, (uint32_t)w4, 4u, p1 - p0,
                                ix->dense.p + (size_t)(first + p0) * wpr, (uint32_t)wpr,
                                (uint32_t)wpr, 1u << g->tlb, g->stream);
            HIP_CHECK(hipGetLastError());
            g->sync();  // the chunk table and the stage are reused by the next piece
        }
        return;
    }
    const size_t wpr = g->npad / 8u;
    if (!chunks) chunks = prepare_chunks(ix, h_off, count);
    g->timed("expand_rows", 4.0 * (double)runs_in_chunk + 4.0 * (double)wpr * count + 16.0 * count,
             [&] {
                 launch_expand_rows(d_off, d_runs, ix->chunk_first.p, count, chunks, g->npad,
                                    ix->dense.p + first * wpr, g->stream);
             });
}

// Append `count` host rows (offsets relative, count + 1 values).
void append_host(cpd_index* ix, uint32_t count, const uint64_t* offsets, const uint32_t* runs) {
    cpd_graph* g = ix->g;
    CPD_REQUIRE(offsets, CPD_E_ARG, "index: null offsets");
    CPD_REQUIRE(count <= ix->nrows - ix->added, CPD_E_ARG, "index: more rows than declared");
    if (!count) return;
    check_chunk_offsets(offsets, count);
    const uint64_t nr = offsets[count];
    CPD_REQUIRE(runs, CPD_E_ARG, "index: null runs");
    hipStream_t s = g->stream;
    if (ix->keep_rle) {
        CPD_REQUIRE(ix->total + nr <= ix->cap, CPD_E_ARG,
                    "index: more runs than the index was created for");
        std::vector<uint64_t> o(count + 1);
        for (uint32_t i = 0; i <= count; ++i) o[i] = ix->total + offsets[i];
        HIP_CHECK(hipMemcpyAsync(ix->runs.p + ix->total, runs, nr * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(ix->off.p + ix->added, o.data(), o.size() * sizeof(uint64_t),
                                 hipMemcpyHostToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
        validate_device_rows(ix, ix->off.p + ix->added, ix->runs.p, o.data(), count);
        ix->offsets.insert(ix->offsets.end(), o.begin() + 1, o.end());
        ix->total += nr;
        ix->added += count;
        return;
    }
    // stream_dense: stage pieces of <= kStageRuns runs (a longer row alone)
    for (uint32_t r0 = 0; r0 < count;) {
        uint32_t r1 = r0 + 1;
        while (r1 < count && offsets[r1 + 1] - offsets[r0] <= kStageRuns) ++r1;
        const uint64_t base = offsets[r0], pr = offsets[r1] - base;
        std::vector<uint64_t> o(r1 - r0 + 1);
        for (uint32_t i = r0; i <= r1; ++i) o[i - r0] = offsets[i] - base;
        ix->stage.alloc(std::max<uint64_t>(pr, std::min<uint64_t>(nr, kStageRuns)));
        ix->stage_off.alloc(std::max<size_t>(o.size(), std::min<size_t>(count + 1, 1u << 20)));
        HIP_CHECK(hipMemcpyAsync(ix->stage.p, runs + base, pr * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(ix->stage_off.p, o.data(), o.size() * sizeof(uint64_t),
                                 hipMemcpyHostToDevice, s));
        const uint32_t ch = validate_device_rows(ix, ix->stage_off.p, ix->stage.p, o.data(), r1 - r0,
                                                 table_move_limit(g));
        expand_into(ix, ix->stage_off.p, ix->stage.p, o.data(), r1 - r0, pr, ix->added, ch);
        g->sync();  // the stage is reused by the next piece
        ix->added += r1 - r0;
        r0 = r1;
    }
}

// Append every row of a device-built cpd_rows (no host round trip): the
// move tables are copied as they are into a dense index, decoded into run
// words for an RLE one (and, for an index created from these rows whose
// AUTO mode resolves to dense, copied too).
void append_built(cpd_index* ix, const cpd_rows* r) {
    cpd_graph* g = ix->g;
    CPD_REQUIRE(r->device == g->device, CPD_E_ARG, "index: rows live on another device");
    r->settle();
    g->select();
    CPD_REQUIRE(r->nrows <= ix->nrows - ix->added, CPD_E_ARG, "index: more rows than declared");
    if (!r->nrows) return;
    // the built rows must be the declared rows at these positions (row i of
    // the index = row_targets[i]): a mismatch would file runs under the
    // wrong target, undetectable once a dense index has dropped them
    for (uint32_t i = 0; i < r->nrows; ++i)
        CPD_REQUIRE(r->targets[i] == ix->row_targets[ix->added + i], CPD_E_ARG,
                    "index: built row " + std::to_string(i) + " (target " +
                        std::to_string(r->targets[i]) + ") is not the declared row " +
                        std::to_string(ix->added + i));
    CPD_REQUIRE(r->n == g->n && r->wpr == (g->npad >> (5u - r->tlb)), CPD_E_ARG,
                "index: rows built for another graph");
    const size_t wpr = g->wpr();
    if (ix->dense.p && (ix->stream_dense || !ix->keep_rle || ix->dense_ready)) {
        if (r->tlb == g->tlb)
            HIP_CHECK(hipMemcpyAsync(ix->dense.p + (size_t)ix->added * wpr, r->moves.p,
                                     (size_t)r->nrows * wpr * sizeof(uint32_t),
                                     hipMemcpyDeviceToDevice, g->stream));
        else  // the rows' nibble tables narrowed to the index's width
            g->timed("repack_moves", 4.0 * ((double)r->wpr + (double)wpr) * r->nrows, [&] {
                launch_repack_moves(r->moves.p, r->wpr, r->wpr, 1u << r->tlb, r->nrows,
                                    ix->dense.p + (size_t)ix->added * wpr, (uint32_t)wpr,
                                    (uint32_t)wpr, 1u << g->tlb, g->stream);
            });
    }
    if (ix->keep_rle) {
        CPD_REQUIRE(ix->total + r->total <= ix->cap, CPD_E_ARG,
                    "index: more runs than the index was created for");
        std::vector<uint64_t> o(r->nrows + 1);
        for (uint32_t i = 0; i <= r->nrows; ++i) o[i] = ix->total + r->offsets[i];
        g->timed("moves_runs", 4.0 * (double)r->wpr * r->nrows + 4.0 * (double)r->total, [&] {
            launch_moves_runs(r->moves.p, r->wpr, r->tlb, r->n, r->nrows, r->off.p, 0,
                              ix->runs.p + ix->total, g->stream);
        });
        HIP_CHECK(hipMemcpyAsync(ix->off.p + ix->added, o.data(), o.size() * sizeof(uint64_t),
                                 hipMemcpyHostToDevice, g->stream));
        HIP_CHECK(hipStreamSynchronize(g->stream));
        ix->offsets.insert(ix->offsets.end(), o.begin() + 1, o.end());
        ix->total += r->total;
    }
    g->sync();
    ix->added += r->nrows;
}

// Append `count` host rows in the compact form (ceil(n * bits / 32) words
// each).  They are staged and, at the tables' width, copied into a dense
// index as they are (a pitched device copy to the table stride), else
// repacked — narrowing checks every move fits; an RLE index decodes them on
// the GPU, counting first.  No other format check is needed: every field is
// some move, and a move naming no out-edge of its column stops the walk
// (unfinished) like the oracle's.
void append_moves(cpd_index* ix, uint32_t count, uint32_t bits, const uint32_t* moves) {
    cpd_graph* g = ix->g;
    CPD_REQUIRE(count <= ix->nrows - ix->added, CPD_E_ARG, "index: more rows than declared");
    if (!count) return;
    CPD_REQUIRE(moves, CPD_E_ARG, "index: null move rows");
    CPD_REQUIRE(bits == 1 || bits == 2 || bits == 4, CPD_E_ARG, "index: bits per move must be 1, 2 or 4");
    const size_t w = ((uint64_t)g->n * bits + 31u) / 32u, wpr = g->wpr();
    const uint32_t tb = 1u << g->tlb;
    hipStream_t s = g->stream;
    // pieces of <= 1 GiB of tables or packed rows
    const uint32_t piece = (uint32_t)std::max<size_t>(1, ((size_t)1 << 28) / std::max(w, wpr));
    ix->lost.alloc(1);
    for (uint32_t r0 = 0; r0 < count; r0 += piece) {
        const uint32_t nr = std::min(piece, count - r0);
        uint32_t* tables = nullptr;
        if (!ix->keep_rle) {
            tables = ix->dense.p + (size_t)ix->added * wpr;
        } else {
            ix->stage.alloc((size_t)std::min(piece, count) * wpr);
            tables = ix->stage.p;
        }
        ix->pstage.alloc((size_t)std::min(piece, count) * w);
        HIP_CHECK(hipMemcpyAsync(ix->pstage.p, moves + (size_t)r0 * w, (size_t)nr * w * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, s));
        const bool narrowing = bits > tb;
        if (bits == tb) {
            HIP_CHECK(hipMemcpy2DAsync(tables, wpr * sizeof(uint32_t), ix->pstage.p,
                                       w * sizeof(uint32_t), w * sizeof(uint32_t), nr,
                                       hipMemcpyDeviceToDevice, s));
        } else {
            if (narrowing) HIP_CHECK(hipMemsetAsync(ix->lost.p, 0, sizeof(uint32_t), s));
            launch_repack_moves(ix->pstage.p, (uint32_t)w, (uint32_t)w, bits, nr, tables,
                                (uint32_t)wpr, (uint32_t)wpr, tb, s, narrowing ? ix->lost.p : nullptr);
            HIP_CHECK(hipGetLastError());
        }
        if (narrowing) {
            uint32_t lost = 0;
            HIP_CHECK(hipMemcpyAsync(&lost, ix->lost.p, sizeof lost, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            CPD_REQUIRE(!lost, CPD_E_ARG,
                        "index: a move does not fit this graph's " + std::to_string(tb) +
                            "-bit move tables (malformed rows)");
        }
        if (!ix->keep_rle) {
            HIP_CHECK(hipStreamSynchronize(s));
            ix->added += nr;
            continue;
        }
        ix->flag.alloc(std::max<size_t>(ix->flag.n, (size_t)std::min(piece, count)));
        launch_moves_count(tables, (uint32_t)wpr, g->tlb, g->n, nr, ix->flag.p, s);
        HIP_CHECK(hipGetLastError());
        std::vector<uint32_t> cnt(nr);
        HIP_CHECK(hipMemcpyAsync(cnt.data(), ix->flag.p, nr * sizeof(uint32_t),
                                 hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        std::vector<uint64_t> o(nr + 1);
        o[0] = ix->total;
        for (uint32_t i = 0; i < nr; ++i) o[i + 1] = o[i] + cnt[i];
        CPD_REQUIRE(o[nr] <= ix->cap, CPD_E_ARG, "index: more runs than the index was created for");
        HIP_CHECK(hipMemcpyAsync(ix->off.p + ix->added, o.data(), o.size() * sizeof(uint64_t),
                                 hipMemcpyHostToDevice, s));
        launch_moves_runs(tables, (uint32_t)wpr, g->tlb, g->n, nr, ix->off.p + ix->added, 0,
                          ix->runs.p, s);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
        ix->offsets.insert(ix->offsets.end(), o.begin() + 1, o.end());
        ix->total = o[nr];
        ix->added += nr;
    }
}

}  // namespace

extern "C" {

int cpd_index_create(cpd_graph* g, const uint32_t* row_targets, uint32_t nrows,
                     const uint64_t* offsets, const uint32_t* runs, cpd_index** out) {
    return guarded([&] {
        CPD_REQUIRE(g && out && row_targets && offsets, CPD_E_ARG, "index: null argument");
        *out = nullptr;
        g->select();
        auto ix = index_init(g, row_targets, nrows);
        ix->declared = offsets[nrows];
        index_keep_rle(ix.get(), ix->declared);
        append_host(ix.get(), nrows, offsets, runs);
        *out = ix.release();
    });
}

int cpd_index_from_rows(cpd_graph* g, const cpd_rows* r, cpd_index** out) {
    return guarded([&] {
        CPD_REQUIRE(g && r && out, CPD_E_ARG, "index: null argument");
        *out = nullptr;
        g->select();
        r->settle();
        g->select();
        auto ix = index_init(g, r->targets.data(), r->nrows);
        ix->declared = r->total;
        index_keep_rle(ix.get(), r->total);
        if (ix->use_dense()) {  // AUTO resolves dense: the rows' tables, copied
            CPD_REQUIRE(g->npad / kFmTile < 65536u, CPD_E_RANGE, "graph too large for dense tables");
            {
                ArenaScope carve;  // an index's move tables
                ix->dense.alloc((size_t)ix->nrows * g->wpr());
            }
            ix->dense_ready = true;
        }
        append_built(ix.get(), r);
        *out = ix.release();
    });
}

int cpd_index_create_empty(cpd_graph* g, const uint32_t* row_targets, uint32_t nrows, int mode,
                           uint64_t total_runs, cpd_index** out) {
    return guarded([&] {
        CPD_REQUIRE(g && out, CPD_E_ARG, "index: null argument");
        CPD_REQUIRE(mode == CPD_INDEX_AUTO || mode == CPD_INDEX_RLE || mode == CPD_INDEX_DENSE,
                    CPD_E_ARG, "index mode must be CPD_INDEX_AUTO, _RLE or _DENSE");
        *out = nullptr;
        g->select();
        auto ix = index_init(g, row_targets, nrows);
        ix->declared = total_runs;
        ix->mode = mode;
        if (ix->use_dense()) index_stream_dense(ix.get());
        else index_keep_rle(ix.get(), total_runs);
        HIP_CHECK(hipStreamSynchronize(g->stream));
        *out = ix.release();
    });
}

int cpd_index_append_rows(cpd_index* ix, uint32_t count, const uint64_t* offsets,
                          const uint32_t* runs) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "index: null argument");
        ix->g->select();
        append_host(ix, count, offsets, runs);
    });
}

int cpd_index_append_moves(cpd_index* ix, uint32_t count, uint32_t bits, const uint32_t* moves) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "index: null argument");
        ix->g->select();
        append_moves(ix, count, bits, moves);
    });
}

int cpd_index_append_built_rows(cpd_index* ix, const cpd_rows* r) {
    return guarded([&] {
        CPD_REQUIRE(ix && r, CPD_E_ARG, "index: null argument");
        ix->g->select();
        append_built(ix, r);
    });
}

int cpd_index_info(const cpd_index* ix, uint32_t* nrows, uint32_t* added, uint64_t* runs_resident,
                   uint64_t* dense_bytes) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "index: null argument");
        if (nrows) *nrows = ix->nrows;
        if (added) *added = ix->added;
        if (runs_resident) *runs_resident = ix->keep_rle ? ix->total : 0;
        if (dense_bytes) *dense_bytes = ix->dense_ready ? ix->dense.n * sizeof(uint32_t) : 0;
    });
}

int cpd_index_set_weights(cpd_index* ix, const uint32_t* w) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "null index");
        cpd_graph* g = ix->g;
        g->select();
        if (!w) {
            if (ix->custom_w) ix->c_ready = false;
            ix->custom_w = false;
            return;
        }
        std::vector<uint32_t> wc(g->m);
        for (uint32_t e = 0; e < g->m; ++e) wc[e] = w[g->edge_perm[e]];
        std::vector<uint32_t> adj = g->packed_adjacency(wc);
        ix->adj_sel.upload(adj.data(), adj.size(), g->stream);
        HIP_CHECK(hipStreamSynchronize(g->stream));
        ix->custom_w = true;
        ix->c_ready = false;  // the search's incumbent tables follow the weights
    });
}

int cpd_query_prepare(cpd_index* ix, const uint32_t* s, const uint32_t* t, uint32_t nq) {
    return guarded([&] {
        CPD_REQUIRE(ix && (nq == 0 || (s && t)), CPD_E_ARG, "query: null argument");
        CPD_REQUIRE(ix->added == ix->nrows, CPD_E_ARG,
                    "query: index incomplete (" + std::to_string(ix->added) + " of " +
                        std::to_string(ix->nrows) + " rows appended)");
        cpd_graph* g = ix->g;
        g->select();
        hipStream_t st = g->stream;
        // on the GPU: columns and target rows of the queries, a stable radix
        // sort by row (a wave's lanes then walk the same row), the sorted
        // columns; the caller's order comes back in cpd_query_fetch
        ix->nq = 0;
        ix->searched = false;
        const size_t m = std::max<uint32_t>(nq, 1u);
        for (DevBuf<uint32_t>* b : {&ix->qin_s, &ix->qin_t, &ix->qkey, &ix->qkey2, &ix->qval,
                                    &ix->qperm, &ix->qs, &ix->qt, &ix->qrow, &ix->hops})
            b->alloc(m);
        ix->qbad.alloc(1);
        ix->cost.alloc(m);
        ix->fin.alloc(m);
        if (nq) {
            HIP_CHECK(hipMemcpyAsync(ix->qin_s.p, s, nq * sizeof(uint32_t), hipMemcpyHostToDevice, st));
            HIP_CHECK(hipMemcpyAsync(ix->qin_t.p, t, nq * sizeof(uint32_t), hipMemcpyHostToDevice, st));
            HIP_CHECK(hipMemsetAsync(ix->qbad.p, 0, sizeof(uint32_t), st));
            launch_query_keys(ix->qin_s.p, ix->qin_t.p, nq, g->n, g->order_d.p, ix->d_row_of_col.p,
                              ix->qkey.p, ix->qval.p, ix->qbad.p, st);
            HIP_CHECK(hipGetLastError());
            uint32_t bad = 0;
            HIP_CHECK(hipMemcpyAsync(&bad, ix->qbad.p, sizeof bad, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            if (bad) {  // name the first offending query (error path only)
                for (uint32_t q = 0; q < nq; ++q) {
                    CPD_REQUIRE(s[q] < g->n && t[q] < g->n, CPD_E_ARG, "query node out of range");
                    if (ix->row_of_col[g->order[t[q]]] == CPD_INF)
                        throw Error(CPD_E_NOROW, "target " + std::to_string(t[q]) +
                                                     " has no CPD row in this index");
                }
            }
            const size_t tb = query_sort_bytes(nq);
            ix->qsort_tmp.alloc(tb);
            launch_query_sort(ix->qsort_tmp.p, ix->qsort_tmp.n, ix->qkey.p, ix->qkey2.p, ix->qval.p,
                              ix->qperm.p, nq, std::max(1u, ix->nrows), st);
            HIP_CHECK(hipGetLastError());
            launch_query_gather(ix->qin_s.p, ix->qin_t.p, g->order_d.p, ix->qkey2.p, ix->qperm.p,
                                nq, ix->qs.p, ix->qt.p, ix->qrow.p, st);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipStreamSynchronize(st));
        }
        ix->nq = nq;
    });
}

}  // extern "C"

namespace {

// Expand the resident RLE rows into dense move tables (once per index).
void ensure_dense(cpd_index* ix) {
    cpd_graph* g = ix->g;
    CPD_REQUIRE(g->npad / kFmTile < 65536u, CPD_E_RANGE, "graph too large for dense tables");
    {
        ArenaScope carve;  // an index's move tables (fifo_auto commits them early)
        ix->dense.alloc((size_t)ix->nrows * g->wpr());
    }
    if (ix->nrows && g->tlb != 2u)  // the runs' moves must fit the narrower tables
        validate_device_rows(ix, ix->off.p, ix->runs.p, ix->offsets.data(), ix->nrows,
                             table_move_limit(g));
    if (ix->nrows)
        expand_into(ix, ix->off.p, ix->runs.p, ix->offsets.data(), ix->nrows, ix->total, 0);
    g->sync();
    ix->dense_ready = true;
}

}  // namespace

extern "C" {

int cpd_index_set_mode(cpd_index* ix, int mode) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "null index");
        CPD_REQUIRE(mode == CPD_INDEX_AUTO || mode == CPD_INDEX_RLE || mode == CPD_INDEX_DENSE,
                    CPD_E_ARG, "index mode must be CPD_INDEX_AUTO, _RLE or _DENSE");
        CPD_REQUIRE(!(ix->stream_dense && mode == CPD_INDEX_RLE), CPD_E_ARG,
                    "index was streamed into dense tables: its runs were not kept");
        if (!ix->stream_dense) ix->mode = mode;
    });
}

int cpd_index_get_mode(const cpd_index* ix, int* mode) {
    return guarded([&] {
        CPD_REQUIRE(ix && mode, CPD_E_ARG, "null argument");
        *mode = ix->use_dense() ? CPD_INDEX_DENSE : CPD_INDEX_RLE;
    });
}

int cpd_query_run(cpd_index* ix, int32_t k_moves, cpd_query_stats* st) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "null index");
        cpd_graph* g = ix->g;
        g->select();
        const uint32_t nq = ix->nq;
        const bool dense = ix->use_dense();
        if (dense && !ix->dense_ready) ensure_dense(ix);
        HIP_CHECK(hipMemsetAsync(ix->agg.p, 0, 4 * sizeof(unsigned long long), g->stream));
        hipEvent_t a = g->get_event(), b = g->get_event();
        HIP_CHECK(hipEventRecord(a, g->stream));
        const uint32_t* adj = ix->custom_w ? ix->adj_sel.p : g->adj.p;
        (void)hipGetLastError();
        if (nq && dense)
            launch_table_search_dense(adj, g->adj_shift, ix->d_row_of_col.p, ix->dense.p, g->npad, g->tlb,
                                      ix->qs.p, ix->qt.p, ix->qrow.p, nq, k_moves, g->n,
                                      ix->cost.p, ix->hops.p, ix->fin.p, ix->agg.p, g->stream);
        else if (nq)
            launch_table_search(adj, g->adj_shift, ix->d_row_of_col.p, ix->off.p, ix->runs.p,
                                ix->qs.p, ix->qt.p, ix->qrow.p, nq, k_moves, g->n, ix->cost.p,
                                ix->hops.p, ix->fin.p, ix->agg.p, g->stream);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipEventRecord(b, g->stream));
        unsigned long long hagg[4] = {0, 0, 0, 0};
        HIP_CHECK(hipMemcpyAsync(hagg, ix->agg.p, sizeof hagg, hipMemcpyDeviceToHost, g->stream));
        HIP_CHECK(hipStreamSynchronize(g->stream));
        if (hagg[3] && search_trace())  // CPD_TS_SHARE: the moves suffix sharing skipped
            std::fprintf(stderr, "[walk] %llu queries, %llu moves, %llu of them taken from "
                         "earlier walks' suffixes\n", (unsigned long long)nq, hagg[1], hagg[3]);
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, a, b));
        g->ev_pool.push_back(a);
        g->ev_pool.push_back(b);
        if (g->timing) {
            Agg& ag = g->agg[dense ? "table_search_dense" : "table_search"];
            ag.launches++;
            ag.ms += ms;
            if (dense) {
                // per query 8 (s,t) + 13 (outputs) + 4 (row); per move one
                // 4-B move word + one 8-B packed edge
                ag.bytes += 25.0 * nq + 12.0 * (double)hagg[1];
            } else {
                // SURVEY.md §8(d) B_q = 8 + 12 + 8 + L * (4 ceil(log2 R) + 16)
                double mean_log = 0.0;
                if (ix->nrows) {
                    double s = 0.0;
                    for (uint32_t i = 0; i < ix->nrows; ++i)
                        s += std::ceil(std::log2((double)std::max<uint64_t>(
                            2, ix->offsets[i + 1] - ix->offsets[i])));
                    mean_log = s / ix->nrows;
                }
                ag.bytes += 28.0 * nq + (double)hagg[1] * (4.0 * mean_log + 16.0);
            }
        }
        if (st) {
            st->queries = nq;
            st->finished = hagg[0];
            st->hops = hagg[1];
            st->cost = hagg[2];
            st->kernel_ms = ms;
        }
    });
}

int cpd_query_fetch(cpd_index* ix, uint64_t* cost, uint32_t* hops, uint8_t* finished) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "null index");
        cpd_graph* g = ix->g;
        g->select();
        const uint32_t nq = ix->nq;
        if (!nq) return;
        // results come back in target-sorted order: scattered to the
        // caller's order on the GPU, then copied out
        hipStream_t st = g->stream;
        ix->qout.alloc((size_t)nq * 8u);
        if (cost) {
            launch_scatter_u64(ix->cost.p, ix->qperm.p, nq, reinterpret_cast<uint64_t*>(ix->qout.p), st);
            HIP_CHECK(hipMemcpyAsync(cost, ix->qout.p, nq * 8ull, hipMemcpyDeviceToHost, st));
        }
        if (hops) {
            HIP_CHECK(hipStreamSynchronize(st));  // qout is reused
            launch_scatter_u32(ix->hops.p, ix->qperm.p, nq, 1u, reinterpret_cast<uint32_t*>(ix->qout.p), st);
            HIP_CHECK(hipMemcpyAsync(hops, ix->qout.p, nq * 4ull, hipMemcpyDeviceToHost, st));
        }
        if (finished) {
            HIP_CHECK(hipStreamSynchronize(st));
            launch_scatter_u8(ix->fin.p, ix->qperm.p, nq, ix->qout.p, st);
            HIP_CHECK(hipMemcpyAsync(finished, ix->qout.p, nq, hipMemcpyDeviceToHost, st));
        }
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(st));
    });
}

int cpd_query_batch(cpd_index* ix, const uint32_t* s, const uint32_t* t, uint32_t nq,
                    int32_t k_moves, uint64_t* cost, uint32_t* hops, uint8_t* finished,
                    cpd_query_stats* st) {
    int rc = cpd_query_prepare(ix, s, t, nq);
    if (rc) return rc;
    rc = cpd_query_run(ix, k_moves, st);
    if (rc) return rc;
    return cpd_query_fetch(ix, cost, hops, finished);
}

void cpd_index_free(cpd_index* ix) {
    if (ix && ix->g) (void)hipSetDevice(ix->g->device);
    delete ix;
}

// ---------------------------------------------------------------------------
// CPD-heuristic search

}  // extern "C"

namespace {

// The search workspace policy (fifo_auto and the bench
// run the same one).  capacity 0 = automatic: the first pass's columns per
// lane are 2^13 when fscale > 0 (a bounded-suboptimal search expands ~140
// nodes on the 1M bench graph) and 2^14 at fscale 0 (~47k expansions on
// average, heavy-tailed: a first pass that stops the long searches early and
// resumes them in fuller waves beats one that spills fewer —
// profiles/search_heap_ab/r05y_*: 5.08k q/s from 2^14, 4.73k from 2^15),
// lowered to 2^10 at most until
// every search of the request gets a lane (profiles/search_cap_ab/,
// search_lanes_ab/); capacity_max 0 = 4x the graph's columns rounded up to
// a power of 2 (a search holds each column once, its heap some stale
// entries more), at most 2^24; workspace_frac 0 = 0.85 of the free HBM.
// An explicit capacity keeps the old defaults (no escalation, 0.25).
uint32_t pow2_at_least(uint64_t x) {
    uint32_t c = 64;
    while (c < x && c < (1u << 24)) c <<= 1;
    return c;
}

bool search_trace() {
    static const bool on = [] {
        const char* e = std::getenv("CPD_SEARCH_TRACE");
        return e && *e && *e != '0';
    }();
    return on;
}

}  // namespace

extern "C" {

int cpd_query_search(cpd_index* ix, const cpd_search_opts* opts, cpd_search_stats* st) {
    return guarded([&] {
        CPD_REQUIRE(ix, CPD_E_ARG, "null index");
        cpd_search_opts o{1.0, 0.0, -1, -1, 0, 0, 0, CPD_SEARCH_AUTO, 0.0, 0};
        if (opts) o = *opts;
        const bool auto_cap = o.capacity == 0;
        CPD_REQUIRE(auto_cap || ((o.capacity & (o.capacity - 1)) == 0 && o.capacity >= 64 &&
                                 o.capacity <= (1u << 24)),
                    CPD_E_ARG, "search capacity must be 0 (automatic) or a power of 2 in [64, 2^24]");
        CPD_REQUIRE(o.capacity_max == 0 ||
                        ((o.capacity_max & (o.capacity_max - 1)) == 0 &&
                         o.capacity_max >= std::max<uint32_t>(o.capacity, 64u) &&
                         o.capacity_max <= (1u << 24)),
                    CPD_E_ARG, "search capacity_max must be 0 or a power of 2 in [capacity, 2^24]");
        CPD_REQUIRE(o.hscale >= 0.0 && o.fscale >= 0.0, CPD_E_ARG,
                    "hscale and fscale must be >= 0");
        CPD_REQUIRE(o.workspace_frac >= 0.0 && o.workspace_frac <= 0.9, CPD_E_ARG,
                    "workspace_frac must be in [0, 0.9]");
        const double wfrac = o.workspace_frac > 0.0 ? o.workspace_frac : auto_cap ? 0.85 : 0.25;
        CPD_REQUIRE(ix->added == ix->nrows, CPD_E_ARG, "search: index incomplete");
        CPD_REQUIRE(o.tables == CPD_SEARCH_AUTO || o.tables == CPD_SEARCH_TABLES ||
                        o.tables == CPD_SEARCH_WALKS,
                    CPD_E_ARG, "search tables must be CPD_SEARCH_AUTO, _TABLES or _WALKS");
        cpd_graph* g = ix->g;
        g->select();
        const uint32_t n = g->n, nq = ix->nq;
        if (!ix->dense_ready) ensure_dense(ix);
        const uint32_t* adj_w = ix->custom_w ? ix->adj_sel.p : g->adj.p;
        // per-row tables (20 B per column per row) when they fit in half of
        // the free HBM (AUTO) or when asked for; else memoised walks
        const size_t cells = (size_t)ix->nrows * n;
        bool tables = o.tables == CPD_SEARCH_TABLES;
        {
            size_t free_b = 0, total_b = 0;
            HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
            const size_t have = ix->hrow.p ? 20u * cells : 0u;
            const bool fits = 20u * cells - have < (free_b + have) / 2;
            if (o.tables == CPD_SEARCH_AUTO) tables = fits;
            CPD_REQUIRE(!tables || fits, CPD_E_OOM,
                        "cpd-search tables need " + std::to_string((20u * cells) >> 20) +
                            " MiB (20 B per column per index row): use the walk form");
        }
        hipEvent_t a = g->get_event(), b = g->get_event();
        double tables_ms = 0.0;
        if (tables && (!ix->h_ready || !ix->c_ready)) {
            size_t free_b = 0, total_b = 0;
            ix->hrow.alloc(cells);
            ix->crow.alloc(cells);
            ix->lrow.alloc(cells);
            std::vector<uint32_t> tc(ix->nrows, 0);
            for (uint32_t c = 0; c < n; ++c)
                if (ix->row_of_col[c] != CPD_INF) tc[ix->row_of_col[c]] = c;
            ix->tcol.upload(tc.data(), tc.size(), g->stream);
            HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
            // scratch for the doubling rounds: 48 B per column per chunk row
            const uint32_t chunk = (uint32_t)std::max<size_t>(
                1, std::min<size_t>(ix->nrows, (size_t)(free_b / 4) / (48ull * n + 1)));
            DevBuf<uint8_t> scratch;
            scratch.alloc((size_t)chunk * n * 48u);
            HIP_CHECK(hipEventRecord(a, g->stream));
            launch_search_tables(ix->dense.p, g->npad, g->tlb, g->adj.p, adj_w, g->adj_shift, ix->tcol.p,
                                 ix->nrows, n, scratch.p, chunk, ix->hrow.p, ix->crow.p,
                                 ix->lrow.p, ix->h_ready ? 0 : 1, g->stream);
            HIP_CHECK(hipEventRecord(b, g->stream));
            HIP_CHECK(hipStreamSynchronize(g->stream));
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, a, b));
            tables_ms = ms;
            ix->h_ready = ix->c_ready = true;
        }
        g->ev_pool.push_back(a);
        g->ev_pool.push_back(b);
        hipStream_t sm = g->stream;
        const uint32_t cap_max = o.capacity_max ? o.capacity_max
                                 : auto_cap     ? pow2_at_least(4ull * std::max(n, 16u))
                                                : o.capacity;
        // HBM the passes may use: what is free plus what this index's search
        // buffers already hold (reused)
        auto avail = [&](size_t live) {
            size_t free_b = 0, total_b = 0;
            HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
            return free_b + ix->sws.n + ix->spool[0].n * 4u + ix->spool[1].n * 4u - live;
        };
        uint32_t cap = o.capacity;
        if (auto_cap) {
            // (walks: 2^14 at fscale > 0 too — a walk's columns count, and
            // at 2^13 the few searches that outgrew it took a second pass of
            // 10% of the time: 271-280k against 245-252k q/s, r05ap)
            cap = std::min(o.fscale > 0.0 && tables ? (1u << 13) : (1u << 14), cap_max);
            const size_t budget = (size_t)(wfrac * (double)avail(0) * (cap < cap_max ? 0.75 : 1.0));
            const uint64_t lanes = nq ? search_slots(nq) : 64u;
            while (cap > (1u << 10) && lanes * search_ws_bytes_per_slot(cap, tables) > budget) cap >>= 1;
        }
        const uint32_t cap0 = cap;
        uint64_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        double ms = 0.0;
        uint64_t reruns = 0, resumed = 0, restarted = 0, wasted = 0, lanes1 = 0;
        uint32_t passes = 0, cap_last = cap;
        ix->qstats.alloc(5ull * std::max(1u, nq));
        ix->sagg.alloc(8);
        ix->stop.alloc(1);
        // The passes: pass 1 runs every query at `cap` columns per lane; a
        // search that would outgrow it stops whole and spills its state
        // (fin 3) or, with the pool full, stops to restart (fin 2); each
        // later pass runs those at 4x the capacity — spilled ones resumed
        // from their records — until none is left or capacity_max (or the
        // HBM) is reached; what is left then reports finished = 2.
        // Pass-local arrays (m queries; pass 1: the index's own, m = nq).
        uint32_t m = nq;
        std::vector<uint32_t> gidx;               // pass query -> caller-sorted query (pass >= 2)
        DevBuf<uint32_t> d_idx, d_q, d_hops, d_st;
        DevBuf<uint64_t> d_cost;
        DevBuf<uint8_t> d_fin;
        DevBuf<unsigned long long> d_agg, d_res;
        int pin = 0;                              // spool[pin]: the records the pass resumes from
        bool have_resume = false;
        while (m) {
            ++passes;
            const bool first = passes == 1;
            const bool more = cap < cap_max;      // a later pass can take what overflows
            const uint32_t* pq_s = first ? ix->qs.p : d_q.p;
            const uint32_t* pq_t = first ? ix->qt.p : d_q.p + m;
            const uint32_t* pq_r = first ? ix->qrow.p : d_q.p + 2ull * m;
            uint64_t* p_cost = first ? ix->cost.p : d_cost.p;
            uint32_t* p_hops = first ? ix->hops.p : d_hops.p;
            uint8_t* p_fin = first ? ix->fin.p : d_fin.p;
            uint32_t* p_st = first ? ix->qstats.p : d_st.p;
            unsigned long long* p_agg = first ? ix->sagg.p : d_agg.p;
            // lanes: as many as the workspace share holds (whole waves),
            // leaving a quarter of it to the spill pool when a later pass
            // can resume; the pool takes the rest of the share
            const size_t live_in = have_resume ? ix->spool[pin].n * 4u : 0u;
            const size_t av = avail(live_in);
            const size_t share = (size_t)(wfrac * (double)av);
            const size_t per_slot = search_ws_bytes_per_slot(cap, tables);
            // (a quarter in pass 1, a tenth later: fewer searches spill again)
            const size_t ws_budget = more ? (first ? share / 4u * 3u : share / 10u * 9u) : share;
            const uint64_t fit = ws_budget / (64ull * per_slot);
            CPD_REQUIRE(fit > 0 || av / 2 >= 64ull * per_slot, CPD_E_OOM,
                        "search workspace of 64 lanes x capacity " + std::to_string(cap) +
                            " does not fit in HBM");
            const uint32_t slots = (uint32_t)std::min<uint64_t>(search_slots(m), std::max<uint64_t>(1, fit) * 64u);
            if (first) lanes1 = slots;
            ix->sws.release();
            ix->sws.alloc((size_t)slots * per_slot);
            SearchSpillArgs sa;
            if (have_resume) {
                sa.resume = d_res.p;
                sa.rin = ix->spool[pin].p;
            }
            if (more) {
                const uint64_t want = (uint64_t)m * search_spill_words(cap, tables);
                const uint64_t left = share > (size_t)slots * per_slot ? share - (size_t)slots * per_slot : 0;
                uint64_t words = std::min<uint64_t>(want, left / 4u);
                // CPD_SEARCH_POOL_WORDS (tests): a smaller pool, so that some
                // records find it full and their searches restart instead
                if (const char* e = std::getenv("CPD_SEARCH_POOL_WORDS"))
                    if (*e) words = std::min<uint64_t>(words, std::strtoull(e, nullptr, 10));
                if (words >= search_spill_words(cap, tables)) {
                    DevBuf<uint32_t>& out = ix->spool[pin ^ 1];
                    out.release();
                    out.alloc(words);
                    ix->sat.alloc(m);
                    sa.rout = out.p;
                    sa.at = ix->sat.p;
                    sa.top = ix->stop.p;
                    sa.cap_words = words;
                    HIP_CHECK(hipMemsetAsync(ix->stop.p, 0, sizeof(unsigned long long), sm));
                }
            }
            HIP_CHECK(hipMemsetAsync(p_agg, 0, 8 * sizeof(unsigned long long), sm));
            hipEvent_t ea = g->get_event(), eb = g->get_event();
            HIP_CHECK(hipEventRecord(ea, sm));
            (void)hipGetLastError();
            launch_cpd_search(g->adj.p, adj_w, g->adj_shift, ix->dense.p, g->npad, g->tlb,
                              tables ? ix->hrow.p : nullptr, ix->crow.p, ix->lrow.p, n, pq_s, pq_t,
                              pq_r, m, o.hscale, o.fscale, o.k_moves, o.itrs, o.time_ns,
                              o.virtual_tick_ns, ix->sws.p, cap, slots, sa, p_cost, p_hops, p_fin,
                              p_st, p_agg, sm);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipEventRecord(eb, sm));
            if (!first) {  // this pass's results over the first pass's
                launch_scatter_u64(d_cost.p, d_idx.p, m, ix->cost.p, sm);
                launch_scatter_u32(d_hops.p, d_idx.p, m, 1u, ix->hops.p, sm);
                launch_scatter_u8(d_fin.p, d_idx.p, m, ix->fin.p, sm);
                launch_scatter_u32(d_st.p, d_idx.p, m, 5u, ix->qstats.p, sm);
            }
            unsigned long long hp[8];
            HIP_CHECK(hipMemcpyAsync(hp, p_agg, sizeof hp, hipMemcpyDeviceToHost, sm));
            HIP_CHECK(hipStreamSynchronize(sm));
            float pms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&pms, ea, eb));
            g->ev_pool.push_back(ea);
            g->ev_pool.push_back(eb);
            ms += pms;
            for (int k = 0; k < 7; ++k) h[k] += hp[k];
            h[7] = hp[7];
            cap_last = cap;
            if (search_trace())
                std::fprintf(stderr, "[cpd_search] pass %u: %u queries, capacity %u, %u lanes, "
                             "%.3f ms, %llu expanded, %llu overflowed, pool %llu words\n",
                             passes, m, cap, slots, pms, (unsigned long long)hp[0],
                             (unsigned long long)hp[7], (unsigned long long)sa.cap_words);
            if (!hp[7]) break;
            // the searches that overflowed: spilled (fin 3) resume, the others
            // (fin 2) restart from scratch — their counters leave the sums
            std::vector<uint8_t> f(m);
            std::vector<uint32_t> qst(5ull * m), hq(3ull * m);
            std::vector<unsigned long long> at(m, ~0ull);
            HIP_CHECK(hipMemcpyAsync(f.data(), p_fin, m, hipMemcpyDeviceToHost, sm));
            HIP_CHECK(hipMemcpyAsync(qst.data(), p_st, 20ull * m, hipMemcpyDeviceToHost, sm));
            HIP_CHECK(hipMemcpyAsync(hq.data(), pq_s, 4ull * m, hipMemcpyDeviceToHost, sm));
            HIP_CHECK(hipMemcpyAsync(hq.data() + m, pq_t, 4ull * m, hipMemcpyDeviceToHost, sm));
            HIP_CHECK(hipMemcpyAsync(hq.data() + 2ull * m, pq_r, 4ull * m, hipMemcpyDeviceToHost, sm));
            if (sa.rout) HIP_CHECK(hipMemcpyAsync(at.data(), ix->sat.p, 8ull * m, hipMemcpyDeviceToHost, sm));
            HIP_CHECK(hipStreamSynchronize(sm));
            // The next capacity, 2x to 4x: the largest at which every search
            // left gets a lane (one round: the long searches run side by side
            // instead of waiting for lanes), else the largest at which 64
            // lanes fit (never throw there — what cannot grow
            // reports finished = 2).  With resumed searches a smaller step
            // wastes nothing.  (Fixed 4x or 2x steps lost their A/Bs, rounds 4-5.)
            uint32_t next = 0;
            if (more) {
                uint32_t left = 0;
                for (uint32_t i = 0; i < m; ++i) left += f[i] == 2u || f[i] == 3u;
                const size_t av2 = avail(sa.rout ? ix->spool[pin ^ 1].n * 4u : 0u);
                const double share2 = wfrac * (double)av2;
                for (uint32_t c = std::min(cap * 4u, cap_max); c > cap; c >>= 1) {
                    const double per = (double)search_ws_bytes_per_slot(c, tables);
                    if (64.0 * per > share2) continue;
                    if (!next) next = c;
                    if ((double)search_slots(left) * per <= 0.9 * share2) {
                        next = c;
                        break;
                    }
                }
            }
            std::vector<uint32_t> idx, sub;
            std::vector<unsigned long long> res;
            bool any_res = false;
            for (uint32_t i = 0; i < m; ++i) {
                if (f[i] != 2u && f[i] != 3u) continue;
                const bool spilled = f[i] == 3u;
                // restarted: its first pass leaves the sums — only when a
                // next pass runs it again; otherwise it ends here as an
                // overflow and its counters stay
                if (!spilled && next) {
                    for (int k = 0; k < 5; ++k) h[k] -= qst[5ull * i + k];
                    wasted += qst[5ull * i];
                }
                idx.push_back(i);
                res.push_back(spilled ? at[i] : ~0ull);
                any_res |= spilled;
            }
            const uint32_t m2 = (uint32_t)idx.size();
            if (!next) {
                // no larger workspace fits: spilled searches are final
                // overflows too (finished = 2, their counters in the sums)
                if (any_res) {
                    for (uint32_t i = 0; i < m; ++i)
                        if (f[i] == 3u) {
                            f[i] = 2u;
                            for (int k = 0; k < 5; ++k) h[k] += qst[5ull * i + k];
                        }
                    HIP_CHECK(hipMemcpyAsync(p_fin, f.data(), m, hipMemcpyHostToDevice, sm));
                    if (!first) launch_scatter_u8(d_fin.p, d_idx.p, m, ix->fin.p, sm);
                    HIP_CHECK(hipStreamSynchronize(sm));
                }
                break;
            }
            reruns += m2;
            for (unsigned long long r : res) (r == ~0ull ? restarted : resumed)++;
            sub.resize(3ull * m2);
            std::vector<uint32_t> g2(m2);
            for (uint32_t j = 0; j < m2; ++j) {
                const uint32_t i = idx[j];  // target-sorted order is kept
                sub[j] = hq[i];
                sub[m2 + j] = hq[m + i];
                sub[2ull * m2 + j] = hq[2ull * m + i];
                g2[j] = first ? i : gidx[i];
            }
            gidx.swap(g2);
            d_idx.upload(gidx.data(), m2, sm);
            d_q.upload(sub.data(), 3ull * m2, sm);
            d_res.upload(res.data(), m2, sm);
            d_hops.alloc(m2);
            d_st.alloc(5ull * m2);
            d_cost.alloc(m2);
            d_fin.alloc(m2);
            d_agg.alloc(8);
            have_resume = any_res;
            ix->spool[pin].release();            // the records this pass resumed from
            if (any_res) {                       // the records just written, kept at their size
                unsigned long long used = 0;
                HIP_CHECK(hipMemcpy(&used, ix->stop.p, sizeof used, hipMemcpyDeviceToHost));
                DevBuf<uint32_t>& full = ix->spool[pin ^ 1];
                used = std::min<unsigned long long>(used, full.n);
                if (used < full.n / 10 * 9) {
                    DevBuf<uint32_t>& fit = ix->spool[pin];
                    fit.alloc(std::max<unsigned long long>(used, 1));
                    HIP_CHECK(hipMemcpyAsync(fit.p, full.p, 4ull * used, hipMemcpyDeviceToDevice, sm));
                    HIP_CHECK(hipStreamSynchronize(sm));
                    full.release();
                } else {
                    pin ^= 1;
                }
            } else {
                ix->spool[pin ^ 1].release();
            }
            m = m2;
            cap = next;
        }
        // the spill pools are scratch: freed with the pass that used them
        ix->spool[0].release();
        ix->spool[1].release();
        if (g->timing) {
            Agg& ag = g->agg["cpd_search"];
            ag.launches += passes;
            ag.ms += ms;
        }
        ix->searched = true;
        if (st) {
            st->queries = nq;
            st->expanded = h[0];
            st->inserted = h[1];
            st->touched = h[2];
            st->updated = h[3];
            st->surplus = h[4];
            st->plen = h[5];
            st->finished = h[6];
            st->overflow = h[7];
            st->kernel_ms = ms;
            st->lanes = lanes1;
            st->tables_ms = tables_ms;
            st->tables = tables ? CPD_SEARCH_TABLES : CPD_SEARCH_WALKS;
            st->reruns = reruns;
            st->resumed = resumed;
            st->restarted = restarted;
            st->wasted_expanded = wasted;
            st->passes = passes;
            st->capacity = cap0;
            st->capacity_last = cap_last;
        }
    });
}

int cpd_query_search_counters(cpd_index* ix, uint32_t* counters) {
    return guarded([&] {
        CPD_REQUIRE(ix && counters, CPD_E_ARG, "null argument");
        ix->g->select();
        const uint32_t nq = ix->nq;
        if (!nq) return;
        CPD_REQUIRE(ix->searched && ix->qstats.n >= 5ull * nq, CPD_E_ARG,
                    "no search has run on these queries (cpd_query_prepare since, or only "
                    "table-search)");
        hipStream_t st = ix->g->stream;
        ix->qout.alloc(20ull * nq);
        launch_scatter_u32(ix->qstats.p, ix->qperm.p, nq, 5u, reinterpret_cast<uint32_t*>(ix->qout.p),
                           st);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(counters, ix->qout.p, 20ull * nq, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
    });
}

// ---------------------------------------------------------------------------
// Timing

int cpd_timing_enable(cpd_graph* g, int enable) {
    return guarded([&] {
        CPD_REQUIRE(g, CPD_E_ARG, "null graph");
        g->timing = enable != 0;
    });
}

int cpd_timing_reset(cpd_graph* g) {
    return guarded([&] {
        CPD_REQUIRE(g, CPD_E_ARG, "null graph");
        g->select();
        g->sync(true);
        fold_late(g, 0);
        g->agg.clear();
    });
}

int cpd_timing_get(const cpd_graph* g, cpd_kernel_time* out, int max, int* count) {
    return guarded([&] {
        CPD_REQUIRE(g && count, CPD_E_ARG, "null argument");
        // emits may still run on the emit stream: fold them in first
        auto* gm = const_cast<cpd_graph*>(g);
        gm->select();
        gm->sync(true);
        fold_late(gm, 0);
        int k = 0;
        for (auto& kv : g->agg) {
            if (out && k < max) {
                std::memset(out[k].name, 0, sizeof out[k].name);
                std::strncpy(out[k].name, kv.first.c_str(), sizeof out[k].name - 1);
                out[k].launches = kv.second.launches;
                out[k].ms = kv.second.ms;
                out[k].bytes = kv.second.bytes;
            }
            ++k;
        }
        *count = std::min(k, out ? max : k);
    });
}

}  // extern "C"

// Host-callable launchers for the GPU contraction (ch_kernels.hip), driven by
// ch_gpu.cpp.  Node ids are the graph's own ids; the overlay graph is an arena
// of (neighbour, weight) arcs with per-node (offset, degree) for the out- and
// the in-lists, each list sorted by neighbour id.
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace cpd {
namespace chk {

struct Overlay {
    const uint32_t* ooff;
    const uint32_t* odeg;
    const uint32_t* ioff;
    const uint32_t* ideg;
    const uint32_t* arcs;  // uint2 (neighbour, weight)
};

// Witness-search lane workspace: hash slots (16 B), heap slots (16 B) and
// target slots (16 B + 4 B settled flag) per lane.
struct WitnessCaps {
    uint32_t hash;  // power of two
    uint32_t heap;
    uint32_t tgt;
};
uint64_t witness_lane_bytes(WitnessCaps c);

// Exclusive scan of n u32 (out[n] = total when in[n] == 0 and n + 1 values
// are scanned by the caller).  tmp / tmp_bytes: scratch; tmp == nullptr
// returns the bytes needed in *tmp_bytes.
void scan_u32(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
              hipStream_t s);

// flag[i] = rem[i] is a local priority minimum among its out- and in-
// neighbours (ch.cpp step 1); flag[R] = 0.
void launch_pick(const uint32_t* rem, uint32_t R, Overlay g, const int64_t* prio,
                 uint32_t* flag, hipStream_t s);
// Stable split of in[0..n) by flag, pos = exclusive scan of flag.
void launch_split(const uint32_t* in, const uint32_t* flag, const uint32_t* pos, uint32_t n,
                  uint32_t* sel, uint32_t* rej, hipStream_t s);
// Selected nodes S: state[v] = 1 and per node c0 = pairs (in-degree if the
// out-list is non-empty), c1 = shortcut slots (pairs x out-degree), c2 =
// out-degree, c3 = in-degree; index k == nS writes zeros.
void launch_sel_counts(const uint32_t* S, uint32_t nS, Overlay g, uint8_t* state, uint32_t* c0,
                       uint32_t* c1, uint32_t* c2, uint32_t* c3, hipStream_t s);
// Witness-search pairs (node, in-list index, first slot, 0) of the nodes in
// list[0..k): node list[i] owns pairs pbase[i].. and slots sbase[i]..
// (sbase may be null: the simulation pass writes no slots).
void launch_make_pairs(const uint32_t* list, uint32_t k, Overlay g, const uint32_t* pbase,
                       const uint32_t* sbase, uint32_t* pairs /* uint4 */, hipStream_t s);
// Witness searches (ch.cpp Witness::run + Contractor::shortcuts_via), one
// lane each, for pairs[plist ? plist[i] : i], i < np.  contract: avoid nodes
// with state 1, store (u, x, w, 1) or zeros per out-list slot in slots and
// 1/0 in sflag; else atomicAdd the shortcut count to sc[node].  A search that
// outgrows the lane workspace, or runs past step_cap pops + relaxations, is appended to ovf (count in ovf_n) and writes
// nothing; a needed shortcut of weight >= 2^32-1 sets err.
void launch_witness(const uint32_t* pairs, const uint32_t* plist, uint32_t np, Overlay g,
                    const uint8_t* state, bool contract, uint32_t settle, void* ws,
                    WitnessCaps caps, uint32_t lanes, uint32_t tag_base, uint32_t step_cap,
                    uint32_t* slots, uint32_t* sflag, uint32_t* sc, uint32_t* ovf,
                    uint32_t* ovf_n, uint32_t* err, hipStream_t s);
// The same searches, one wave each with the search's table and heap in LDS
// (witness_wave_lds_bytes(size) per workgroup; size 0: 512 table / 384 heap
// slots / 32 targets, 1: 1024 / 768 / 64, 2: 2048 / 1792 / 128): for the
// core rounds' large searches.  A search that outgrows LDS goes to ovf as above.
void launch_witness_wave(const uint32_t* pairs, const uint32_t* plist, uint32_t np, Overlay g,
                         const uint8_t* state, bool contract, uint32_t settle, uint32_t blocks,
                         int size, uint32_t* slots, uint32_t* sflag, uint32_t* sc, uint32_t* ovf,
                         uint32_t* ovf_n, uint32_t* err, hipStream_t s);
uint32_t witness_wave_lds_bytes(int size);
// Record the contracted nodes S (ranks rank0 + i): rank[v], rec_* per rank,
// their out-/in-lists copied to the up / down pools at upos / dpos (+ base),
// neighbours' deleted / depth / aff updated, state[v] = 2.
void launch_record(const uint32_t* S, uint32_t nS, uint32_t rank0, Overlay g,
                   const uint32_t* upos, const uint32_t* dpos, uint64_t ubase, uint64_t dbase,
                   uint32_t* rank, uint32_t* rec_v, uint64_t* rec_uo, uint32_t* rec_un,
                   uint64_t* rec_do, uint32_t* rec_dn, uint32_t* upool, uint32_t* dpool,
                   uint32_t* deleted, uint32_t* depth, uint32_t* aff, uint8_t* state,
                   hipStream_t s);
// Compact valid slots into sc (uint4 u, x, w, 0) and count them per endpoint
// (cnt_o[u]++, cnt_i[x]++, aff of both = 1).
void launch_compact_shortcuts(const uint32_t* slots, const uint32_t* sflag, const uint32_t* spos,
                              uint32_t nslots, uint32_t* sc, uint32_t* cnt_o, uint32_t* cnt_i,
                              uint32_t* aff, hipStream_t s);
// Affected list A (nodes of R' with aff): capacities of their new lists
// (c0 out, c1 in) and shortcut counts (c2 out, c3 in); zeros at index nA.
void launch_aff_counts(const uint32_t* A, uint32_t nA, Overlay g, const uint32_t* cnt_o,
                       const uint32_t* cnt_i, uint32_t* c0, uint32_t* c1, uint32_t* c2,
                       uint32_t* c3, hipStream_t s);
// Per-node bucket starts (bo_o / bo_i indexed by node) from the scans over A.
void launch_bucket_starts(const uint32_t* A, uint32_t nA, const uint32_t* s2, const uint32_t* s3,
                          uint32_t* bo_o, uint32_t* bo_i, hipStream_t s);
// Scatter shortcuts into the per-node buckets (uint2 key, w): bucket_o by
// tail (key = head), bucket_i by head (key = tail).  cur_o / cur_i: zeroed.
void launch_fill_buckets(const uint32_t* sc, uint32_t nsc, const uint32_t* bo_o,
                         const uint32_t* bo_i, uint32_t* cur_o, uint32_t* cur_i,
                         uint32_t* bucket_o, uint32_t* bucket_i, hipStream_t s);
// New lists of the affected nodes: old list minus done nodes merged with the
// node's bucket (sorted by (key, w)), lightest weight per neighbour, written
// at the arena offsets obase + s0[i] (out) / ibase + s1[i] (in); degrees
// updated, *maxdeg = max degree seen.
void launch_merge(const uint32_t* A, uint32_t nA, uint32_t* ooff, uint32_t* odeg, uint32_t* ioff,
                  uint32_t* ideg, uint32_t* arcs, const uint8_t* state, const uint32_t* s0,
                  const uint32_t* s1, uint32_t obase, uint32_t ibase, const uint32_t* bo_o,
                  const uint32_t* bo_i, const uint32_t* cnt_o, const uint32_t* cnt_i,
                  uint32_t* bucket_o, uint32_t* bucket_i, uint32_t* maxdeg, hipStream_t s);
// Simulation pair counts of list[0..k) (c0 = in-degree if out-degree > 0,
// index k: 0); sc[node] = 0.
void launch_sim_counts(const uint32_t* list, uint32_t k, Overlay g, uint32_t* c0, uint32_t* sc,
                       hipStream_t s);
// prio = a*(sc - in - out) + b*deleted + c*depth for list[0..k); aff, cnt_o,
// cnt_i, cur_o, cur_i of those nodes cleared.
void launch_prio(const uint32_t* list, uint32_t k, Overlay g, const uint32_t* sc,
                 const uint32_t* deleted, const uint32_t* depth, int64_t a, int64_t b, int64_t c,
                 int64_t* prio, uint32_t* aff, uint32_t* cnt_o, uint32_t* cnt_i, uint32_t* cur_o,
                 uint32_t* cur_i, hipStream_t s);
// Copy the lists of list[0..k) to a fresh arena at s0 (out) / s1 + ibase (in)
// — arena compaction; s0 / s1 scans of the degrees.
void launch_compact_lists(const uint32_t* list, uint32_t k, uint32_t* ooff, const uint32_t* odeg,
                          uint32_t* ioff, const uint32_t* ideg, const uint32_t* arcs_old,
                          uint32_t* arcs_new, const uint32_t* s0, const uint32_t* s1,
                          uint32_t ibase, hipStream_t s);
// flag[i] = f[list[i]] != 0 (index k: 0).
void launch_gather_flag(const uint32_t* list, uint32_t k, const uint32_t* f, uint32_t* flag,
                        hipStream_t s);
// c0[i] = odeg[list[i]], c1[i] = ideg[list[i]] (index k: 0).
void launch_deg_counts(const uint32_t* list, uint32_t k, Overlay g, uint32_t* c0, uint32_t* c1,
                       hipStream_t s);

}  // namespace chk
}  // namespace cpd

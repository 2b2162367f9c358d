// Host-callable launchers for the gfx950 kernels in cpd_kernels.hip.
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace cpd {

// Arm a start/stop event pair for the NEXT launch on this thread (consumed by
// it); the events record the kernel's own begin/end timestamps.
void set_launch_events(hipEvent_t start, hipEvent_t stop);

// Narrow final-distance rows (the down-sweep's output, read by first_moves):
// per 256-target group g of the batch (one wave: 64 lanes x 4 targets) and
// column c, base[g * n + c] = the minimum of the group's finite distances
// (0xFFFFFFFF if none) and d16[c * B + target] = distance - base as u16, with
// 0xFFFF = unreachable.  Halves the bytes of the two dominant kernels.  (The
// group-major base layout lets neighbouring slots, which gather neighbouring
// columns, share base lines; column-major, which puts a wave's two groups in
// one line, measured 6% slower in the down-sweep: 31.0 vs 29.1 ms/step.)  A
// group row whose finite spread reaches 0xFFFF is stored 32-bit in a pool
// row instead (1 KiB: the group's 256 distances), with base 0xFFFFFFFE and
// the pool row's index in every u32 word of its d16 group row; *ovf (zeroed
// before the down-sweep) counts the pool rows taken — past `cap` they were
// not stored and the batch must be rebuilt narrower.  Every finite distance
// must stay below 0xFFFFFFFE.  d16 == nullptr: every row in the dense `dist`.
struct NarrowRows {
    uint16_t* d16;
    uint32_t* base;
    uint32_t n;
    uint32_t* ovf;
    uint32_t* pool;
    uint32_t cap;
};

// The up-sweep's rows live in their own compact store, up[u][B] u32 (and
// live[u]), u = ascending slot - ubase: only nodes of upward level >= 2 (the
// levels below are closed forms) own a row there.  Ascending arcs into such
// nodes carry u (not the column); the down-sweep reads a node's own up row
// at the index its descriptor word 3 (narrow) or uidx[slot] (dense) holds
// (~0: none).  Two stores, one per batch slot, so batch k+1's up-sweep runs
// beside batch k's down-sweep.

// One CH sweep level: `count` node slots starting at `slot0` of the
// level-ordered node list; count * slabs workgroups of 256 threads, one slab =
// 1024 targets of the B-wide batch row, XCD-remapped (CPD_XCD=0: off).
// asc_*: the ascending sweep's arrays, read by both directions for the
// level-1 closed forms (see kL1Bit in cpd_kernels.hip).
// live (n u32, may be null = no skipping): bit b of live[col] = slab b of the
// column's up-sweep row holds finite values; the up-sweep computes and writes
// only those (sweep_up_sparse), the down-sweep's own-row reads skip the rest.
// tmask (n u32): bit b of tmask[col] = col is a target of slab b
// (launch_target_mask); B <= 32768 so that a mask fits in 32 bits.
// fmleaf (may be null; down-sweep, 4-bit sets, shift <= 2): leaf slots take
// their out-edges from adj and also store their first-move sets there.
// up / ubase / uidx: the compact up store (above); dist: the dense final rows
// (down-sweep without narrow rows only).
void launch_sweep(bool ascend, const uint32_t* nodes, const uint32_t* arc_off,
                  const uint32_t* arcs /* (col or up index, w) pairs */, uint32_t slot0,
                  uint32_t count, uint32_t* dist, uint32_t* up, uint32_t ubase,
                  const uint32_t* uidx, const uint32_t* tgt, uint32_t B, uint32_t slabs,
                  const uint32_t* asc_nodes, const uint32_t* asc_off, const uint32_t* asc_arcs,
                  uint32_t* live, const uint32_t* tmask, const uint32_t* adj, uint32_t shift,
                  uint16_t* fmleaf, NarrowRows nr, const uint32_t* desc, hipStream_t s);

// Down-sweep slot descriptors for the narrow down-sweep (desc arg of
// launch_sweep): 32 u32 per slot = node word, first arc, end arc, up index, then the
// slot's first down_desc_arcs() arcs as (column, weight), (kNoEdge, 0) past
// the end of its list; words 16.. for a level-1 node (kL1Bit): its column,
// its number of (leaf) down-arcs, then the first 4 of them as (column,
// weight) — the ascending list's arcs with the leaf bit cleared.
uint32_t down_desc_arcs();

// Narrow upward levels, chunked: items (slot, first arc, end arc, 0) of at
// most sweep_chunk_arcs() arcs each, nitems x slabs workgroups, partial
// minima folded in with atomicMin.  The rows of every node handled this way
// must first be set to their leaf form by launch_sweep_up_init (slots: their
// ascending slots), which also seeds live[u] = tmask[col].
void launch_sweep_up_init(const uint32_t* slots, uint32_t nslots, const uint32_t* nodes,
                          uint32_t* up, uint32_t ubase, const uint32_t* tgt, uint32_t B,
                          uint32_t slabs, uint32_t* live, const uint32_t* tmask, hipStream_t s);
void launch_sweep_up_chunks(const uint32_t* items /* uint4 each */, uint32_t nitems,
                            const uint32_t* arcs, uint32_t* up, uint32_t ubase,
                            const uint32_t* tgt, uint32_t B, uint32_t slabs,
                            const uint32_t* asc_nodes, const uint32_t* asc_off,
                            const uint32_t* asc_arcs, uint32_t* live, const uint32_t* tmask,
                            hipStream_t s);
uint32_t sweep_chunk_arcs();

// tmask[tgt[i]] |= 1 << (i / 1024) for i < B; tmask must be zeroed first.
void launch_target_mask(const uint32_t* tgt, uint32_t B, uint32_t* tmask, hipStream_t s);

// Row counts behind the live masks for the bytes model (timing runs): over
// node slots [slot0, slot1) of one sweep direction, stat[2 * lvl_of[slot]]
// += rows stored (up) / own rows read (down), stat[2 * lvl + 1] += rows
// gathered (up).  stat must be zeroed by the caller.  live is indexed by up
// index: slot - ubase (ascending), uidx[slot] (descending).
void launch_live_stats(bool ascend, const uint32_t* nodes, const uint32_t* arc_off,
                       const uint32_t* arcs, const uint32_t* lvl_of, uint32_t slot0,
                       uint32_t slot1, uint32_t ubase, const uint32_t* uidx,
                       const uint32_t* live, unsigned int* stat, hipStream_t s);

// Bits per first-move set for a packed adjacency of 2^shift slots per column:
// max(4, 2^shift) (>= the max out-degree); sets are stored 32/bits per u32.
uint32_t fm_bits(uint32_t shift);

// adj: the packed fixed-stride adjacency (free-flow weights), 2^shift slots;
// fm: [rows][npad] sets of fm_bits(shift) bits, npad * bits / 32 words per row.
// leafbits (npad/32 words, bit = column is a CH leaf) + fmleaf ([col][B/4]
// u16, 4 nibbles per lane, written by the down-sweep): leaf columns copy their
// sets instead of recomputing them; both null = every column computed.  Only
// for 4-bit sets (shift <= 2).
// seg_order (may be null; npad / 32 entries, a permutation): the order the
// 32-column segments are handed to the workgroups (the narrow 4-slot kernel).
void launch_first_moves(const uint32_t* adj, uint32_t shift, const uint32_t* dist,
                        const uint32_t* tgt, uint32_t B, uint32_t rows, uint32_t n,
                        uint32_t npad, uint32_t* fm, const uint32_t* leafbits,
                        const uint16_t* fmleaf, NarrowRows nr, hipStream_t s,
                        const uint32_t* seg_order = nullptr);
// Whether that launch reads each computed column's own distance row (the
// pipelined narrow kernel derives it from the neighbour rows instead).
bool first_moves_reads_own(uint32_t shift, bool narrow);

// Row width of the tiled first-move rows: npad is a multiple of this.
constexpr uint32_t kFmTile = 2048;

// Greedy RLE count, one wave per row: counts[row] = runs per row, and per
// 32-column segment the scan's entry state and the runs ending inside it
// (st / rc, [nrows][npad/32] u32 / u8).  fmb = fm_bits(shift).  gate (may be
// null): the launch does nothing unless *gate != 0 when it runs.
void launch_rle_count(const uint32_t* fm, uint32_t fmb, uint32_t npad, uint32_t nrows,
                      uint32_t* counts, uint32_t* st, uint8_t* rc, hipStream_t s,
                      const uint32_t* gate = nullptr);

// The compact row form: each row's greedy RLE row as a move table at
// 2^lb bits per column (lb = 0, 1, 2; column c in bits [b c, b c + b) of the
// row, npad * b / 32 words per row — the dense table the walks read), from
// the first-move sets and the count pass's segment states st / rc; batch row
// r goes to dense row out_row[r].
void launch_rle_moves(const uint32_t* fm, uint32_t fmb, uint32_t npad, uint32_t nrows,
                      const uint32_t* st, const uint8_t* rc, const uint32_t* out_row,
                      uint32_t lb, uint32_t* dense, hipStream_t s);
// Count and emit fused (4-bit sets; cpd_kernels.hip rle_emit4): the move
// tables as launch_rle_moves writes them and counts[r] = row r's runs, each
// set read once, no segment states; then rle_emit_fix redoes the rare chunk
// whose guessed entry was wrong.  xe / xs / cc: nrows x rle_emit_chunks(npad)
// u32 each (the chunks' guessed entries, exits and breaks).
uint32_t rle_emit_chunks(uint32_t npad);
void launch_rle_emit(const uint32_t* fm, uint32_t npad, uint32_t nrows, const uint32_t* out_row,
                     uint32_t lb, uint32_t* dense, uint32_t* xe, uint32_t* xs, uint32_t* cc,
                     uint32_t* counts, hipStream_t s);
// Rows of moves from one width to another: src rows of s_bits per column at
// s_stride words per row (s_words of them valid), dst rows of d_bits at
// d_stride, d_words written per row (input past s_words reads as 0).  The
// file / wire form is d_words = d_stride = ceil(n * bits / 32).  lost (may be
// null): |= 1 when some move does not fit d_bits.
void launch_repack_moves(const uint32_t* src, uint32_t s_stride, uint32_t s_words,
                         uint32_t s_bits, uint32_t rows, uint32_t* dst, uint32_t d_stride,
                         uint32_t d_words, uint32_t d_bits, hipStream_t s,
                         uint32_t* lost = nullptr);
// Move tables (row r at dense + r * stride words, 2^lb bits per column) back
// to RLE words: runs start at column 0 and wherever the move changes (columns
// >= n ignored).  count: counts[r] = runs of row r; runs: row r's words at
// runs[off[r] - base].
void launch_moves_count(const uint32_t* dense, uint32_t stride, uint32_t lb, uint32_t n,
                        uint32_t nrows, uint32_t* counts, hipStream_t s);
void launch_moves_runs(const uint32_t* dense, uint32_t stride, uint32_t lb, uint32_t n,
                       uint32_t nrows, const uint64_t* off, uint64_t base, uint32_t* runs,
                       hipStream_t s);

// Chunked RLE count (4-bit sets; cpd_kernels.hip rle_count_ch): the same st /
// rc as launch_rle_count, with each chunk of segments scanned by one lane
// from a guessed entry state; launch_rle_fix then repairs the chunk seams and
// writes counts[row], or sets *hard (zeroed by the caller) when a row's runs
// are too long for that to be cheap: the caller then runs launch_rle_count
// on the batch instead.  cc: nrows x rle_count_chunks(npad) u32; xs: twice
// that (the chunks' exit states, then their guessed entry states).
// (8- and 16-bit sets use launch_rle_count.)
uint32_t rle_count_chunks(uint32_t npad);
void launch_rle_count_ch(const uint32_t* fm, uint32_t npad, uint32_t nrows, uint32_t* st,
                         uint8_t* rc, uint32_t* xs, uint32_t* cc, hipStream_t s);
void launch_rle_fix(const uint32_t* fm, uint32_t npad, uint32_t nrows, uint32_t* st,
                    uint8_t* rc, uint32_t* xs, uint32_t* cc, uint32_t* counts, uint32_t* hard,
                    hipStream_t s);

// *bad |= 1 if some row [0, nrows) of (offsets, runs) does not start at column
// 0, has non-increasing run columns, a column >= n or a move >= mlimit (16:
// any; a narrower table's 2^bits) (empty rows: refused by the caller).  Rows
// from outside the library pass this before expand_rows / the walks touch
// them.  chunk_first / total_chunks as for launch_expand_rows.
void launch_validate_rows(const uint64_t* offsets, const uint32_t* runs,
                          const uint32_t* chunk_first, uint32_t nrows, uint32_t total_chunks,
                          uint32_t n, uint32_t mlimit, uint32_t* bad, hipStream_t s);

// RLE rows -> dense 4-bit move tables, npad/8 words per row (narrower
// tables: into a stage, then launch_repack_moves).  Work is cut in
// chunks of expand_chunk_runs() runs: chunk_first[row] (nrows + 1 values) =
// sum over earlier rows of ceil(R / expand_chunk_runs()), total_chunks its
// last value.  Rows must be well formed (validate_rows).
uint32_t expand_chunk_runs();
void launch_expand_rows(const uint64_t* offsets, const uint32_t* runs, const uint32_t* chunk_first,
                        uint32_t nrows, uint32_t total_chunks, uint32_t npad, uint32_t* dense,
                        hipStream_t s);
// Query batches on the GPU (cpd_query_prepare / _fetch): key[q] = row of
// t[q]'s column (row_of_col[order[t[q]]]), val[q] = q, *bad |= 1 for a node
// >= n, 2 for a target without a row; a stable radix sort of (key, val) by
// the low ceil(log2 nrows) bits (tmp: query_sort_bytes(nq) bytes); the
// sorted queries' columns and rows; results back to the caller's order
// (out[perm[i] * k + j] = in[i * k + j]).
void launch_query_keys(const uint32_t* s, const uint32_t* t, uint32_t nq, uint32_t n,
                       const uint32_t* order, const uint32_t* row_of_col, uint32_t* key,
                       uint32_t* val, uint32_t* bad, hipStream_t st);
size_t query_sort_bytes(uint32_t nq);
void launch_query_sort(void* tmp, size_t tmp_bytes, const uint32_t* key_in, uint32_t* key_out,
                       const uint32_t* val_in, uint32_t* val_out, uint32_t nq, uint32_t nrows,
                       hipStream_t st);
void launch_query_gather(const uint32_t* s, const uint32_t* t, const uint32_t* order,
                         const uint32_t* key, const uint32_t* val, uint32_t nq, uint32_t* qs,
                         uint32_t* qt, uint32_t* qrow, hipStream_t st);
void launch_scatter_u64(const uint64_t* in, const uint32_t* perm, uint32_t nq, uint64_t* out,
                        hipStream_t st);
void launch_scatter_u32(const uint32_t* in, const uint32_t* perm, uint32_t nq, uint32_t k,
                        uint32_t* out, hipStream_t st);
void launch_scatter_u8(const uint8_t* in, const uint32_t* perm, uint32_t nq, uint8_t* out,
                       hipStream_t st);

// table-search over dense move tables.  qs / qt: query columns, sorted by
// target row; qrow[q]: the row of query q's target (row_of_col is unused).
void launch_table_search_dense(const uint32_t* adj, uint32_t shift, const uint32_t* row_of_col,
                               const uint32_t* dense, uint32_t npad, uint32_t lb,
                               const uint32_t* qs, const uint32_t* qt, const uint32_t* qrow,
                               uint32_t nq, int32_t kmoves, uint32_t n, uint64_t* cost,
                               uint32_t* hops, uint8_t* fin, unsigned long long* agg,
                               hipStream_t s);

// adj: packed fixed-stride adjacency, (dst column, weight) pairs, 2^shift
// slots per column, dst = 0xFFFFFFFF past the out-degree.
void launch_table_search(const uint32_t* adj, uint32_t shift, const uint32_t* row_of_col,
                         const uint64_t* offsets, const uint32_t* runs, const uint32_t* qs,
                         const uint32_t* qt, const uint32_t* qrow, uint32_t nq, int32_t kmoves,
                         uint32_t n, uint64_t* cost, uint32_t* hops, uint8_t* fin,
                         unsigned long long* agg, hipStream_t s);

// CPD-heuristic search (cpd_kernels.hip "CPD-heuristic search"): one search
// per query (sorted by target row, qrow as for table-search) over the dense
// move rows (2^lb bits per column); adj_f / adj_w: packed adjacency with
// free-flow / selected weights.  The CPD path values come from the per-row
// tables hrow / crow / lrow (n per row; launch_search_tables) when hrow is
// non-null, else from CPD walks memoised in the workspace.  cost / plen / fin
// per query, qstats[5 q + k] = expanded, inserted, touched, updated, surplus;
// agg[8] (zeroed by the caller) += sums of those, plen, finished,
// overflowed.  time_ns: 0 = none; tick_ns: 0 = wall clock, else the virtual
// clock (tick_ns per expansion and per touched edge).
// Tables for index rows [0, rows) by pointer jumping in chunks of chunk_rows
// rows; scratch = 48 B x chunk_rows x n; tcol[r] = row r's target column.
void launch_search_tables(const uint32_t* dense, uint32_t npad, uint32_t lb, const uint32_t* adj_f,
                          const uint32_t* adj_w, uint32_t shift, const uint32_t* tcol,
                          uint32_t rows, uint32_t n, void* scratch, uint32_t chunk_rows,
                          uint64_t* hrow, uint64_t* crow, uint32_t* lrow, int write_h,
                          hipStream_t s);
// Lane slots the search launches for nq queries (a multiple of 64); the
// workspace holds search_ws_bytes_per_slot(cap, tables) bytes per slot.
uint32_t search_slots(uint32_t nq);
uint64_t search_ws_bytes_per_slot(uint32_t cap, bool tables);
// Resumable overflow (cpd_kernels.hip "Resumable overflow"): a search that
// would outgrow its workspace stops before the pop and, when rout is set,
// copies its state into that pool (a record of at most
// search_spill_words(cap, tables) u32 words; *top bumps, cap_words bounds
// it), reports fin = 3 and at[q] = the record's word offset (fin = 2: no
// room in the pool, it restarts).  resume[q] != ~0 (resume may be null):
// query q continues from its record at rin + resume[q].
struct SearchSpillArgs {
    const unsigned long long* resume = nullptr;
    const uint32_t* rin = nullptr;
    unsigned long long* at = nullptr;
    uint32_t* rout = nullptr;
    unsigned long long* top = nullptr;
    unsigned long long cap_words = 0;
};
uint64_t search_spill_words(uint32_t cap, bool tables);
void launch_cpd_search(const uint32_t* adj_f, const uint32_t* adj_w, uint32_t shift,
                       const uint32_t* dense, uint32_t npad, uint32_t lb, const uint64_t* hrow,
                       const uint64_t* crow, const uint32_t* lrow, uint32_t n,
                       const uint32_t* qs, const uint32_t* qt, const uint32_t* qrow, uint32_t nq,
                       double hscale, double fscale, int32_t kmoves, int64_t itrs,
                       uint64_t time_ns, uint64_t tick_ns, void* ws, uint32_t cap,
                       uint32_t slots, const SearchSpillArgs& spill, uint64_t* cost,
                       uint32_t* plen, uint8_t* fin, uint32_t* qstats, unsigned long long* agg,
                       hipStream_t s);

}  // namespace cpd

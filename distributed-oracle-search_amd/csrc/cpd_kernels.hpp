// Host-callable launchers for the gfx950 kernels in cpd_kernels.hip.
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace cpd {

// Arm a start/stop event pair for the NEXT launch on this thread (consumed by
// it); the events record the kernel's own begin/end timestamps.
void set_launch_events(hipEvent_t start, hipEvent_t stop);

// One CH sweep level: `count` node slots starting at `slot0` of the
// level-ordered node list; grid (count, slabs) x 256 threads, one slab =
// 1024 targets of the B-wide batch row.
// asc_*: the ascending sweep's arrays, read by both directions for the
// level-1 closed forms (see kL1Bit in cpd_kernels.hip).
void launch_sweep(bool ascend, const uint32_t* nodes, const uint32_t* arc_off,
                  const uint32_t* arcs /* (col, w) pairs */, uint32_t slot0, uint32_t count, uint32_t* dist,
                  const uint32_t* tgt, uint32_t B, uint32_t slabs, const uint32_t* asc_nodes,
                  const uint32_t* asc_off, const uint32_t* asc_arcs, hipStream_t s);

// adj: the packed fixed-stride adjacency (free-flow weights), 2^shift slots
void launch_first_moves(const uint32_t* adj, uint32_t shift, const uint32_t* dist,
                        const uint32_t* tgt, uint32_t B, uint32_t rows, uint32_t n,
                        uint32_t npad, uint16_t* fm, hipStream_t s);

// Row width of the tiled first-move rows: npad is a multiple of this.
constexpr uint32_t kFmTile = 2048;

// Greedy RLE scan, one wave per row: runs per row, then the runs themselves
// written at off[row] (uint64 offsets into `runs`).
void launch_rle_count(const uint16_t* fm, uint32_t npad, uint32_t nrows, uint32_t* counts,
                      hipStream_t s);
void launch_rle_emit(const uint16_t* fm, uint32_t npad, uint32_t nrows, const uint64_t* off,
                     uint32_t* runs, hipStream_t s);

// RLE rows -> dense 4-bit move tables, npad/8 words per row.
void launch_expand_rows(const uint64_t* offsets, const uint32_t* runs, uint32_t nrows,
                        uint32_t npad, uint32_t* dense, hipStream_t s);
// table-search over dense move tables
void launch_table_search_dense(const uint32_t* adj, uint32_t shift, const uint32_t* row_of_col,
                               const uint32_t* dense, uint32_t npad, const uint32_t* qs,
                               const uint32_t* qt, uint32_t nq, int32_t kmoves, uint32_t n,
                               uint64_t* cost, uint32_t* hops, uint8_t* fin,
                               unsigned long long* agg, hipStream_t s);

// adj: packed fixed-stride adjacency, (dst column, weight) pairs, 2^shift
// slots per column, dst = 0xFFFFFFFF past the out-degree.
void launch_table_search(const uint32_t* adj, uint32_t shift, const uint32_t* row_of_col,
                         const uint64_t* offsets, const uint32_t* runs, const uint32_t* qs,
                         const uint32_t* qt, uint32_t nq, int32_t kmoves, uint32_t n,
                         uint64_t* cost, uint32_t* hops, uint8_t* fin, unsigned long long* agg,
                         hipStream_t s);

}  // namespace cpd

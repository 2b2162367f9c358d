// HIP kernels for gfx950 (MI355X, CDNA4).  Integer/byte work, HBM-bound: no
// MFMA.  Every kernel is written for wave64 and 256-thread workgroups.
//
// Data layout in HBM (column space = DFS-preorder position of a node):
//   dist  [col][B]   u32   one batch row of B targets per column; a wave's
//                          16-B/lane access covers 256 targets = 1 KiB
//   fm    [row][npad] FMB-bit first-move sets, row-major for the RLE scan;
//                          FMB = max(4, slots of the packed adjacency) >= the
//                          max out-degree: 4 bits on road lattices, a quarter
//                          of a u16; columns >= n are padded with the wildcard
//   moves [row][npad/8] u32  the rows as 4-bit move tables (rle_moves); RLE
//                          words (column << 4 | move) are decoded from them
//                          on demand (moves_runs)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "cpd_kernels.hpp"

namespace cpd {
namespace kern {

constexpr uint32_t INF = 0xFFFFFFFFu;
constexpr uint32_t kNoEdge = 0xFFFFFFFFu;  // packed adjacency padding past the out-degree

__device__ __forceinline__ uint32_t sat_add(uint32_t d, uint32_t w) {
    uint32_t s = d + w;
    return (s < d) ? INF : s;  // d == INF or overflow -> INF
}

// First-move rows are plain row-major [row][npad] FMB-bit sets: the first-move
// kernel writes each target's 32-column segment as FMB/4 16-B stores (one
// 16-B store at FMB = 4), and the RLE scan's lane l reads its 32 columns the
// same way.  The wildcard is all FMB bits: every real set lies inside them
// (FMB >= out-degree), so S & wildcard == S and lowest-bit(wildcard) == 0 as
// with the u16 0xFFFF of the oracle — the scan's output is unchanged.
#ifndef CPD_RLE_LOOKBACK
#define CPD_RLE_LOOKBACK 16  // RLE guess: columns of the predecessor's segment rescanned
#endif
constexpr uint32_t kSeg = 32;          // columns per lane
constexpr uint32_t kTile = 64 * kSeg;  // columns per wave tile (npad % kTile == 0)

template <int FMB>
struct FmFmt {
    static_assert(FMB == 4 || FMB == 8 || FMB == 16, "first-move set width");
    static constexpr uint32_t kAll = (1u << FMB) - 1u;  // wildcard
    static constexpr int kPer = 32 / FMB;               // columns per u32 word
    static constexpr int kWords = (int)kSeg / kPer;     // words per 32-column segment (= FMB)
};

// 4-bit first-move rows are stored row-group interleaved: the 32-column
// segment `seg` of rows 4g..4g+3 is one 64-B sector, row 4g + i's 16 B at
// piece i.  The first-move kernels' lane owns exactly those 4 rows, so it
// stores whole sectors (row-major 16-B pieces reached HBM as partial
// sectors: 1.83x the algorithmic write bytes); the RLE scan's block runs the
// 4 rows of a group in its 4 waves, which read the same sectors together.
// fm4_piece = uint4 index of row `row`'s piece of segment `seg`.
__device__ __forceinline__ size_t fm4_piece(uint32_t row, uint32_t nseg, uint32_t seg) {
    return ((size_t)(row >> 2) * nseg + seg) * 4u + (row & 3u);
}

// Workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share
// one; MI355X_MICROARCH.md "Workgroup dispatch, XCD placement").  Remap so that
// each XCD runs one contiguous range of logical blocks: neighbouring nodes and
// column segments, which gather the same distance rows, then share an XCD's
// 4 MiB L2.  A bijection on [0, total) for any total; speed only, never
// correctness.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t total) {
    const uint32_t q = total >> 3, r = total & 7u, x = b & 7u;
    return x * q + min(x, r) + (b >> 3);
}

// Closed forms for the two lowest upward levels, so they are never stored.
// A level-0 node ("leaf": no down-arcs) has d_up = 0 at its own target, INF
// elsewhere.  A level-1 node's down-arcs all end in leaves, so its d_up is
// min(leaf form of itself, w_j + leaf form of each leaf j) — a few compares
// against the lane's targets.  Encoding (arcs and down-sweep node slots):
//   kLeafBit | column            -> leaf closed form
//   kL1Bit   | ascending slot s  -> level-1 closed form over the ascending
//                                   list's node s and its (leaf) arcs
//   up index u (ascending arcs)  -> a row of the compact up store (gather)
//   column (down-sweep)          -> a final distance row (gather)
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kL1Bit = 0x40000000u;
constexpr uint32_t kIdxMask = 0x3FFFFFFFu;

__device__ __forceinline__ void min4(uint4& acc, const uint4 d, uint32_t w) {
    acc.x = min(acc.x, sat_add(d.x, w));
    acc.y = min(acc.y, sat_add(d.y, w));
    acc.z = min(acc.z, sat_add(d.z, w));
    acc.w = min(acc.w, sat_add(d.w, w));
}

__device__ __forceinline__ uint4 leaf4(const uint4 t, uint32_t col, uint32_t w) {
    return make_uint4(t.x == col ? w : INF, t.y == col ? w : INF, t.z == col ? w : INF,
                      t.w == col ? w : INF);
}

// The ascending sweep's arrays, read for level-1 closed forms.
struct Closed {
    const uint32_t* __restrict__ nodes;
    const uint32_t* __restrict__ off;
    const uint2* __restrict__ arcs;
};

__device__ __forceinline__ uint4 l1_val(const Closed& cf, uint32_t s, const uint4 t) {
    uint4 acc = leaf4(t, cf.nodes[s], 0u);
    const uint32_t a1 = cf.off[s + 1];
    for (uint32_t a = cf.off[s]; a < a1; ++a) {
        const uint2 e = cf.arcs[a];  // e.x = kLeafBit | leaf column
        min4(acc, leaf4(t, e.x & kIdxMask, 0u), e.y);
    }
    return acc;
}

// Up-sweep sparsity.  d_up(x, t) is finite only for x in t's upward search
// space: a few per cent of the (node, 1024-target slab) pairs at up-levels
// >= 2 on road graphs when a slab's targets are neighbours.
// live[col] bit b = slab b of the column's row holds a finite value (and was
// stored); the up-sweep computes exactly those slabs, readers of d_up (its own
// gathers, the down-sweep's own-row init) take INF outside them.  The mask of
// a row follows from its inputs alone — slabs holding the node as a target,
// plus the masks of its down-arcs' rows (closed forms: the slabs holding the
// leaf / level-1 targets) — because a finite input plus an arc weight stays
// finite (cpd_plan_create bounds every distance below 2^32 - 1).
// tmask[col] bit b = column col is a target of slab b (target_mask kernel).

// Value an arc contributes (before adding its weight); INF if !live.
__device__ __forceinline__ uint4 arc_val(const uint4* __restrict__ d4, const uint4 t, uint2 e,
                                         uint32_t B4, uint32_t l4, const Closed& cf,
                                         bool live) {
    if (!live) return make_uint4(INF, INF, INF, INF);
    if (e.x & kLeafBit) return leaf4(t, e.x & kIdxMask, 0u);
    if (e.x & kL1Bit) return l1_val(cf, e.x & kIdxMask, t);
    return d4[(size_t)e.x * B4 + l4];
}

// Narrow final-distance rows (NarrowRows in cpd_kernels.hpp): a wave's 256
// targets (group g = l4 / 64, wave-uniform) share one u32 base per column and
// hold u16 offsets from it, 0xFFFF = unreachable.  A lane's 4 targets are one
// 8-B access (512 B per wave instruction), half the wide row's bytes.  A group
// row whose finite spread does not fit is stored wide instead, in a 1-KiB
// pool row whose index fills its d16 words, and its base says so (kWideRow):
// readers branch on the (wave-uniform) base and read the pool row at the
// index their own d16 load brought.
constexpr uint32_t kNarrowInf = 0xFFFFu;
constexpr uint32_t kWideRow = 0xFFFFFFFEu;  // > every finite distance (cpd_graph_create)

__device__ __forceinline__ uint32_t wave_group(uint32_t l4) {
    return __builtin_amdgcn_readfirstlane(l4 >> 6);
}

__device__ __forceinline__ uint32_t dec16(uint32_t b, uint32_t q) {
    return q == kNarrowInf ? INF : b + q;
}

// A narrow row read in two halves, so that a kernel issues all of its
// gathers' base and offset loads before it waits for any (nl_issue), then
// decodes them (nl_finish): only the rare wide rows cost a second round trip.
struct NLoad {
    uint32_t b;
    uint2 q;
};

__device__ __forceinline__ NLoad nl_issue(const NarrowRows& nr, uint32_t col, uint32_t grp,
                                          uint32_t B4, uint32_t l4) {
    return NLoad{nr.base[(size_t)grp * nr.n + col],
                 reinterpret_cast<const uint2*>(nr.d16)[(size_t)col * B4 + l4]};
}

// pool row of a wide group row, as uint4 (64 per 256 targets)
__device__ __forceinline__ const uint4* pool_row(const NarrowRows& nr, uint32_t idx) {
    return reinterpret_cast<const uint4*>(nr.pool) + (size_t)idx * 64u;
}

__device__ __forceinline__ uint4 nl_finish(const NLoad& p, const NarrowRows& nr, uint32_t l4) {
    uint4 r = make_uint4(dec16(p.b, p.q.x & 0xFFFFu), dec16(p.b, p.q.x >> 16),
                         dec16(p.b, p.q.y & 0xFFFFu), dec16(p.b, p.q.y >> 16));
    if (p.b == kWideRow) r = pool_row(nr, p.q.x)[l4 & 63u];  // wave-uniform, rare
    return r;
}

__device__ __forceinline__ uint32_t enc16(uint32_t d, uint32_t b, bool& bad) {
    if (d == INF) return kNarrowInf;
    const uint32_t q = d - b;
    bad |= q >= kNarrowInf;
    return q;
}

// One CH sweep level, dense.  Logical block = (slot in the level, 1024-target
// slab), slots fastest, XCD-remapped (remap != 0): node v = nodes[slot]; its
// arcs (ref, w) are wave-uniform (scalar loads); each lane owns 4 consecutive
// targets.  ASCEND: upward sweep into the up store (row slot - ubase), init 0
// at the lane's own target else INF (used only when skipping is off,
// CPD_LIVE=0), gathers from up rows.  !ASCEND: downward sweep into the dense
// final rows `dist`, init = the node's up row uidx[slot] (INF outside
// live[u] when live != null) or its closed form for levels 0/1; gathers
// from final rows.  acc = min(acc, w + d[arc]) over the arcs, eight gathers
// in flight per wave.
//
// Leaf first moves (lf.out != null, 4-bit sets): a leaf (no down-arcs) has
// only higher-ranked out-neighbours, all final when the down-sweep reaches
// it, and its up-arcs ARE its out-edges.  So its block walks the out-edges in
// file order from the packed adjacency instead: d(v) = min over them (self
// loops excluded), and FM(v) = {k : w_k + d(v_k) == d(v)} from the same
// gathers, stored as 4 nibbles per lane in lf.out[col][B/4] (u16) for
// first_moves to copy — the leaf's own row and neighbour rows are not read
// again there.
struct LeafFm {
    const uint2* __restrict__ adj;  // packed adjacency, 2^shift <= 4 slots
    uint32_t shift;
    uint16_t* __restrict__ out;
};

template <bool ASCEND>
__global__ __launch_bounds__(256) void sweep_level(const uint32_t* __restrict__ nodes,
                                                   const uint32_t* __restrict__ arc_off,
                                                   const uint2* __restrict__ arcs,
                                                   uint32_t slot0, uint32_t count, uint32_t remap,
                                                   uint32_t* __restrict__ dist,
                                                   uint32_t* __restrict__ up, uint32_t ubase,
                                                   const uint32_t* __restrict__ uidx,
                                                   const uint4* __restrict__ tgt4,
                                                   uint32_t B4, Closed cf,
                                                   const uint32_t* __restrict__ live, LeafFm lf) {
    const uint32_t L = remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t slab = L / count;
    const uint32_t slot = slot0 + (L - slab * count);
    const uint32_t l4 = slab * blockDim.x + threadIdx.x;  // slab = blockDim.x x 4 targets
    const uint32_t vraw = nodes[slot];
    uint4* __restrict__ u4 = reinterpret_cast<uint4*>(up);
    // rows written and gathered: up rows (ASCEND), final rows (!ASCEND)
    uint4* __restrict__ d4 = ASCEND ? u4 : reinterpret_cast<uint4*>(dist);
    uint32_t row;  // the row this slot writes

    const uint4 t = tgt4[l4];
    uint32_t v;
    uint4 acc;
    if (ASCEND) {
        v = vraw;
        row = slot - ubase;
        acc = leaf4(t, v, 0u);
    } else if (vraw & kLeafBit) {
        v = vraw & kIdxMask;
        acc = leaf4(t, v, 0u);
        if (lf.out) {
            const uint32_t ns = 1u << lf.shift;
            uint2 e[4];
            uint4 x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                e[k] = (uint32_t)k < ns ? lf.adj[((size_t)v << lf.shift) + k]
                                        : make_uint2(0xFFFFFFFFu, 0u);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                x[k] = (e[k].x != 0xFFFFFFFFu && e[k].x != v) ? d4[(size_t)e[k].x * B4 + l4]
                                                              : make_uint4(INF, INF, INF, INF);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (e[k].x != 0xFFFFFFFFu && e[k].x != v) min4(acc, x[k], e[k].y);
            uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (e[k].x == 0xFFFFFFFFu) continue;
                const uint4 dv = e[k].x == v ? acc : x[k];  // self loop: d(v) itself
                const uint32_t w = e[k].y;
                b0 |= (sat_add(dv.x, w) == acc.x ? 1u : 0u) << k;
                b1 |= (sat_add(dv.y, w) == acc.y ? 1u : 0u) << k;
                b2 |= (sat_add(dv.z, w) == acc.z ? 1u : 0u) << k;
                b3 |= (sat_add(dv.w, w) == acc.w ? 1u : 0u) << k;
            }
            b0 = (t.x == v || acc.x == INF) ? 0xFu : b0;  // wildcard (target, unreachable)
            b1 = (t.y == v || acc.y == INF) ? 0xFu : b1;
            b2 = (t.z == v || acc.z == INF) ? 0xFu : b2;
            b3 = (t.w == v || acc.w == INF) ? 0xFu : b3;
            d4[(size_t)v * B4 + l4] = acc;
            lf.out[(size_t)v * B4 + l4] = (uint16_t)(b0 | (b1 << 4) | (b2 << 8) | (b3 << 12));
            return;
        }
    } else if (vraw & kL1Bit) {
        v = cf.nodes[vraw & kIdxMask];
        acc = l1_val(cf, vraw & kIdxMask, t);
    } else {
        v = vraw;
        const uint32_t u = uidx[slot];
        const bool own = !live || ((live[u] >> (l4 >> 8)) & 1u);  // live bits: 1024 targets
        acc = own ? u4[(size_t)u * B4 + l4] : make_uint4(INF, INF, INF, INF);
    }
    if (!ASCEND) row = v;
    const uint32_t a0 = arc_off[slot], a1 = arc_off[slot + 1];
    uint32_t a = a0;
    for (; a + 8 <= a1; a += 8) {
        uint2 e[8];
        uint4 x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = arcs[a + i];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = arc_val(d4, t, e[i], B4, l4, cf, true);
#pragma unroll
        for (int i = 0; i < 8; ++i) min4(acc, x[i], e[i].y);
    }
    for (; a < a1; ++a) {
        const uint2 e = arcs[a];
        min4(acc, arc_val(d4, t, e, B4, l4, cf, true), e.y);
    }
    d4[(size_t)row * B4 + l4] = acc;
}

// Down-sweep into narrow rows, 8 targets per lane.  The narrow rows halve the
// bytes per target, so a lane takes twice the targets of sweep_level to keep
// 16 B per lane per access (1 KiB per wave instruction): the same number of
// memory instructions moves the whole row in half the bytes.  Lanes 0-31 and
// 32-63 of a wave are two 256-target groups (base per group).  Logical block =
// (slot, 8 x blockDim targets), slots fastest, XCD-remapped; otherwise the
// same computation as sweep_level<false> (own init, closed forms, leaf first
// moves with lf.out).
struct U8 {
    uint4 a, b;
};

#ifndef CPD_DOWN8_INLINE
#define CPD_DOWN8_INLINE 6
#endif
// arcs inline in a down-sweep slot descriptor (4..6; a leaf's <= 4 out-edges
// always fit), gathered together; the rest of a list streams from `arcs`
constexpr uint32_t kDescArcs = CPD_DOWN8_INLINE;
static_assert(kDescArcs >= 4 && kDescArcs <= 6, "descriptor arcs");

__device__ __forceinline__ U8 inf8() {
    return U8{make_uint4(INF, INF, INF, INF), make_uint4(INF, INF, INF, INF)};
}

__device__ __forceinline__ void min8(U8& acc, const U8& d, uint32_t w) {
    min4(acc.a, d.a, w);
    min4(acc.b, d.b, w);
}

struct NLoad8 {
    uint32_t b;
    uint4 q;
};

__device__ __forceinline__ NLoad8 nl8_issue(const NarrowRows& nr, uint32_t col, uint32_t grp,
                                            uint32_t B8, uint32_t l8) {
    return NLoad8{nr.base[(size_t)grp * nr.n + col],
                  reinterpret_cast<const uint4*>(nr.d16)[(size_t)col * B8 + l8]};
}

__device__ __forceinline__ U8 nl8_finish(const NLoad8& p, const NarrowRows& nr, uint32_t l8) {
    U8 r{make_uint4(dec16(p.b, p.q.x & 0xFFFFu), dec16(p.b, p.q.x >> 16),
                    dec16(p.b, p.q.y & 0xFFFFu), dec16(p.b, p.q.y >> 16)),
         make_uint4(dec16(p.b, p.q.z & 0xFFFFu), dec16(p.b, p.q.z >> 16),
                    dec16(p.b, p.q.w & 0xFFFFu), dec16(p.b, p.q.w >> 16))};
    if (p.b == kWideRow) {  // uniform per half-wave, rare
        const uint4* pr = pool_row(nr, p.q.x) + 2u * (l8 & 31u);
        r.a = pr[0];
        r.b = pr[1];
    }
    return r;
}

// A half-wave (one 256-target group) stores its row narrow, or — when the
// spread does not fit 16 bits — takes a pool row (the head's atomic on the
// pool counter) and stores it there, the index in every d16 word.  Past the
// pool's capacity nothing is stored: the counter tells the host, which
// rebuilds the batch in pieces the pool holds (readers stay in bounds).
__device__ __forceinline__ void narrow_store8(const NarrowRows& nr, uint32_t col, uint32_t grp,
                                              uint32_t B8, uint32_t l8, const U8& acc) {
    uint32_t b = min(min(min(acc.a.x, acc.a.y), min(acc.a.z, acc.a.w)),
                     min(min(acc.b.x, acc.b.y), min(acc.b.z, acc.b.w)));
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) b = min(b, (uint32_t)__shfl_xor(b, o, 64));  // half-wave
    bool bad = false;
    const uint32_t q0 = enc16(acc.a.x, b, bad), q1 = enc16(acc.a.y, b, bad);
    const uint32_t q2 = enc16(acc.a.z, b, bad), q3 = enc16(acc.a.w, b, bad);
    const uint32_t q4 = enc16(acc.b.x, b, bad), q5 = enc16(acc.b.y, b, bad);
    const uint32_t q6 = enc16(acc.b.z, b, bad), q7 = enc16(acc.b.w, b, bad);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t m = __ballot(bad);
    const bool half_bad = ((lane < 32u ? m : (m >> 32)) & 0xFFFFFFFFull) != 0;
    const bool head = (lane & 31u) == 0;
    if (half_bad) {
        uint32_t p = 0;
        if (head) p = atomicAdd(nr.ovf, 1u);
        p = (uint32_t)__shfl((int)p, (int)(lane & 32u), 64);
        const bool fits = p < nr.cap;
        p = fits ? p : nr.cap - 1u;
        if (fits) {
            uint4* pr = reinterpret_cast<uint4*>(nr.pool) + (size_t)p * 64u + 2u * (l8 & 31u);
            pr[0] = acc.a;
            pr[1] = acc.b;
        }
        reinterpret_cast<uint4*>(nr.d16)[(size_t)col * B8 + l8] = make_uint4(p, p, p, p);
        if (head) nr.base[(size_t)grp * nr.n + col] = kWideRow;
        return;
    }
    const uint4 q = make_uint4(q0 | (q1 << 16), q2 | (q3 << 16), q4 | (q5 << 16), q6 | (q7 << 16));
    reinterpret_cast<uint4*>(nr.d16)[(size_t)col * B8 + l8] = q;
    if (head) nr.base[(size_t)grp * nr.n + col] = b;
}

__device__ __forceinline__ void fm_nib(const uint4& dv, const uint4& acc, uint32_t w, int k,
                                       uint32_t (&bits)[4]) {
    bits[0] |= (sat_add(dv.x, w) == acc.x ? 1u : 0u) << k;
    bits[1] |= (sat_add(dv.y, w) == acc.y ? 1u : 0u) << k;
    bits[2] |= (sat_add(dv.z, w) == acc.z ? 1u : 0u) << k;
    bits[3] |= (sat_add(dv.w, w) == acc.w ? 1u : 0u) << k;
}

__device__ __forceinline__ uint32_t fm_pack4(const uint4& t, const uint4& acc, uint32_t v,
                                             const uint32_t (&bits)[4]) {
    const uint32_t b0 = (t.x == v || acc.x == INF) ? 0xFu : bits[0];  // wildcard (target, unreachable)
    const uint32_t b1 = (t.y == v || acc.y == INF) ? 0xFu : bits[1];
    const uint32_t b2 = (t.z == v || acc.z == INF) ? 0xFu : bits[2];
    const uint32_t b3 = (t.w == v || acc.w == INF) ? 0xFu : bits[3];
    return b0 | (b1 << 4) | (b2 << 8) | (b3 << 12);
}

// Leaf slot of the narrow down-sweep: d(v) = min over the out-edges (all to
// final, higher-ranked nodes; a self loop never lowers it) and FM(v) = the
// edges attaining it, folded per neighbour as it is decoded (argmin set: a
// strictly smaller value restarts the set, an equal one joins it), so no
// neighbour row is held after its fold — the slot's registers stay at one
// pending gather set.  A self loop joins iff its weight is 0 (w + d(v) ==
// d(v)); the wildcard at the target and at unreachable v overrides.
// bits: the sets of 4 targets, one nibble each (target i at bits 4i..4i+3),
// packed to keep the slot's registers low.
template <int I>
__device__ __forceinline__ void argmin_fold(uint32_t& a, uint32_t& bits, uint32_t val, int k) {
    const uint32_t bit = 1u << (4 * I + k);
    const uint32_t restart = (bits & ~(0xFu << (4 * I))) | bit;
    bits = val < a ? restart : (val == a ? (bits | bit) : bits);
    a = min(a, val);
}

// 4 nibbles -> the stored sets with the wildcard at the target and at
// unreachable columns.
__device__ __forceinline__ uint32_t fm_wild4(const uint4& t, const uint4& acc, uint32_t v,
                                             uint32_t bits) {
    bits |= (t.x == v || acc.x == INF) ? 0x000Fu : 0u;
    bits |= (t.y == v || acc.y == INF) ? 0x00F0u : 0u;
    bits |= (t.z == v || acc.z == INF) ? 0x0F00u : 0u;
    bits |= (t.w == v || acc.w == INF) ? 0xF000u : 0u;
    return bits;
}

__device__ __forceinline__ void leaf_finish8(const uint2* e, const NLoad8 (&pl)[kDescArcs],
                                             uint32_t v, U8& acc, const U8& t, uint32_t l8,
                                             uint32_t grp, uint32_t B8,
                                             uint16_t* __restrict__ fmleaf, const NarrowRows& nr) {
    uint32_t ba = 0, bb = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (e[k].x == kNoEdge || e[k].x == v) continue;
        const U8 x = nl8_finish(pl[k], nr, l8);
        const uint32_t w = e[k].y;
        argmin_fold<0>(acc.a.x, ba, sat_add(x.a.x, w), k);
        argmin_fold<1>(acc.a.y, ba, sat_add(x.a.y, w), k);
        argmin_fold<2>(acc.a.z, ba, sat_add(x.a.z, w), k);
        argmin_fold<3>(acc.a.w, ba, sat_add(x.a.w, w), k);
        argmin_fold<0>(acc.b.x, bb, sat_add(x.b.x, w), k);
        argmin_fold<1>(acc.b.y, bb, sat_add(x.b.y, w), k);
        argmin_fold<2>(acc.b.z, bb, sat_add(x.b.z, w), k);
        argmin_fold<3>(acc.b.w, bb, sat_add(x.b.w, w), k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (e[k].x == v && e[k].y == 0u) {  // zero-weight self loop (wave-uniform)
            ba |= 0x1111u << k;
            bb |= 0x1111u << k;
        }
    const uint32_t sets = fm_wild4(t.a, acc.a, v, ba) | (fm_wild4(t.b, acc.b, v, bb) << 16);
    narrow_store8(nr, v, grp, B8, l8, acc);
    reinterpret_cast<uint32_t*>(fmleaf)[(size_t)v * B8 + l8] = sets;  // 8 nibbles
}

__device__ __forceinline__ void leaf_slot8(const uint2* e, uint32_t v, U8& acc, const U8& t,
                                           uint32_t l8, uint32_t grp, uint32_t B8,
                                           uint16_t* __restrict__ fmleaf, const NarrowRows& nr) {
    NLoad8 pl[kDescArcs];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (e[k].x != kNoEdge && e[k].x != v) pl[k] = nl8_issue(nr, e[k].x, grp, B8, l8);
    leaf_finish8(e, pl, v, acc, t, l8, grp, B8, fmleaf, nr);
}

// A down-sweep slot's descriptor (see down_desc_arcs): the 64-B head (node
// word, arc range, up index, first kDescArcs arcs) and, for a level-1 node, the
// closed-form part (c0..c2), all loaded together (one 128-B scalar fetch).
struct Desc8 {
    uint4 h, i0, i1, i2, c0, c1, c2;
};

__device__ __forceinline__ Desc8 load_desc8(const uint4* __restrict__ desc, uint32_t slot) {
    const uint4* __restrict__ dp = desc + (size_t)slot * 8u;
    return Desc8{dp[0], dp[1], dp[2], dp[3], dp[4], dp[5], dp[6]};
}

// Gathers in flight per step of a long arc list (past the descriptor's
// kDescArcs): the list tail is rare, and its registers set the kernel's
// occupancy (8 in flight: 88 VGPRs, 5 waves per SIMD).
#ifndef CPD_DOWN8_LONG
#define CPD_DOWN8_LONG 4
#endif
constexpr int kLong = CPD_DOWN8_LONG;

// One slot of the narrow down-sweep for the lane's 8 targets t.
__device__ __forceinline__ void down8_slot(const Desc8& D, const U8& t, uint32_t l8, uint32_t grp,
                                           uint32_t B4, uint32_t B8, const uint4* __restrict__ u4,
                                           const uint2* __restrict__ arcs, const Closed& cf,
                                           const uint32_t* __restrict__ live,
                                           uint16_t* __restrict__ fmleaf, const NarrowRows& nr) {
    // (node word, first arc, end arc, up index) + its first kDescArcs arcs (a
    // leaf's out-edges in file order); for a level-1 node also its column and
    // its <= 4 leaf arcs (closed form)
    const uint4 i0 = D.i0, i1 = D.i1, i2 = D.i2;
    const uint2 all6[6] = {make_uint2(i0.x, i0.y), make_uint2(i0.z, i0.w),
                           make_uint2(i1.x, i1.y), make_uint2(i1.z, i1.w),
                           make_uint2(i2.x, i2.y), make_uint2(i2.z, i2.w)};
    uint2 inl[kDescArcs];
#pragma unroll
    for (int i = 0; i < (int)kDescArcs; ++i) inl[i] = all6[i];
    const uint32_t vraw = D.h.x, a0 = D.h.y, a1 = D.h.z;
    uint32_t v;
    U8 acc;
    if (vraw & kLeafBit) {
        v = vraw & kIdxMask;
        acc = U8{leaf4(t.a, v, 0u), leaf4(t.b, v, 0u)};
        if (fmleaf) {  // out-degree <= 4 (4-bit sets): all inline
            leaf_slot8(inl, v, acc, t, l8, grp, B8, fmleaf, nr);
            return;
        }
    } else if (vraw & kL1Bit) {  // closed form from the descriptor
        const uint4 c0 = D.c0, c1 = D.c1, c2 = D.c2;
        v = c0.x;
        acc = U8{leaf4(t.a, v, 0u), leaf4(t.b, v, 0u)};
        const uint2 la[4] = {make_uint2(c0.z, c0.w), make_uint2(c1.x, c1.y),
                             make_uint2(c1.z, c1.w), make_uint2(c2.x, c2.y)};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if ((uint32_t)i < c0.y) {
                min4(acc.a, leaf4(t.a, la[i].x, 0u), la[i].y);
                min4(acc.b, leaf4(t.b, la[i].x, 0u), la[i].y);
            }
        if (c0.y > 4u) {  // more leaf arcs than fit: the ascending arrays
            const uint32_t s1 = vraw & kIdxMask;
            for (uint32_t a = cf.off[s1] + 4u; a < cf.off[s1 + 1]; ++a) {
                const uint2 e = cf.arcs[a];
                min4(acc.a, leaf4(t.a, e.x & kIdxMask, 0u), e.y);
                min4(acc.b, leaf4(t.b, e.x & kIdxMask, 0u), e.y);
            }
        }
    } else {
        v = vraw;
        const uint32_t u = D.h.w;  // its row in the up store
        const bool own = !live || ((live[u] >> (l8 >> 7)) & 1u);  // live bits: 1024 targets
        acc = own ? U8{u4[(size_t)u * B4 + 2u * l8], u4[(size_t)u * B4 + 2u * l8 + 1u]} : inf8();
    }
    {  // the inline arcs (kNoEdge past the list), gathers in flight together
        NLoad8 pl[kDescArcs];
#pragma unroll
        for (int i = 0; i < (int)kDescArcs; ++i)
            if (inl[i].x != kNoEdge) pl[i] = nl8_issue(nr, inl[i].x, grp, B8, l8);
#pragma unroll
        for (int i = 0; i < (int)kDescArcs; ++i)
            if (inl[i].x != kNoEdge) min8(acc, nl8_finish(pl[i], nr, l8), inl[i].y);
    }
    uint32_t a = a0 + kDescArcs;  // the rest of a long list (rare), kLong gathers at a time
    for (; a + kLong <= a1; a += kLong) {
        uint2 e[kLong];
#pragma unroll
        for (int i = 0; i < kLong; ++i) e[i] = arcs[a + i];
        NLoad8 pl[kLong];
#pragma unroll
        for (int i = 0; i < kLong; ++i) pl[i] = nl8_issue(nr, e[i].x, grp, B8, l8);
#pragma unroll
        for (int i = 0; i < kLong; ++i) min8(acc, nl8_finish(pl[i], nr, l8), e[i].y);
    }
    for (; a < a1; ++a) {
        const uint2 e = arcs[a];
        min8(acc, nl8_finish(nl8_issue(nr, e.x, grp, B8, l8), nr, l8), e.y);
    }
    narrow_store8(nr, v, grp, B8, l8, acc);
}


// Narrow down-sweep launch: logical block = (slot, 8 x blockDim targets),
// slots fastest, XCD-remapped; one slot per wave.  (Round 2 measured K > 1
// slots per wave with the next descriptor prefetched, and P slots' gathers in
// flight per wave: no faster — the scalar descriptor fetch is not on the
// critical path — and removed in round 3.)
__global__ __launch_bounds__(256) void sweep_down8(const uint4* __restrict__ desc,
                                                   const uint2* __restrict__ arcs,
                                                   uint32_t slot0, uint32_t count, uint32_t remap,
                                                   const uint32_t* __restrict__ up,
                                                   const uint4* __restrict__ tgt4, uint32_t B4,
                                                   Closed cf, const uint32_t* __restrict__ live,
                                                   uint16_t* __restrict__ fmleaf, NarrowRows nr) {
    const uint32_t L = remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t blk = L / count;
    const uint32_t s0 = slot0 + (L - blk * count);
    const uint32_t l8 = blk * blockDim.x + threadIdx.x;  // targets 8 l8 .. 8 l8 + 7
    const uint32_t grp = l8 >> 5;                        // uniform per half-wave
    const uint32_t B8 = B4 / 2u;
    const uint4* __restrict__ u4 = reinterpret_cast<const uint4*>(up);
    const U8 t{tgt4[2u * l8], tgt4[2u * l8 + 1u]};
    down8_slot(load_desc8(desc, s0), t, l8, grp, B4, B8, u4, arcs, cf, live, fmleaf, nr);
}

// Slab mask of an arc's source row (see "Up-sweep sparsity").
__device__ __forceinline__ uint32_t arc_mask(uint32_t ex, const uint32_t* __restrict__ live,
                                             const uint32_t* __restrict__ tmask,
                                             const Closed& cf) {
    if (ex & kLeafBit) return tmask[ex & kIdxMask];
    if (ex & kL1Bit) {
        const uint32_t s = ex & kIdxMask;
        uint32_t m = tmask[cf.nodes[s]];
        for (uint32_t a = cf.off[s]; a < cf.off[s + 1]; ++a) m |= tmask[cf.arcs[a].x & kIdxMask];
        return m;
    }
    return live[ex];
}

// Upward sweep level with row skipping.  Logical block = (slot, j), slots
// fastest, XCD-remapped; the block computes node v's live slabs b with
// b % nsplit == j (nsplit = 1 on wide levels: one block per node, its arcs
// read once; > 1 on narrow top levels so they still fill the GPU).  Each
// live slab: 256 threads x 4 targets as in sweep_level, gathers only from
// arcs live in that slab.  live[v] = the node's mask (every split writes the
// same value); nothing else of a dead slab is read or written.
// The up-sweep runs on its own stream beside the down-sweep and the first
// moves, so its kernels are one-wave workgroups of <= 64 VGPRs: a workgroup
// of four 96-VGPR waves needed four SIMDs of one CU to free room at once
// while the main stream's 58-VGPR waves refilled every hole first — the up
// levels waited 200-450 us each (round 6, profiles/up_store_ab/); one wave
// of <= 64 VGPRs fits the slot any retiring down-sweep wave leaves.  A wave
// covers a quarter slab (256 targets, 4 per lane): q = its quarter.
constexpr uint32_t kUpQ = 4;  // waves (quarters) per 1024-target slab

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) void sweep_up_sparse(
    const uint32_t* __restrict__ nodes, const uint32_t* __restrict__ arc_off,
    const uint2* __restrict__ arcs, uint32_t slot0, uint32_t count, uint32_t nsplit,
    uint32_t remap, uint32_t* __restrict__ up, uint32_t ubase, const uint4* __restrict__ tgt4,
    uint32_t B4, Closed cf, uint32_t* __restrict__ live, const uint32_t* __restrict__ tmask,
    uint32_t active) {
    const uint32_t L = remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t jq = L / count;
    const uint32_t slot = slot0 + (L - jq * count);
    const uint32_t j = jq / kUpQ, q = jq - j * kUpQ;
    const uint32_t v = nodes[slot];   // column: the target test and tmask
    const uint32_t u = slot - ubase;  // row in the up store
    const uint32_t a0 = arc_off[slot], a1 = arc_off[slot + 1];
    const uint32_t* __restrict__ live_in = live;  // rows of finished levels only
    uint32_t m = tmask[v];
    for (uint32_t a = a0; a < a1; ++a) m |= arc_mask(arcs[a].x, live_in, tmask, cf);
    m &= active;
    if (threadIdx.x == 0 && j == 0 && q == 0) live[u] = m;
    uint4* __restrict__ d4 = reinterpret_cast<uint4*>(up);
    for (uint32_t mm = m; mm; mm &= mm - 1u) {
        const uint32_t slab = (uint32_t)__builtin_ctz(mm);
        if (slab % nsplit != j) continue;
        const uint32_t l4 = slab * 256u + q * 64u + threadIdx.x;
        const uint4 t = tgt4[l4];
        uint4 acc = leaf4(t, v, 0u);
        uint32_t a = a0;
        for (; a + 8 <= a1; a += 8) {
            uint2 e[8];
            uint4 x[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) e[i] = arcs[a + i];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                x[i] = arc_val(d4, t, e[i], B4, l4, cf,
                               (arc_mask(e[i].x, live_in, tmask, cf) >> slab) & 1u);
#pragma unroll
            for (int i = 0; i < 8; ++i) min4(acc, x[i], e[i].y);
        }
        for (; a < a1; ++a) {
            const uint2 e = arcs[a];
            min4(acc, arc_val(d4, t, e, B4, l4, cf, (arc_mask(e.x, live_in, tmask, cf) >> slab) & 1u),
                 e.y);
        }
        d4[(size_t)u * B4 + l4] = acc;
    }
}

// Narrow upward levels (the top of the hierarchy: few nodes, each with up to
// hundreds of down-arcs) are latency-bound when one block walks a node's arcs
// eight at a time.  There, work items = (node, chunk of <= kChunk arcs) x
// slab: every block issues its chunk's mask loads and gathers at once and
// folds its partial minimum into the row with atomicMin; the rows start as the
// leaf form (sweep_up_init, once per batch) and live[v] collects the chunks'
// masks with atomicOr.
constexpr int kChunk = 8;

// Grid-stride over (column, slab) rows with a small grid: the init runs on the
// early up-sweep stream beside the previous batch's first moves, and one block
// per 4-KiB row (~240k blocks at 1M nodes) would be dispatched round-robin
// with first_moves' blocks and end with it, holding back every up level.
__global__ __launch_bounds__(64) void sweep_up_init(const uint32_t* __restrict__ slots,
                                                     uint32_t nslots, uint32_t total,
                                                     const uint32_t* __restrict__ nodes,
                                                     uint32_t* __restrict__ up, uint32_t ubase,
                                                     const uint4* __restrict__ tgt4, uint32_t B4,
                                                     uint32_t* __restrict__ live,
                                                     const uint32_t* __restrict__ tmask,
                                                     uint32_t active) {
    for (uint32_t L = blockIdx.x; L < total; L += gridDim.x) {  // (slot, quarter slab)
        const uint32_t sq = L / nslots;
        const uint32_t s = slots[L - sq * nslots];
        const uint32_t v = nodes[s], u = s - ubase;
        const uint32_t l4 = sq * 64u + threadIdx.x;
        reinterpret_cast<uint4*>(up)[(size_t)u * B4 + l4] = leaf4(tgt4[l4], v, 0u);
        if (sq == 0 && threadIdx.x == 0) live[u] = tmask[v] & active;
    }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) void sweep_up_chunks(
    const uint4* __restrict__ items, uint32_t nitems, uint32_t remap,
    const uint2* __restrict__ arcs, uint32_t* __restrict__ up, uint32_t ubase,
    const uint4* __restrict__ tgt4, uint32_t B4, Closed cf,
    uint32_t* __restrict__ live, const uint32_t* __restrict__ tmask, uint32_t active) {
    const uint32_t L = remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t sq = L / nitems;  // (slab, quarter)
    const uint32_t slab = sq / kUpQ, q = sq - slab * kUpQ;
    const uint4 it = items[L - sq * nitems];  // (slot, first arc, end arc, -)
    const uint32_t v = it.x - ubase;              // its row in the up store
    const uint32_t* __restrict__ live_in = live;  // lower levels' masks only
    uint2 e[kChunk];
    uint32_t mk[kChunk], pm = 0;
#pragma unroll
    for (int i = 0; i < kChunk; ++i) e[i] = it.y + i < it.z ? arcs[it.y + i] : make_uint2(0u, 0u);
#pragma unroll
    for (int i = 0; i < kChunk; ++i) {
        mk[i] = it.y + i < it.z ? arc_mask(e[i].x, live_in, tmask, cf) & active : 0u;
        pm |= mk[i];
    }
    if (sq == 0 && threadIdx.x == 0 && pm) atomicOr(&live[v], pm);
    if (!((pm >> slab) & 1u)) return;
    const uint32_t l4 = slab * 256u + q * 64u + threadIdx.x;
    const uint4 t = tgt4[l4];
    const uint4* __restrict__ d4 = reinterpret_cast<const uint4*>(up);
    uint4 x[kChunk];
#pragma unroll
    for (int i = 0; i < kChunk; ++i) x[i] = arc_val(d4, t, e[i], B4, l4, cf, (mk[i] >> slab) & 1u);
    uint4 acc = make_uint4(INF, INF, INF, INF);
#pragma unroll
    for (int i = 0; i < kChunk; ++i) min4(acc, x[i], e[i].y);
    uint32_t* row = up + ((size_t)v * B4 + l4) * 4u;
    if (acc.x != INF) atomicMin(row + 0, acc.x);
    if (acc.y != INF) atomicMin(row + 1, acc.y);
    if (acc.z != INF) atomicMin(row + 2, acc.z);
    if (acc.w != INF) atomicMin(row + 3, acc.w);
}


// tmask[col] |= 1 << slab for every target lane (4 per thread) of the batch;
// the caller zeroes tmask first.
__global__ __launch_bounds__(64) void target_mask(const uint32_t* __restrict__ tgt, uint32_t B,
                                                  uint32_t* __restrict__ tmask) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i < B) atomicOr(&tmask[tgt[i]], 1u << (i >> 10));
}

// Row counts of one batch's sweeps for the bytes model (timing runs only),
// thread per node slot of one sweep direction:
//   ASCEND (slots of up-levels >= 2): stat[2 l] += rows stored (slabs of the
//     slot's live mask), stat[2 l + 1] += rows gathered (its materialised
//     arcs' live slabs);
//   !ASCEND: stat[2 l] += own rows read (live slabs of materialised slots).
// lvl_of[slot] = the slot's level; counts are aggregated per wave when all
// lanes share a level (slots are level-ordered), so atomics are few — a
// per-block atomic on one word per level would serialise ~10^6 blocks.
template <bool ASCEND>
__global__ __launch_bounds__(256) void live_stats(const uint32_t* __restrict__ nodes,
                                                  const uint32_t* __restrict__ arc_off,
                                                  const uint2* __restrict__ arcs,
                                                  const uint32_t* __restrict__ lvl_of,
                                                  uint32_t slot0, uint32_t slot1, uint32_t ubase,
                                                  const uint32_t* __restrict__ uidx,
                                                  const uint32_t* __restrict__ live,
                                                  unsigned int* __restrict__ stat) {
    const uint32_t slot = slot0 + blockIdx.x * 256u + threadIdx.x;
    uint32_t own = 0, gathered = 0, lvl = 0xFFFFFFFFu;
    if (slot < slot1) {
        lvl = lvl_of[slot];
        const uint32_t v = nodes[slot];
        if (ASCEND) own = __builtin_popcount(live[slot - ubase]);
        else if (!(v & (kLeafBit | kL1Bit))) own = __builtin_popcount(live[uidx[slot]]);
        if (ASCEND)
            for (uint32_t a = arc_off[slot]; a < arc_off[slot + 1]; ++a) {
                const uint32_t c = arcs[a].x;
                if (!(c & (kLeafBit | kL1Bit))) gathered += __builtin_popcount(live[c]);
            }
    }
    const uint32_t l0 = __shfl(lvl, 0, 64);
    if (__all(lvl == l0)) {
        if (l0 == 0xFFFFFFFFu) return;
        unsigned int o = own, g = gathered;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) {
            o += __shfl_xor(o, d, 64);
            g += __shfl_xor(g, d, 64);
        }
        if ((threadIdx.x & 63u) == 0) {
            atomicAdd(&stat[2 * l0], o);
            if (ASCEND) atomicAdd(&stat[2 * l0 + 1], g);
        }
    } else if (lvl != 0xFFFFFFFFu) {
        atomicAdd(&stat[2 * lvl], own);
        if (ASCEND) atomicAdd(&stat[2 * lvl + 1], gathered);
    }
}

__device__ __forceinline__ uint32_t fm_bit(uint32_t dv, uint32_t w, uint32_t dn, uint32_t k) {
    return (sat_add(dv, w) == dn ? 1u : 0u) << k;
}

template <int FMB>
__device__ __forceinline__ uint32_t fm_final(uint32_t c, uint32_t tc, uint32_t dn, uint32_t bits) {
    return (c == tc || dn == INF) ? FmFmt<FMB>::kAll : bits;
}

// First-move sets.  Logical block = (one 32-column lane segment, 1024-target
// slab), segments fastest, XCD-remapped; thread = 4 consecutive targets (16-B
// dist accesses: 1 KiB per wave instruction, like the sweeps).  For each
// column c: fm = bits k with w_k + d(dst_k) == d(c), wildcard at the target and
// at unreachable columns; the segment's 32 sets per target are FMB/4 16-B
// stores into the target's row.  Edges come from the packed fixed-stride
// adjacency (SLOTS = 2^shift per column, kNoEdge padding), so a group of G
// columns issues its G own-row and G*SLOTS neighbour gathers back to back,
// with no dependent CSR lookups.

template <int SLOTS, int G, bool NARROW>
__global__ __launch_bounds__(256) void first_moves(const uint2* __restrict__ adj,
                                                   const uint32_t* __restrict__ dist,
                                                   const uint32_t* __restrict__ tgt,
                                                   uint32_t B, uint32_t n, uint32_t npad,
                                                   uint32_t remap, uint32_t* __restrict__ fm,
                                                   const uint32_t* __restrict__ leafbits,
                                                   const uint16_t* __restrict__ fmleaf,
                                                   NarrowRows nr) {
    constexpr int FMB = SLOTS < 4 ? 4 : SLOTS;
    using F = FmFmt<FMB>;
    const uint32_t nseg = npad / kSeg;
    const uint32_t L = remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t slab = L / nseg;
    const uint32_t l4 = slab * blockDim.x + threadIdx.x;  // slab = blockDim.x x 4 targets
    const uint32_t B4 = B / 4u;
    const uint32_t c0 = (L - slab * nseg) * kSeg;
    const uint4 tc = reinterpret_cast<const uint4*>(tgt)[l4];
    const uint4* __restrict__ d4 = reinterpret_cast<const uint4*>(dist);
    const uint32_t grp = wave_group(l4);
    uint32_t pk[4][F::kWords];
#pragma unroll
    for (int p = 0; p < F::kWords; ++p) pk[0][p] = pk[1][p] = pk[2][p] = pk[3][p] = 0xFFFFFFFFu;
    constexpr int KC = SLOTS < 4 ? SLOTS : 4;  // slots gathered per chunk
    // leaf columns (bit set, 4-bit sets only): sets computed by the down-sweep
    const uint32_t lbits = (FMB == 4 && leafbits) ? leafbits[c0 / kSeg] : 0u;
#pragma unroll
    for (int cg = 0; cg < (int)kSeg; cg += G) {
        uint4 dn[G];
        uint2 e[G][SLOTS];  // wave-uniform: scalar registers
        uint32_t b[G][4], lv[G];
        NLoad pn[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint32_t c = c0 + (uint32_t)(cg + j);
            const bool ok = c < n;  // wave-uniform
            const bool leaf = (lbits >> (cg + j)) & 1u;
#pragma unroll
            for (int k = 0; k < SLOTS; ++k)
                e[j][k] = ok && !leaf ? adj[(size_t)c * SLOTS + k] : make_uint2(kNoEdge, 0u);
            if (NARROW) {
                if (ok && !leaf) pn[j] = nl_issue(nr, c, grp, B4, l4);
            } else {
                dn[j] = ok && !leaf ? d4[(size_t)c * B4 + l4] : make_uint4(INF, INF, INF, INF);
            }
            lv[j] = ok && leaf ? fmleaf[(size_t)c * B4 + l4] : 0u;
            b[j][0] = b[j][1] = b[j][2] = b[j][3] = 0;
        }
        // narrow: the own rows are decoded once the first neighbour loads are
        // in flight too
        bool dn_done = !NARROW;
        auto finish_dn = [&] {
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const uint32_t c = c0 + (uint32_t)(cg + j);
                dn[j] = c < n && !((lbits >> (cg + j)) & 1u) ? nl_finish(pn[j], nr, l4)
                                                             : make_uint4(INF, INF, INF, INF);
            }
            dn_done = true;
        };
#pragma unroll
        for (int kb = 0; kb < SLOTS; kb += KC) {
            bool any = false;  // edges are packed first: an empty chunk ends them all
#pragma unroll
            for (int j = 0; j < G; ++j) any |= e[j][kb].x != kNoEdge;
            if (!any) break;
            uint4 dv[G][KC];
            if (NARROW) {
                NLoad pv[G][KC];
#pragma unroll
                for (int j = 0; j < G; ++j)
#pragma unroll
                    for (int k = 0; k < KC; ++k)
                        if (e[j][kb + k].x != kNoEdge)
                            pv[j][k] = nl_issue(nr, e[j][kb + k].x, grp, B4, l4);
                if (!dn_done) finish_dn();
#pragma unroll
                for (int j = 0; j < G; ++j)
#pragma unroll
                    for (int k = 0; k < KC; ++k)
                        if (e[j][kb + k].x != kNoEdge)
                            dv[j][k] = nl_finish(pv[j][k], nr, l4);
            } else {
#pragma unroll
                for (int j = 0; j < G; ++j)
#pragma unroll
                    for (int k = 0; k < KC; ++k)
                        if (e[j][kb + k].x != kNoEdge)
                            dv[j][k] = d4[(size_t)e[j][kb + k].x * B4 + l4];
            }
#pragma unroll
            for (int j = 0; j < G; ++j)
#pragma unroll
                for (int k = 0; k < KC; ++k) {
                    if (e[j][kb + k].x == kNoEdge) continue;
                    const uint32_t we = e[j][kb + k].y;
                    b[j][0] |= fm_bit(dv[j][k].x, we, dn[j].x, kb + k);
                    b[j][1] |= fm_bit(dv[j][k].y, we, dn[j].y, kb + k);
                    b[j][2] |= fm_bit(dv[j][k].z, we, dn[j].z, kb + k);
                    b[j][3] |= fm_bit(dv[j][k].w, we, dn[j].w, kb + k);
                }
        }
        if (!dn_done) finish_dn();
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint32_t c = c0 + (uint32_t)(cg + j);
            if (c >= n) continue;  // stays the wildcard padding
            const int cc = cg + j;
            uint32_t f0, f1, f2, f3;
            if ((lbits >> cc) & 1u) {  // 4 nibbles, wildcards included
                f0 = lv[j] & 0xFu;
                f1 = (lv[j] >> 4) & 0xFu;
                f2 = (lv[j] >> 8) & 0xFu;
                f3 = lv[j] >> 12;
            } else {
                f0 = fm_final<FMB>(c, tc.x, dn[j].x, b[j][0]);
                f1 = fm_final<FMB>(c, tc.y, dn[j].y, b[j][1]);
                f2 = fm_final<FMB>(c, tc.z, dn[j].z, b[j][2]);
                f3 = fm_final<FMB>(c, tc.w, dn[j].w, b[j][3]);
            }
            const int wi = cc / F::kPer, sh = FMB * (cc % F::kPer);
            const uint32_t keep = ~(F::kAll << sh);  // clear this column's field
            pk[0][wi] = (pk[0][wi] & keep) | (f0 << sh);
            pk[1][wi] = (pk[1][wi] & keep) | (f1 << sh);
            pk[2][wi] = (pk[2][wi] & keep) | (f2 << sh);
            pk[3][wi] = (pk[3][wi] & keep) | (f3 << sh);
        }
    }
    if (FMB == 4) {  // row-group interleaved (fm4_piece): one 64-B sector
        uint4* __restrict__ o = reinterpret_cast<uint4*>(fm) + fm4_piece(4u * l4, nseg, c0 / kSeg);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = make_uint4(pk[i][0], pk[i][1], pk[i][2], pk[i][3]);
        return;
    }
    const size_t row_words = npad / F::kPer;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint4* seg = reinterpret_cast<uint4*>(fm + (size_t)(4u * l4 + (uint32_t)i) * row_words +
                                              c0 / F::kPer);
#pragma unroll
        for (int q = 0; q < F::kWords / 4; ++q)
            seg[q] = make_uint4(pk[i][4 * q], pk[i][4 * q + 1], pk[i][4 * q + 2], pk[i][4 * q + 3]);
    }
}

// First-move sets from narrow rows, 4-slot adjacency (out-degree <= 4, 4-bit
// sets): the same sets as first_moves<4, G, true>, with the latency chain
// cut.  The segment's adjacency (32 columns x 4 slots x 8 B = 1 KiB) is ONE
// 16-B load per lane up front — lane L holds slots 2(L&1), 2(L&1)+1 of column
// L/2, read back with readlane — instead of a dependent scalar load per
// column group; and the loads of group g+1 are issued before group g is
// decoded (two groups in flight), so a wave waits about one memory round trip
// per group instead of two.
//
// The column's own row is not read: for c != t, d(c) = min over c's
// out-edges of w_k + d(v_k) (a shortest path to t leaves c by some edge; a
// self loop adds w + d(c) >= d(c) and so never lowers the minimum), all of
// them final here, and d(c) == INF exactly when every term is INF — so the
// sets {k : w_k + d(v_k) == d(c)} follow from the neighbour rows alone,
// bit-identical, one gather per column fewer.  (Reading it, CPD_FM_OWN in
// round 2, was slower and is gone.)
template <int G>
struct FmGroup {  // edges are re-read from the lanes when needed (no SGPR pressure)
    NLoad nb[G][4];  // a leaf column's sets (fmleaf) ride in nb[j][0].q.x
};

// One workgroup per (32-column segment, slab of 4 x blockDim targets).  The
// lane's 4 rows of a segment are one 64-B sector of the row-group interleaved
// layout (fm4_piece), stored whole by the lane: each row's word goes to an
// LDS stage as soon as its 8 columns are done (4 words live instead of 16: 8
// waves per SIMD instead of 6) and the sector is stored from there at the end
// — storing the 4-B words straight to HBM measured 4x the write bytes (34 vs
// 8.8 GB per launch: L2 does not merge them) and 24.4 vs 12.6 ms.  Columns
// are gathered G = 2 at a time, the next group issued before the current one
// is finished (G = 1 measured 16.2 against 15.3 ms; two segments per
// workgroup, CPD_FM_SEGS = 2, 101 VGPRs and slower: both removed in round 3).
// Held to 64 VGPRs for 8 waves per SIMD (round 6: 65 VGPRs had given 7; the
// cap spills 7 rarely-used values to scratch): 22.8-23.0 against 26.6-26.8
// ms beside the up-sweep, 429.9-430.2k against 419.7-420.8k rows/s
// (profiles/fm_packed_ab/r06w_*).
template <int G>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) void first_moves_n4(const uint2* __restrict__ adj,
                                                      const uint32_t* __restrict__ dist,
                                                      const uint32_t* __restrict__ tgt, uint32_t B,
                                                      uint32_t n, uint32_t npad, uint32_t remap,
                                                      uint32_t* __restrict__ fm,
                                                      const uint32_t* __restrict__ leafbits,
                                                      const uint16_t* __restrict__ fmleaf,
                                                      NarrowRows nr,
                                                      const uint32_t* __restrict__ seg_order,
                                                      uint32_t spw) {
    static_assert(kSeg % G == 0, "group size");
    const uint32_t nseg = npad / kSeg, ngrp = nseg / spw;
    const uint32_t L = remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t slab = L / ngrp;
    const uint32_t l4 = slab * blockDim.x + threadIdx.x;  // slab = blockDim.x x 4 targets
    const uint32_t B4 = B / 4u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint4 tc = reinterpret_cast<const uint4*>(tgt)[l4];
    const uint32_t grp = wave_group(l4);
    // each row word is staged in LDS (64 B per lane, dynamic shared memory) as
    // soon as its 8 columns are done, so only the current word of each row is
    // live in registers
    extern __shared__ uint32_t fm_stage[];
    // spw segments one after another (a neighbour row shared by the end of one
    // and the start of the next is read again while it is still in L2),
    // in the order seg_order gives (spatially compact runs), else in column
    // order
    for (uint32_t it = 0; it < spw; ++it) {
    const uint32_t sl = (L - slab * ngrp) * spw + it;
    const uint32_t cb = (seg_order ? seg_order[sl] : sl) * kSeg;
    uint32_t pk[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p) pk[0][p] = pk[1][p] = pk[2][p] = pk[3][p] = 0xFFFFFFFFu;
    // the segment's adjacency (1 KiB) and leaf bits up front; the group
    // pipeline then runs over its 32 columns without a bubble
    const uint32_t lb = leafbits ? leafbits[cb / kSeg] : 0u;
    const uint4 sa = cb + lane / 2u < n ? reinterpret_cast<const uint4*>(adj)[(size_t)cb * 2u + lane]
                                        : make_uint4(kNoEdge, 0u, kNoEdge, 0u);
    auto edge = [&](int cc, int k) -> uint2 {  // wave-uniform; cc in [0, 32)
        const int ln = 2 * cc + (k >> 1);
        const uint32_t x = __builtin_amdgcn_readlane((k & 1) ? sa.z : sa.x, ln);
        const uint32_t w = __builtin_amdgcn_readlane((k & 1) ? sa.w : sa.y, ln);
        return make_uint2(x, w);
    };
    auto is_leaf = [&](int cc) -> bool { return (lb >> cc) & 1u; };
    auto issue = [&](FmGroup<G>& g, int cg) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint32_t c = cb + (uint32_t)(cg + j);
            const bool ok = c < n;
            const bool leaf = is_leaf(cg + j);
            if (ok && !leaf) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint2 e = edge(cg + j, k);
                    if (e.x != kNoEdge) g.nb[j][k] = nl_issue(nr, e.x, grp, B4, l4);
                }
            }
            if (ok && leaf) g.nb[j][0].q.x = fmleaf[(size_t)c * B4 + l4];  // a leaf gathers nothing
        }
    };
    auto finish = [&](const FmGroup<G>& g, int cg) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint32_t c = cb + (uint32_t)(cg + j);
            if (c >= n) continue;  // stays the wildcard padding
            const int cc = cg + j;
            uint32_t bits;
            if (is_leaf(cc)) {  // 4 nibbles, wildcards included
                bits = g.nb[j][0].q.x;
            } else {  // argmin set folded per neighbour (see leaf_finish8)
                uint4 dn = make_uint4(INF, INF, INF, INF);
                bits = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint2 e = edge(cc, k);
                    if (e.x == kNoEdge) continue;
                    const uint4 dv = nl_finish(g.nb[j][k], nr, l4);
                    argmin_fold<0>(dn.x, bits, sat_add(dv.x, e.y), k);
                    argmin_fold<1>(dn.y, bits, sat_add(dv.y, e.y), k);
                    argmin_fold<2>(dn.z, bits, sat_add(dv.z, e.y), k);
                    argmin_fold<3>(dn.w, bits, sat_add(dv.w, e.y), k);
                }
                bits = fm_wild4(tc, dn, c, bits);
            }
            const uint32_t f0 = bits & 0xFu, f1 = (bits >> 4) & 0xFu;
            const uint32_t f2 = (bits >> 8) & 0xFu, f3 = (bits >> 12) & 0xFu;
            const int wi = cc / 8, sh = 4 * (cc % 8);
            const uint32_t keep = ~(0xFu << sh);
            pk[0][wi] = (pk[0][wi] & keep) | (f0 << sh);
            pk[1][wi] = (pk[1][wi] & keep) | (f1 << sh);
            pk[2][wi] = (pk[2][wi] & keep) | (f2 << sh);
            pk[3][wi] = (pk[3][wi] & keep) | (f3 << sh);
        }
    };
    constexpr int NC = (int)kSeg;
    static_assert(8 % G == 0, "a group never straddles a word");
    FmGroup<G> cur, nxt;
    issue(cur, 0);
#pragma unroll
    for (int cg = 0; cg < NC; cg += G) {
        if (cg + G < NC) issue(nxt, cg + G);
        finish(cur, cg);
        if ((cg + G) % 8 == 0) {  // the 4 rows' words of these 8 columns -> LDS
            const int wi = (cg + G) / 8 - 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) fm_stage[(threadIdx.x * 4u + (uint32_t)i) * 4u + wi] = pk[i][wi];
        }
        cur = nxt;
    }
    // the lane's own staged sector: whole 64-B stores (no barrier: same lane)
    uint4* __restrict__ o = reinterpret_cast<uint4*>(fm) + fm4_piece(4u * l4, nseg, cb / kSeg);
    const uint4* st = reinterpret_cast<const uint4*>(fm_stage) + threadIdx.x * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = st[i];
    }
}

// One lane's greedy pass over its 32 columns (warthog graph_oracle::add_row
// [U]: keep S = AND of the current run's first-move sets; a column that would
// empty S ends the run — word (head << 4 | lowest bit of S) — and starts a new
// one at that column).  v holds the segment's 32 FMB-bit sets, 32/FMB per word.
template <int FMB>
__device__ __forceinline__ void seg_pass(const uint32_t (&v)[FmFmt<FMB>::kWords], uint32_t c0,
                                         uint32_t& h, uint32_t& S, uint32_t& cnt) {
    using F = FmFmt<FMB>;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t f = (v[k / F::kPer] >> (FMB * (k % F::kPer))) & F::kAll;
        const bool brk = (S & f) == 0u;
        cnt += brk ? 1u : 0u;
        h = brk ? c0 + (uint32_t)k : h;
        S = brk ? f : (S & f);
    }
}

template <int FMB>
__device__ __forceinline__ uint32_t set_at(const uint32_t (&v)[FmFmt<FMB>::kWords], int k) {
    using F = FmFmt<FMB>;
    return (v[k / F::kPer] >> (FMB * (k % F::kPer))) & F::kAll;
}

// Per-(row, 32-column segment) RLE entry states, written by the count pass
// and read by the move-table emit (rle_moves), which needs no speculation of
// its own:
//   st[row * nseg + seg] = state of the greedy scan entering the segment:
//                          head << 4 | S for 4-bit sets (rle_fix compares
//                          whole states), S alone for wider ones,
//   rc[row * nseg + seg] = runs that end inside the segment (<= 32) = the
//                          columns of the segment where a new run starts.
struct RleState {
    uint32_t* st;
    uint8_t* rc;
};

// Greedy RLE count, one row per wave, 2048-column tiles (lane l owns columns
// 32l..32l+31 of the tile).  The scan is sequential by definition, so each
// lane guesses the state entering its segment — the predecessor lane's last
// 16 columns scanned from a fresh run: the greedy state forgets its past
// within a few runs, so the guess is usually exact — runs its segment from
// the guess, then re-runs from its predecessor's end state until no lane's
// input changes (exact for any input: at most 64 rounds).  counts[row] =
// runs in the row; the segment entry states and counts go to rs.  (The
// chunked count rle_count_ch + rle_fix replaces this for 4-bit sets; this
// pass serves wider sets and rows whose long runs the seam repair gives up
// on.)
// gate (may be null): run only if *gate != 0 — the re-count of a batch
// whose seam repair gave up, queued unconditionally after rle_fix.
template <int FMB>
__global__ __launch_bounds__(256) void rle_scan(const uint32_t* __restrict__ fm, uint32_t npad,
                                                uint32_t nrows, uint32_t* __restrict__ counts,
                                                RleState rs, const uint32_t* __restrict__ gate) {
    using F = FmFmt<FMB>;
    constexpr int Q = F::kWords / 4;  // 16-B loads per lane per tile
    constexpr int LB = CPD_RLE_LOOKBACK;  // lookback columns
    const uint32_t row = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (row >= nrows) return;
    if (gate && *gate == 0u) return;
    const uint32_t nseg = npad / kSeg;
    // this lane's 16-B pieces of the row: 4-bit rows are row-group interleaved
    // (fm4_piece), wider ones row-major; tile t is `step` pieces further on
    const uint4* __restrict__ src =
        FMB == 4 ? reinterpret_cast<const uint4*>(fm) + fm4_piece(row, nseg, lane)
                 : reinterpret_cast<const uint4*>(fm + (size_t)row * (npad / F::kPer)) + lane * Q;
    const size_t step = FMB == 4 ? 64u * 4u : 64u * Q;
    const bool keep = rs.st != nullptr;
    const bool track_h = keep && FMB == 4;  // heads matter only in packed 4-bit states
    uint32_t carry_h = 0, carry_S = F::kAll, total = 0;
    const uint32_t ntiles = npad / kTile;
    const size_t sbase = (size_t)row * nseg + lane;
    uint4 nx[Q];  // tile t's segment of this lane, prefetched one tile ahead
#pragma unroll
    for (int q = 0; q < Q; ++q) nx[q] = src[q];
    for (uint32_t t = 0; t < ntiles; ++t) {
        uint32_t v[F::kWords];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            v[4 * q] = nx[q].x;
            v[4 * q + 1] = nx[q].y;
            v[4 * q + 2] = nx[q].z;
            v[4 * q + 3] = nx[q].w;
        }
        if (t + 1 < ntiles) {
#pragma unroll
            for (int q = 0; q < Q; ++q) nx[q] = src[(size_t)(t + 1) * step + q];
        }
        const uint32_t c0 = t * kTile + lane * kSeg;
        // guess: the predecessor's last LB columns from a fresh run
        constexpr int PW = LB / F::kPer;  // words holding those columns
        static_assert(LB % F::kPer == 0 && PW <= F::kWords, "lookback: whole words");
        uint32_t pv[PW];
#pragma unroll
        for (int i = 0; i < PW; ++i) pv[i] = __shfl_up(v[F::kWords - PW + i], 1, 64);
        uint32_t gh = c0 - LB, gS = F::kAll;
#pragma unroll
        for (int k = 0; k < LB; ++k) {
            const uint32_t f = (pv[k / F::kPer] >> (FMB * (k % F::kPer))) & F::kAll;
            const bool brk = (gS & f) == 0u;
            gh = brk ? c0 - LB + (uint32_t)k : gh;
            gS = brk ? f : (gS & f);
        }
        uint32_t in_h = lane == 0 ? carry_h : gh;
        uint32_t in_S = lane == 0 ? carry_S : gS;
        uint32_t eh = in_h, eS = in_S, cnt = 0;
        seg_pass<FMB>(v, c0, eh, eS, cnt);
        for (int round = 0; round < 64; ++round) {
            uint32_t nh = __shfl_up(eh, 1, 64), nS = __shfl_up(eS, 1, 64);
            if (lane == 0) {
                nh = carry_h;
                nS = carry_S;
            }
            const bool need = nS != in_S || (track_h && nh != in_h);
            if (!__any(need)) break;
            if (need) {
                in_h = nh;
                in_S = nS;
                eh = nh;
                eS = nS;
                cnt = 0;
                seg_pass<FMB>(v, c0, eh, eS, cnt);
            }
        }
        if (keep) {  // coalesced: 64 lanes x 4 B + 64 x 1 B per tile
            rs.st[sbase + (size_t)t * 64u] = FMB == 4 ? (in_h << 4) | in_S : in_S;
            rs.rc[sbase + (size_t)t * 64u] = (uint8_t)cnt;
        }
        uint32_t sum = cnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
        total += sum;
        carry_h = __shfl(eh, 63, 64);
        carry_S = __shfl(eS, 63, 64);
    }
    if (lane == 0) counts[row] = total + 1;  // + the final run
}

// ---------------------------------------------------------------------------
// Compact rows: the greedy RLE row as a 4-bit move table.
//
// Every column of a run gets the run's move (lowest set bit of the AND of the
// run's sets, taken where the run closes), and consecutive runs always carry
// different moves: a run closes at column c only when S & FM(c) == 0, its move
// lies in S and the next run's in FM(c).  So the table is the RLE row
// expanded — n/2 bytes per row against 4 B per run (R ~ 0.62 n on the bench
// graphs: 5x smaller) — and the runs come back exactly as
// {0} U {c : move(c) != move(c - 1)} (moves_runs below).  Column c of a row
// is nibble c % 8 of word c / 8: the dense table the walks read, so an index
// takes the rows as they are.
//
// A column's move depends on where its run CLOSES, to its right; the scan
// state depends on the columns to its left, which the count pass has already
// resolved (st: every segment's entry state).  So a wave takes kMoveTiles
// consecutive 2048-column tiles of one row and walks them right to left,
// carrying the move of the run still open at the right edge:
//   forward (per lane, 32 columns from the segment's entry set): the break
//     mask and L_k = lowest bit of the running set after column k; the run
//     entering the segment closes at its first break b, with move F = L_{b-1}
//     (the entry set's lowest bit when b = 0);
//   resolve (per wave): a lane's open tail run closes in the first lane to
//     its right that has a break (that lane's F), else right of the tile
//     (the carry);
//   backward (per lane): column k takes the move of the run holding it.
// The carry entering the chunk comes from a look-ahead to the first segment
// right of it whose count rc is non-zero (one uniform segment scan); when no
// run closes right of the chunk, the open run is the row's last, and its move
// is the lowest bit of the set at the row's end.  One 16-B store per lane per
// tile: a wave writes 1 KiB contiguous.
constexpr uint32_t kMoveTiles = 16;
// tiles per chunk of the fused emit: one wave of rle_emit8 (64 lanes x
// kE8Cols columns of eight rows); rle_emit_fix redoes a chunk with
// emit_chunk4 (4 * kEmitTiles VGPRs of sets)
// columns per lane of rle_emit8 (32 or 64, build time): 32 measured
// 431.5-433.3k against 428.3-431.7k rows/s for 64 (the emit 7.6 against 9.7
// ms beside the down-sweep: 8 instead of 16 KiB of LDS per wave, 81 instead
// of 113 VGPRs; profiles/emit8_cols_ab/)
#ifndef CPD_E8_COLS
#define CPD_E8_COLS 32
#endif
constexpr uint32_t kE8Cols = CPD_E8_COLS;
static_assert(kE8Cols == 32 || kE8Cols == 64, "rle_emit8 lane width");
constexpr uint32_t kEmitTiles = kE8Cols / 32u;

// Move tables at 2^lb bits per column (lb = 0, 1, 2: 1, 2 or 4 bits, by the
// graph's max out-degree — a move indexes its column's out-list, so every
// valid move fits), column c in bits [b·c, b·c + b) of its row, npad·b/32
// words per row.  The emit computes 32 columns per lane as four nibble words
// and narrows them on the store; readers of whole 32-column groups widen
// them back; the walks read one column's field.
struct Tbl {
    uint32_t lb;
    __device__ __forceinline__ uint32_t move(const uint32_t* __restrict__ row, uint32_t c) const {
        return (row[c >> (5u - lb)] >> ((c & (31u >> lb)) << lb)) & ((1u << (1u << lb)) - 1u);
    }
};

// 8 nibbles (each < 4) -> 16 bits of 2-bit fields; (each < 2) -> 8 bits
__device__ __forceinline__ uint32_t nib_to2(uint32_t x) {
    x &= 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    return (x | (x >> 8)) & 0x0000FFFFu;
}
__device__ __forceinline__ uint32_t nib_to1(uint32_t x) {
    x &= 0x11111111u;
    x = (x | (x >> 3)) & 0x03030303u;
    x = (x | (x >> 6)) & 0x000F000Fu;
    return (x | (x >> 12)) & 0x000000FFu;
}
__device__ __forceinline__ uint32_t nib_from2(uint32_t y) {  // 16 bits -> 8 nibbles
    y &= 0xFFFFu;
    y = (y | (y << 8)) & 0x00FF00FFu;
    y = (y | (y << 4)) & 0x0F0F0F0Fu;
    return (y | (y << 2)) & 0x33333333u;
}
__device__ __forceinline__ uint32_t nib_from1(uint32_t y) {  // 8 bits -> 8 nibbles
    y &= 0xFFu;
    y = (y | (y << 12)) & 0x000F000Fu;
    y = (y | (y << 6)) & 0x03030303u;
    return (y | (y << 3)) & 0x11111111u;
}

// Columns [32 g, 32 g + 32) of a table row, as four nibble words o[0..3]
// (column 32 g + k in nibble k % 8 of o[k / 8]): one 16-, 8- or 4-B access.
__device__ __forceinline__ void store_cols32(uint32_t* __restrict__ row, uint32_t g, uint32_t lb,
                                             const uint32_t (&o)[4]) {
    if (lb == 2u) {
        reinterpret_cast<uint4*>(row)[g] = make_uint4(o[0], o[1], o[2], o[3]);
    } else if (lb == 1u) {
        reinterpret_cast<uint2*>(row)[g] =
            make_uint2(nib_to2(o[0]) | (nib_to2(o[1]) << 16), nib_to2(o[2]) | (nib_to2(o[3]) << 16));
    } else {
        row[g] = nib_to1(o[0]) | (nib_to1(o[1]) << 8) | (nib_to1(o[2]) << 16) | (nib_to1(o[3]) << 24);
    }
}

// store_cols32 by a whole wave whose lane l holds segment g0 + l: the packed
// widths' 8-B (2-bit) and 4-B (1-bit) pieces gathered into 16-B stores by
// every second / fourth lane (per-lane 8-B / 4-B stores measured 378.7k
// against 380.7k rows/s and were removed in round 6)
__device__ __forceinline__ void store_cols32_wave(uint32_t* __restrict__ row, uint32_t g,
                                                  uint32_t lb, const uint32_t (&o)[4],
                                                  uint32_t lane) {
    if (lb == 2u) {
        store_cols32(row, g, lb, o);
    } else if (lb == 1u) {
        const uint32_t a = nib_to2(o[0]) | (nib_to2(o[1]) << 16);
        const uint32_t b = nib_to2(o[2]) | (nib_to2(o[3]) << 16);
        const uint32_t na = (uint32_t)__shfl_down((int)a, 1, 64);
        const uint32_t nb = (uint32_t)__shfl_down((int)b, 1, 64);
        if (!(lane & 1u)) reinterpret_cast<uint4*>(row)[g >> 1] = make_uint4(a, b, na, nb);
    } else {
        const uint32_t w = nib_to1(o[0]) | (nib_to1(o[1]) << 8) | (nib_to1(o[2]) << 16) |
                           (nib_to1(o[3]) << 24);
        const uint32_t w1 = (uint32_t)__shfl_down((int)w, 1, 64);
        const uint32_t w2 = (uint32_t)__shfl_down((int)w, 2, 64);
        const uint32_t w3 = (uint32_t)__shfl_down((int)w, 3, 64);
        if (!(lane & 3u)) reinterpret_cast<uint4*>(row)[g >> 2] = make_uint4(w, w1, w2, w3);
    }
}
__device__ __forceinline__ void load_cols32(const uint32_t* __restrict__ row, uint32_t g, uint32_t lb,
                                            uint32_t (&x)[4]) {
    if (lb == 2u) {
        const uint4 q = reinterpret_cast<const uint4*>(row)[g];
        x[0] = q.x;
        x[1] = q.y;
        x[2] = q.z;
        x[3] = q.w;
    } else if (lb == 1u) {
        const uint2 q = reinterpret_cast<const uint2*>(row)[g];
        x[0] = nib_from2(q.x);
        x[1] = nib_from2(q.x >> 16);
        x[2] = nib_from2(q.y);
        x[3] = nib_from2(q.y >> 16);
    } else {
        const uint32_t q = row[g];
        x[0] = nib_from1(q);
        x[1] = nib_from1(q >> 8);
        x[2] = nib_from1(q >> 16);
        x[3] = nib_from1(q >> 24);
    }
}

__device__ __forceinline__ uint32_t low_bit(uint32_t S) {
    return (uint32_t)__builtin_ctz(S | 0x8000u);  // S != 0: every set is non-empty
}

// nibble i (runtime index) of a 32-nibble value held in 4 words
__device__ __forceinline__ uint32_t nib_at(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                           uint32_t i) {
    const uint32_t x = i < 16u ? (i < 8u ? w0 : w1) : (i < 24u ? w2 : w3);
    return (x >> (4u * (i & 7u))) & 0xFu;
}

struct SegMoves {
    uint32_t brk;   // bit k: a new run starts at column k
    uint32_t L[4];  // nibble k: lowest set bit of the running set after column k
    uint32_t S;     // the running set after column 31
};

template <int FMB>
__device__ __forceinline__ SegMoves seg_moves(const uint32_t (&v)[FmFmt<FMB>::kWords],
                                              uint32_t S) {
    SegMoves r;
    r.brk = 0;
    r.L[0] = r.L[1] = r.L[2] = r.L[3] = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t f = set_at<FMB>(v, k);
        const uint32_t T = S & f;
        const bool b = T == 0u;
        r.brk |= (b ? 1u : 0u) << k;
        S = b ? f : T;
        r.L[k >> 3] |= low_bit(S) << (4 * (k & 7));
    }
    r.S = S;
    return r;
}

// move of the run entering the segment (it closes at the first break)
__device__ __forceinline__ uint32_t seg_entry_move(const SegMoves& r, uint32_t Sin) {
    const uint32_t b0 = (uint32_t)__builtin_ctz(r.brk | 0x80000000u);
    return b0 == 0u ? low_bit(Sin) : nib_at(r.L[0], r.L[1], r.L[2], r.L[3], b0 - 1u);
}

template <int FMB>
__device__ __forceinline__ void load_seg(const uint32_t* __restrict__ fm, uint32_t npad,
                                         uint32_t row, uint32_t seg,
                                         uint32_t (&v)[FmFmt<FMB>::kWords]) {
    using F = FmFmt<FMB>;
    const uint32_t nseg = npad / kSeg;
    if (FMB == 4) {
        const uint4 q = reinterpret_cast<const uint4*>(fm)[fm4_piece(row, nseg, seg)];
        v[0] = q.x;
        v[1] = q.y;
        v[2] = q.z;
        v[3] = q.w;
    } else {
        constexpr int Q = F::kWords / 4;
        const uint4* s =
            reinterpret_cast<const uint4*>(fm + (size_t)row * (npad / F::kPer)) + (size_t)seg * Q;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint4 x = s[q];
            v[4 * q] = x.x;
            v[4 * q + 1] = x.y;
            v[4 * q + 2] = x.z;
            v[4 * q + 3] = x.w;
        }
    }
}

// Batch row `brow` (fm / st / rc row) goes to table row out_row[brow].
template <int FMB>
__global__ __launch_bounds__(256) void rle_moves(const uint32_t* __restrict__ fm, uint32_t npad,
                                                 uint32_t nrows, const uint32_t* __restrict__ st,
                                                 const uint8_t* __restrict__ rc,
                                                 const uint32_t* __restrict__ out_row,
                                                 uint32_t lb, uint32_t* __restrict__ dense) {
    using F = FmFmt<FMB>;
    const uint32_t brow = blockIdx.y * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (brow >= nrows) return;  // wave-uniform
    const uint32_t nseg = npad / kSeg, ntiles = npad / kTile;
    const uint32_t t0 = blockIdx.x * kMoveTiles;
    if (t0 >= ntiles) return;
    const uint32_t t1 = min(ntiles, t0 + kMoveTiles);
    constexpr uint32_t smask = FMB == 4 ? 0xFu : F::kAll;  // 4-bit states carry the head
    const uint32_t* __restrict__ strow = st + (size_t)brow * nseg;
    const uint8_t* __restrict__ rcrow = rc + (size_t)brow * nseg;
    // carry: the move of the run open at the right edge of the tile in hand
    uint32_t carry = 0;
    bool have = false;  // wave-uniform
    for (uint32_t s0 = t1 * 64u; s0 < nseg && !have; s0 += 64u) {
        const uint64_t m = __ballot(s0 + lane < nseg && rcrow[s0 + lane] != 0);
        if (m) {
            const uint32_t sj = s0 + (uint32_t)__builtin_ctzll(m);
            uint32_t v[F::kWords];
            load_seg<FMB>(fm, npad, brow, sj, v);
            const uint32_t Sin = strow[sj] & smask;
            carry = seg_entry_move(seg_moves<FMB>(v, Sin), Sin);
            have = true;
        }
    }
    if (!have) {  // no run closes right of the chunk: the row's final run
        uint32_t v[F::kWords];
        load_seg<FMB>(fm, npad, brow, nseg - 1u, v);
        carry = low_bit(seg_moves<FMB>(v, strow[nseg - 1u] & smask).S);
    }
    uint32_t* __restrict__ orow = dense + (size_t)out_row[brow] * (npad >> (5u - lb));
    for (uint32_t t = t1; t-- > t0;) {
        const uint32_t seg = t * 64u + lane;
        uint32_t v[F::kWords];
        load_seg<FMB>(fm, npad, brow, seg, v);
        const uint32_t Sin = strow[seg] & smask;
        const SegMoves r = seg_moves<FMB>(v, Sin);
        const uint32_t fl = seg_entry_move(r, Sin);
        const uint64_t m = __ballot(r.brk != 0u);
        const uint64_t right = lane == 63u ? 0ull : (m >> (lane + 1u)) << (lane + 1u);
        const uint32_t j = right ? (uint32_t)__builtin_ctzll(right) : lane;
        const uint32_t fj = (uint32_t)__shfl((int)fl, (int)j, 64);
        uint32_t mv = right ? fj : carry;
        uint32_t o[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 31; k >= 0; --k) {
            o[k >> 3] |= mv << (4 * (k & 7));
            if (k > 0 && ((r.brk >> k) & 1u)) mv = (r.L[(k - 1) >> 3] >> (4 * ((k - 1) & 7))) & 0xFu;
        }
        store_cols32(orow, t * 64u + lane, lb, o);
        if (m) carry = (uint32_t)__shfl((int)fl, (int)__builtin_ctzll(m), 64);
    }
}

// rle_moves for 4-bit sets on the packed nibbles (the per-column kernel
// above serves 8- and 16-bit sets; identical tables).  Per lane:
//   forward: only the running sets S_k (one nibble insert per column);
//   breaks:  a run starts at column k iff S_{k-1} & f_k == 0 — the running
//            sets shifted up a nibble (the entry set at nibble 0) AND the
//            segment's sets, zero nibbles found with the carry trick; the
//            shifted sets also hold, at each break, the closing set of the
//            run it ends;
//   fill:    every column takes its run's closing set: run ends (a break at
//            k + 1; column 31 with the tail run's set) keep theirs, the rest
//            copy from the right in five doubling steps;
//   moves:   the lowest set bit of every nibble at once.
// The carry and the lanes' entry values are closing SETS here, not moves.
struct Seg4 {
    uint32_t S[4];  // nibble k: running set after column k
    uint32_t P[4];  // nibble k: running set before column k (the entry set at 0)
    uint32_t Z[4];  // bit 3 of nibble k: a run starts at column k
};

__device__ __forceinline__ Seg4 seg4_scan(const uint32_t (&v)[4], uint32_t Sin) {
    Seg4 r;
    r.S[0] = r.S[1] = r.S[2] = r.S[3] = 0u;
    uint32_t S = Sin;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t f = (v[k >> 3] >> (4 * (k & 7))) & 0xFu;
        const uint32_t T = S & f;
        S = T ? T : f;
        r.S[k >> 3] |= S << (4 * (k & 7));
    }
    r.P[0] = (r.S[0] << 4) | Sin;
    r.P[1] = __builtin_amdgcn_alignbit(r.S[1], r.S[0], 28);
    r.P[2] = __builtin_amdgcn_alignbit(r.S[2], r.S[1], 28);
    r.P[3] = __builtin_amdgcn_alignbit(r.S[3], r.S[2], 28);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t a = r.P[i] & v[i];
        r.Z[i] = ~(((a & 0x77777777u) + 0x77777777u) | a) & 0x88888888u;
    }
    return r;
}

// closing set of the run entering the segment (it closes at the first break);
// only meaningful when the segment has a break
__device__ __forceinline__ uint32_t seg4_entry_set(const Seg4& r) {
    const uint32_t b0 = r.Z[0] ? ((uint32_t)__builtin_ctz(r.Z[0]) >> 2)
                      : r.Z[1] ? 8u + ((uint32_t)__builtin_ctz(r.Z[1]) >> 2)
                      : r.Z[2] ? 16u + ((uint32_t)__builtin_ctz(r.Z[2]) >> 2)
                               : 24u + ((uint32_t)__builtin_ctz(r.Z[3] | 0x80000000u) >> 2);
    return nib_at(r.P[0], r.P[1], r.P[2], r.P[3], b0);
}

// One tile's move table from its segments' scans (lane = segment), right to
// left: `carry` is the closing set of the run open at the tile's right edge
// on entry, at its left edge on exit.  Each column takes the set of the run
// it belongs to, the move = that set's lowest bit.
__device__ __forceinline__ void fill_tile4(const Seg4& r, uint32_t& carry,
                                           uint32_t* __restrict__ orow, uint32_t seg,
                                           uint32_t lb, uint32_t lane) {
    const bool any = (r.Z[0] | r.Z[1] | r.Z[2] | r.Z[3]) != 0u;
    const uint32_t fl = seg4_entry_set(r);
    const uint64_t m = __ballot(any);
    const uint64_t right = lane == 63u ? 0ull : (m >> (lane + 1u)) << (lane + 1u);
    const uint32_t j = right ? (uint32_t)__builtin_ctzll(right) : lane;
    const uint32_t fj = (uint32_t)__shfl((int)fl, (int)j, 64);
    const uint32_t tail = right ? fj : carry;
    // run ends: a break at the next column (nibble mask, shifted down one
    // nibble), and column 31 carrying the tail run's set
    uint32_t V[4], X[4];
    {
        uint32_t nz[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) nz[i] = r.Z[i] | (r.Z[i] - (r.Z[i] >> 3));
        V[0] = __builtin_amdgcn_alignbit(nz[1], nz[0], 4);
        V[1] = __builtin_amdgcn_alignbit(nz[2], nz[1], 4);
        V[2] = __builtin_amdgcn_alignbit(nz[3], nz[2], 4);
        V[3] = (nz[3] >> 4) | 0xF0000000u;
        X[0] = r.S[0];
        X[1] = r.S[1];
        X[2] = r.S[2];
        X[3] = (r.S[3] & 0x0FFFFFFFu) | (tail << 28);
    }
    // every other column copies the nearest run end to its right
#pragma unroll
    for (int sh = 4; sh <= 16; sh <<= 1) {
        uint32_t xs[4], vs[4];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            xs[i] = __builtin_amdgcn_alignbit(X[i + 1], X[i], sh);
            vs[i] = __builtin_amdgcn_alignbit(V[i + 1], V[i], sh);
        }
        xs[3] = X[3] >> sh;
        vs[3] = V[3] >> sh;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            X[i] = (V[i] & X[i]) | (~V[i] & xs[i]);
            V[i] |= vs[i];
        }
    }
#pragma unroll
    for (int w = 1; w <= 2; w <<= 1) {  // 32- and 64-bit steps: whole words
        uint32_t xs[4], vs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            xs[i] = i + w < 4 ? X[i + w] : 0u;
            vs[i] = i + w < 4 ? V[i + w] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            X[i] = (V[i] & X[i]) | (~V[i] & xs[i]);
            V[i] |= vs[i];
        }
    }
    // lowest set bit of every (non-empty) nibble
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t b0 = ~X[i] & 0x11111111u;
        const uint32_t b1 = ~(X[i] >> 1) & b0;
        const uint32_t b2 = ~(X[i] >> 2) & b1;
        o[i] = b0 + b1 + b2;
    }
    store_cols32_wave(orow, seg, lb, o, lane);
    if (m) carry = (uint32_t)__shfl((int)fl, (int)__builtin_ctzll(m), 64);
}

__global__ __launch_bounds__(256) void rle_moves4(const uint32_t* __restrict__ fm, uint32_t npad,
                                                  uint32_t nrows, const uint32_t* __restrict__ st,
                                                  const uint8_t* __restrict__ rc,
                                                  const uint32_t* __restrict__ out_row,
                                                  uint32_t lb, uint32_t* __restrict__ dense) {
    const uint32_t brow = blockIdx.y * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (brow >= nrows) return;  // wave-uniform
    const uint32_t nseg = npad / kSeg, ntiles = npad / kTile;
    const uint32_t t0 = blockIdx.x * kMoveTiles;
    if (t0 >= ntiles) return;
    const uint32_t t1 = min(ntiles, t0 + kMoveTiles);
    const uint32_t* __restrict__ strow = st + (size_t)brow * nseg;
    const uint8_t* __restrict__ rcrow = rc + (size_t)brow * nseg;
    const uint4* __restrict__ f4 = reinterpret_cast<const uint4*>(fm);
    auto load = [&](uint32_t seg, uint32_t (&v)[4]) {
        const uint4 q = f4[fm4_piece(brow, nseg, seg)];
        v[0] = q.x;
        v[1] = q.y;
        v[2] = q.z;
        v[3] = q.w;
    };
    // carry: the closing set of the run open at the right edge of the tile
    uint32_t carry = 0;
    bool have = false;  // wave-uniform
    for (uint32_t s0 = t1 * 64u; s0 < nseg && !have; s0 += 64u) {
        const uint64_t m = __ballot(s0 + lane < nseg && rcrow[s0 + lane] != 0);
        if (m) {
            const uint32_t sj = s0 + (uint32_t)__builtin_ctzll(m);
            uint32_t v[4];
            load(sj, v);
            carry = seg4_entry_set(seg4_scan(v, strow[sj] & 0xFu));
            have = true;
        }
    }
    if (!have) {  // no run closes right of the chunk: the row's final run
        uint32_t v[4];
        load(nseg - 1u, v);
        carry = seg4_scan(v, strow[nseg - 1u] & 0xFu).S[3] >> 28;
    }
    uint32_t* __restrict__ orow = dense + (size_t)out_row[brow] * (npad >> (5u - lb));
    for (uint32_t t = t1; t-- > t0;) {
        const uint32_t seg = t * 64u + lane;
        uint32_t v[4];
        load(seg, v);
        fill_tile4(seg4_scan(v, strow[seg] & 0xFu), carry, orow, seg, lb, lane);
    }
}

// ---------------------------------------------------------------------------
// One pass per row chunk: count + emit fused (4-bit sets).
// rle_count_ch + rle_fix + rle_moves4 read every first-move set twice (the
// count, then the emit) and write and re-read the per-segment entry states:
// ~50 GB of HBM per 24576-row step for 12.3 GB of sets and 12.3 GB of
// tables.  Here a wave owns a chunk of kEmitTiles tiles of one row (round 6:
// the bulk of the emit is rle_emit8 below, eight rows per wave; this one-row
// form, emit_chunk4, remains rle_emit_fix's redo of a chunk) and:
//   forward  resolves every segment's entry set itself: lane L guesses its
//            entry by scanning lane L-1's last 16 columns from a wildcard
//            set, scans its 32 columns, and takes lane L-1's exit instead
//            wherever the guess differs — repeated until no lane changes (a
//            fixed point reached left to right: one round as a rule); lane
//            0 starts from the previous tile's exit.  The entry sets go to
//            LDS (a byte per segment), the breaks are counted on the way;
//   ahead    finds the closing set of the run open at the chunk's right
//            edge: before the first break the running set is the exit set
//            ANDed with every set passed, so a wave-wide prefix-AND of the
//            segments' own ANDs finds the segment holding the break, which
//            one lane scans (the row's last run: its set at the end);
//   backward fills the move table right to left as rle_moves4 does, the
//            entry sets from LDS and the look-ahead's closing set as carry;
// so each set is read once from HBM (the backward pass re-reads the chunk's
// 64 KiB per 4-row workgroup from L2) and only the tables are written.  The
// chunk's own entry is a guess too (its first segment scanned from its left
// neighbour's last 16 columns; exact for chunk 0): rle_emit_fix then walks
// each row's chunks, and a chunk whose guess differs from its left
// neighbour's exit is done again from the true entry by the same code —
// only that chunk: its left neighbour's look-ahead started from its own
// exact exit set.  Per chunk: the guessed entry, the exit set and the breaks
// (xe, xs, cc, [nrows][nch] u32); the row's runs = its breaks + 1.
struct EmitChunks {
    uint32_t* xe;
    uint32_t* xs;
    uint32_t* cc;
};

// the greedy running set after 32 columns from S, and the breaks among them
__device__ __forceinline__ uint32_t scan32_breaks(const uint32_t (&v)[4], uint32_t& S) {
    uint32_t brk = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t f = (v[k >> 3] >> (4 * (k & 7))) & 0xFu;
        const uint32_t T = S & f;
        brk += T == 0u ? 1u : 0u;
        S = T ? T : f;
    }
    return brk;
}

// The chunk [t0, t1) of row `brow` from entry set Sin (wave-cooperative; every
// lane of the wave calls it with the same arguments).  ent: 64 * kEmitTiles
// bytes of LDS for this wave.  Writes the chunk's move table; returns the
// exit set (wave-uniform) and adds the chunk's breaks to `breaks` (per lane).
// The chunk's sets stay in registers (4 * kEmitTiles VGPRs a lane), loaded
// all at once up front (round 5, at 16-tile chunks: the wave's whole 16 KiB
// in flight instead of one tile per dependent scan), and the backward pass
// reads nothing again.
__device__ uint32_t emit_chunk4(const uint4* __restrict__ f4, uint32_t brow, uint32_t nseg,
                                uint32_t ntiles, uint32_t t0, uint32_t t1, uint32_t Sin,
                                uint8_t* ent, uint32_t* __restrict__ orow, uint32_t lb,
                                uint32_t lane, uint32_t& breaks) {
    auto load = [&](uint32_t seg, uint32_t (&v)[4]) {
        const uint4 q = f4[fm4_piece(brow, nseg, seg)];
        v[0] = q.x;
        v[1] = q.y;
        v[2] = q.z;
        v[3] = q.w;
    };
    const uint32_t L = t1 - t0;  // tiles in the chunk, 1..kEmitTiles (wave-uniform)
    uint32_t C[kEmitTiles][4];
#pragma unroll
    for (uint32_t i = 0; i < kEmitTiles; ++i)
        if (i < L) load((t0 + i) * 64u + lane, C[i]);
    // forward: the segments' entry sets
    uint32_t carry = Sin;  // the set entering the tile in hand
#pragma unroll
    for (uint32_t i = 0; i < kEmitTiles; ++i) {
        if (i < L) {
        const uint32_t(&v)[4] = C[i];
        const uint32_t p2 = (uint32_t)__shfl_up((int)v[2], 1, 64);
        const uint32_t p3 = (uint32_t)__shfl_up((int)v[3], 1, 64);
        uint32_t in = 0xFu;  // the guess: lane - 1's last 16 columns from a wildcard
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t f = ((k < 8 ? p2 : p3) >> (4 * (k & 7))) & 0xFu;
            const uint32_t T = in & f;
            in = T ? T : f;
        }
        if (lane == 0) in = carry;
        uint32_t out, nb;
        for (;;) {
            out = in;
            nb = scan32_breaks(v, out);
            uint32_t pe = (uint32_t)__shfl_up((int)out, 1, 64);
            if (lane == 0) pe = carry;
            const bool fix = pe != in;
            if (!__any(fix)) break;
            if (fix) in = pe;
        }
        ent[i * 64u + lane] = (uint8_t)in;
        breaks += nb;
        carry = (uint32_t)__shfl((int)out, 63, 64);
        }
    }
    const uint32_t exitS = carry;
    // ahead: the closing set of the run open at the right edge
    uint32_t close = 0;
    {
        uint32_t P = exitS;
        bool found = false;  // wave-uniform
        for (uint32_t t = t1; t < ntiles && !found; ++t) {
            uint32_t v[4];
            load(t * 64u + lane, v);
            uint32_t a = v[0] & v[1] & v[2] & v[3];
            a &= a >> 16;
            a &= a >> 8;
            a &= a >> 4;
            const uint32_t A = a & 0xFu;
            uint32_t incl = A;  // inclusive prefix-AND over the lanes
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
                if (lane >= (uint32_t)o) incl &= y;
            }
            uint32_t excl = (uint32_t)__shfl_up((int)incl, 1, 64);
            if (lane == 0) excl = 0xFu;
            const uint32_t Pl = P & excl;
            const uint64_t m = __ballot((Pl & A) == 0u);
            if (m) {
                const uint32_t j = (uint32_t)__builtin_ctzll(m);
                uint32_t c = 0;
                if (lane == j) {  // the set just before the break
                    uint32_t S = Pl;
                    for (int k = 0; k < 32; ++k) {
                        const uint32_t T = S & ((v[k >> 3] >> (4 * (k & 7))) & 0xFu);
                        if (!T) break;
                        S = T;
                    }
                    c = S;
                }
                close = (uint32_t)__shfl((int)c, (int)j, 64);
                found = true;
            } else {
                P &= (uint32_t)__shfl((int)incl, 63, 64);
            }
        }
        if (!found) close = P;  // no run closes right of the chunk: the row's last run
    }
    // backward: the move table, right to left; the tile in hand is always
    // C[kEmitTiles - 1] (static register indices: the array shifts up a tile
    // per step, after a shift by kEmitTiles - L for a short chunk)
    for (uint32_t s = L; s < kEmitTiles; ++s) {
#pragma unroll
        for (int i = (int)kEmitTiles - 1; i >= 1; --i)
#pragma unroll
            for (int w = 0; w < 4; ++w) C[i][w] = C[i - 1][w];
    }
    carry = close;
    for (uint32_t t = t1; t-- > t0;) {
        fill_tile4(seg4_scan(C[kEmitTiles - 1], ent[(t - t0) * 64u + lane]), carry, orow,
                   t * 64u + lane, lb, lane);
#pragma unroll
        for (int i = (int)kEmitTiles - 1; i >= 1; --i)
#pragma unroll
            for (int w = 0; w < 4; ++w) C[i][w] = C[i - 1][w];
    }
    return exitS;
}

// The chunks' seams, a wave per row: lane j holds chunk b + j's guessed entry,
// exit and breaks; the first chunk whose guess differs from its left
// neighbour's (true) exit is done again from that exit (emit_chunk4, the
// whole wave), which may change its exit for the next comparison.
// counts[row] = the row's runs.
__global__ __launch_bounds__(64) void rle_emit_fix(const uint32_t* __restrict__ fm, uint32_t npad,
                                                   uint32_t nrows, const uint32_t* __restrict__ out_row,
                                                   uint32_t lb, uint32_t* __restrict__ dense,
                                                   EmitChunks ck, uint32_t* __restrict__ counts) {
    __shared__ uint8_t ent[64 * kEmitTiles];
    const uint32_t row = blockIdx.x;
    if (row >= nrows) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nseg = npad / kSeg, ntiles = npad / kTile;
    const uint32_t nch = (ntiles + kEmitTiles - 1u) / kEmitTiles;
    const uint4* __restrict__ f4 = reinterpret_cast<const uint4*>(fm);
    uint32_t* __restrict__ orow = dense + (size_t)out_row[row] * (npad >> (5u - lb));
    uint32_t carry = 0xFu, total = 0;
    for (uint32_t b = 0; b < nch; b += 64u) {
        const uint32_t c = b + lane;
        const bool valid = c < nch;
        const size_t at = (size_t)row * nch + c;
        uint32_t in = valid ? ck.xe[at] : 0u;
        uint32_t ex = valid ? ck.xs[at] : 0u;
        uint32_t cnt = valid ? ck.cc[at] : 0u;
        for (;;) {
            uint32_t pred = (uint32_t)__shfl_up((int)ex, 1, 64);
            if (lane == 0) pred = carry;
            const uint64_t m = __ballot(valid && pred != in);
            if (!m) break;
            const uint32_t j = (uint32_t)__builtin_ctzll(m);
            const uint32_t Sj = (uint32_t)__shfl((int)pred, (int)j, 64);
            const uint32_t t0 = (b + j) * kEmitTiles;
            uint32_t br = 0;
            const uint32_t xj = emit_chunk4(f4, row, nseg, ntiles, t0, min(ntiles, t0 + kEmitTiles), Sj,
                                            ent, orow, lb, lane, br);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) br += (uint32_t)__shfl_xor((int)br, o, 64);
            if (lane == j) {
                in = Sj;
                ex = xj;
                cnt = br;
            }
        }
        uint32_t sum = cnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += (uint32_t)__shfl_xor((int)sum, o, 64);
        total += sum;
        carry = (uint32_t)__shfl((int)ex, 63, 64);
    }
    if (lane == 0) counts[row] = total + 1u;  // + the row's first run
}

// ---------------------------------------------------------------------------
// The fused emit, eight rows per wave (round 6).  rle_emit4's wave scanned
// one row, so each greedy step moved one 4-bit set: ~17 VALU instructions
// per (row, column), and the emit, ALU-bound, took 15 ms of every step's
// CUs.  Here a lane holds one COLUMN of eight rows per 32-bit word (nibble i
// = row 8·oct + i; the 64-B sectors of the two row groups transposed in
// registers, three byte/nibble swap stages per 8x8 block), and one step of
// the scan — T = S & F, a zero-nibble test, S = T, or F where T is empty —
// advances all eight rows in nine instructions.  Lane L owns the kE8Cols = 32
// columns [c0 + 32 L, c0 + 32 L + 32) of a 2048-column chunk (kEmitTiles
// tiles: the chunk of rle_emit_fix and emit_chunk4):
//   guess    the running sets entering the lane: the 16 columns before it
//            scanned from a wildcard (lane 0: the previous chunk's last 16,
//            the chunk's guessed entry; a wildcard for chunk 0);
//   forward  its columns from that entry, each running set to LDS (8 KiB
//            per wave); a lane whose entry differs from lane L-1's exit scans
//            again from that exit (lane 0 keeps the chunk's entry) until no
//            lane changes;
//   ahead    the closing sets of the runs open at the chunk's right edge:
//            the following columns one per lane, a prefix-AND from the
//            chunk's exit, the first empty set per row;
//   backward right to left, each column's closing set (the set at the last
//            column of its run; a run ends before a break: S_c & S_c+1 is
//            empty), the breaks counted; the lane's trailing run is left
//            empty;
//   tails    the trailing run closes where the first lane to the right has,
//            per row, a break: at its column 0 with the lane's entry set,
//            else with that lane's first run's closing set; past the last
//            lane with the ahead set (a suffix scan over the lanes);
//   store    the lowest set bit per nibble, neighbouring columns merged to
//            the table's 1/2/4-bit fields and transposed back to rows: one
//            4-, 8- or 16-B store per row and lane, a wave writing 256 B-1
//            KiB contiguous per row.
// It records per (row, chunk) what round 5's one-row rle_emit4 recorded
// (guessed entry, exit, breaks), so rle_emit_fix repairs a wrong chunk guess
// with emit_chunk4, the one-row form, as before.
__device__ __forceinline__ uint32_t zero_nib(uint32_t a) {  // bit 3 of nibble k: nibble k is 0
    return ~(((a & 0x77777777u) + 0x77777777u) | a) & 0x88888888u;
}
__device__ __forceinline__ uint32_t nib_mask(uint32_t z) {  // bit-3 flags -> whole nibbles
    return z | (z - (z >> 3));
}
__device__ __forceinline__ uint32_t step8(uint32_t S, uint32_t F) {  // one column, 8 rows
    const uint32_t T = S & F;
    return T | (F & nib_mask(zero_nib(T)));
}
// 8x8 nibble transpose: nibble k of a[r] <-> nibble r of a[k] (the index bits
// 2, 1, 0 of word and nibble swapped in turn: half words, bytes, nibbles)
__device__ __forceinline__ void tr8(uint32_t (&a)[8]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t x = a[r], y = a[r + 4];
        a[r] = __builtin_amdgcn_perm(y, x, 0x05040100u);
        a[r + 4] = __builtin_amdgcn_perm(y, x, 0x07060302u);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (i & 1) | ((i & 2) << 1);  // 0, 1, 4, 5
        const uint32_t x = a[r], y = a[r + 2];
        a[r] = __builtin_amdgcn_perm(y, x, 0x06020400u);
        a[r + 2] = __builtin_amdgcn_perm(y, x, 0x07030501u);
    }
#pragma unroll
    for (int r = 0; r < 8; r += 2) {
        const uint32_t x = a[r], y = a[r + 1];
        a[r] = (x & 0x0F0F0F0Fu) | ((y << 4) & 0xF0F0F0F0u);
        a[r + 1] = ((x >> 4) & 0x0F0F0F0Fu) | (y & 0xF0F0F0F0u);
    }
}
__device__ __forceinline__ uint32_t low_bits8(uint32_t X) {  // lowest set bit of every nibble
    const uint32_t b0 = ~X & 0x11111111u;
    const uint32_t b1 = ~(X >> 1) & b0;
    const uint32_t b2 = ~(X >> 2) & b1;
    return b0 + b1 + b2;
}

static_assert(kEmitTiles * kTile == 64u * kE8Cols, "a chunk is 64 lanes x kE8Cols columns");

template <uint32_t LB>
__global__ __launch_bounds__(64) void rle_emit8(const uint32_t* __restrict__ fm, uint32_t npad,
                                                uint32_t nrows, const uint32_t* __restrict__ out_row,
                                                uint32_t* __restrict__ dense, EmitChunks ck,
                                                uint32_t remap) {
    __shared__ uint32_t run_set[kE8Cols * 64u];  // [column][lane]
    const uint32_t nseg = npad / kSeg, ntiles = npad / kTile;
    const uint32_t nch = (ntiles + kEmitTiles - 1u) / kEmitTiles;
    const uint32_t Lb = remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t oct = Lb / nch, ch = Lb - oct * nch;
    const uint32_t lane = threadIdx.x;
    const uint32_t r0 = oct * 8u;
    if (r0 >= nrows) return;  // wave-uniform
    const uint32_t c0 = ch * kEmitTiles * kTile;
    const uint32_t cl = c0 + lane * kE8Cols;   // the lane's first column
    const bool have = cl < npad;               // (a short last chunk: lanes past the row)
    const uint32_t last = min(63u, (npad - c0) / kE8Cols - 1u);  // the chunk's last lane
    const uint4* __restrict__ f4 = reinterpret_cast<const uint4*>(fm);
    uint32_t F[kE8Cols];  // column words (the running sets go to run_set, then the closing sets)
    {
        constexpr int NS = (int)kE8Cols / 32;  // segments per lane
        uint32_t R[8][4 * NS];                 // [row][8-column group]
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int h = 0; h < NS; ++h)
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const uint4 q = have ? f4[fm4_piece(r0 + 4u * g + p, nseg, cl / kSeg + h)]
                                         : make_uint4(~0u, ~0u, ~0u, ~0u);
                    R[4 * g + p][4 * h + 0] = q.x;
                    R[4 * g + p][4 * h + 1] = q.y;
                    R[4 * g + p][4 * h + 2] = q.z;
                    R[4 * g + p][4 * h + 3] = q.w;
                }
#pragma unroll
        for (int j = 0; j < 4 * NS; ++j) {
            uint32_t a[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) a[r] = R[r][j];
            tr8(a);
#pragma unroll
            for (int k = 0; k < 8; ++k) F[8 * j + k] = a[k];
        }
    }
    // guess: the 16 columns before the lane from a wildcard
    uint32_t in = ~0u;
    if (cl > 0u && have) {
        const uint2* __restrict__ f2 = reinterpret_cast<const uint2*>(fm);
        const uint32_t sp = cl / kSeg - 1u;
        uint32_t a[8], b[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint2 q = f2[fm4_piece(r0 + (uint32_t)r, nseg, sp) * 2u + 1u];  // columns 16..31
            a[r] = q.x;
            b[r] = q.y;
        }
        tr8(a);
        tr8(b);
        uint32_t S = a[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) S = step8(S, a[k]);
#pragma unroll
        for (int k = 0; k < 8; ++k) S = step8(S, b[k]);
        in = S;
    }
    const uint32_t guess0 = (uint32_t)__shfl((int)in, 0, 64);  // the chunk's guessed entry
    // forward, until every lane's entry is its left neighbour's exit
    uint32_t ex;
    for (;;) {
        uint32_t S = in;
#pragma unroll
        for (int c = 0; c < (int)kE8Cols; ++c) {
            S = step8(S, F[c]);
            run_set[(uint32_t)c * 64u + lane] = S;
            // (written as it goes: held back to the end, the 64 sets took 64 VGPRs more)
            if (c & 1) __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t pe = (uint32_t)__shfl_up((int)S, 1, 64);
        if (lane == 0) pe = in;
        const bool fix = have && pe != in;
        if (!__any(fix)) {
            ex = S;
            break;
        }
        if (fix) in = pe;
    }
    const uint32_t E = (uint32_t)__shfl((int)ex, (int)last, 64);  // the chunk's exit
    // ahead: per row, the set before the first break right of the chunk
    uint32_t A = 0u, open = ~0u, P = E;
    for (uint32_t cb = c0 + (last + 1u) * kE8Cols; cb < npad && open; cb += 64u) {
        const uint32_t col = cb + lane;
        uint32_t w = ~0u;
        if (col < npad) {
            const uint32_t seg = col / kSeg, wd = (col % kSeg) / 8u, sh = 4u * (col % 8u);
            w = 0u;
#pragma unroll
            for (int r = 0; r < 8; ++r)
                w |= ((fm[fm4_piece(r0 + (uint32_t)r, nseg, seg) * 4u + wd] >> sh) & 0xFu) << (4 * r);
        }
        uint32_t incl = w;  // prefix-AND over the lanes
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
            if (lane >= (uint32_t)d) incl &= y;
        }
        const uint32_t Rs = P & incl;             // the running set, no break since the edge
        const uint32_t z = zero_nib(Rs) & open;   // broken by this column
        uint32_t zp = (uint32_t)__shfl_up((int)z, 1, 64);
        uint32_t Rp = (uint32_t)__shfl_up((int)Rs, 1, 64);
        if (lane == 0) {
            zp = 0u;
            Rp = P;
        }
        const uint32_t first = z & ~zp;
        uint32_t got = Rp & nib_mask(first), res = first;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            got |= (uint32_t)__shfl_xor((int)got, o, 64);
            res |= (uint32_t)__shfl_xor((int)res, o, 64);
        }
        A |= got;
        open &= ~nib_mask(res);
        P = (uint32_t)__shfl((int)Rs, 63, 64);
    }
    A |= P & open;  // no break up to the row's end: the set there
    // backward: closing sets (the trailing run left 0), breaks counted
    uint32_t c4 = 0u, ce = 0u, co = 0u;  // nibble counters; even / odd rows' byte counters
    uint32_t W;                          // the run entering from the left: its closing set or 0
    {
        uint32_t Sn = run_set[(kE8Cols - 1u) * 64u + lane];
        uint32_t X = 0u;
        run_set[(kE8Cols - 1u) * 64u + lane] = 0u;
#pragma unroll
        for (int c = (int)kE8Cols - 2; c >= 0; --c) {
            const uint32_t Sc = run_set[(uint32_t)c * 64u + lane];
            const uint32_t z = zero_nib(Sc & Sn);  // a break at column c + 1
            const uint32_t m = nib_mask(z);
            X = (Sc & m) | (X & ~m);
            run_set[(uint32_t)c * 64u + lane] = X;
            if (c & 1) __builtin_amdgcn_sched_barrier(0);
            c4 += z >> 3;
            if (((int)kE8Cols - 2 - c) % 15 == 14) {
                ce += c4 & 0x0F0F0F0Fu;
                co += (c4 >> 4) & 0x0F0F0F0Fu;
                c4 = 0u;
            }
            Sn = Sc;
        }
        const uint32_t z0 = zero_nib(in & Sn);  // a break at column 0 (Sn = S_0)
        c4 += z0 >> 3;
        ce += c4 & 0x0F0F0F0Fu;
        co += (c4 >> 4) & 0x0F0F0F0Fu;
        const uint32_t m0 = nib_mask(z0);
        W = (in & m0) | (X & ~m0);
    }
    // tails: the first lane to the right with a closing set, per row
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = (uint32_t)__shfl_down((int)W, d, 64);
        if (lane + (uint32_t)d >= 64u) y = A;
        W |= nib_mask(zero_nib(W)) & y;
    }
    uint32_t tail = (uint32_t)__shfl_down((int)W, 1, 64);
    if (lane == 63u) tail = A;
    for (int c = (int)kE8Cols - 1; c >= 0; --c) {  // the trailing run: right to left, short
        const uint32_t x = run_set[(uint32_t)c * 64u + lane];
        const uint32_t z = zero_nib(x);
        if (!__any(z != 0u)) break;
        run_set[(uint32_t)c * 64u + lane] = x | (nib_mask(z) & tail);
    }
    // per-row breaks summed over the wave (16-bit halves: rows 0,4 / 2,6 / 1,5 / 3,7)
    uint32_t s0 = ce & 0x00FF00FFu, s1 = (ce >> 8) & 0x00FF00FFu;
    uint32_t s2 = co & 0x00FF00FFu, s3 = (co >> 8) & 0x00FF00FFu;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s0 += (uint32_t)__shfl_xor((int)s0, o, 64);
        s1 += (uint32_t)__shfl_xor((int)s1, o, 64);
        s2 += (uint32_t)__shfl_xor((int)s2, o, 64);
        s3 += (uint32_t)__shfl_xor((int)s3, o, 64);
    }
    if (have) {
        const size_t wpr = npad >> (5u - LB);
        constexpr int kWords = (int)(kE8Cols / 32u) << LB;  // table words per row and lane
        uint32_t out[8][kWords];
#pragma unroll
        for (int q = 0; q < kWords; ++q) {
            uint32_t a[8];
            constexpr int per = 4 >> LB;  // columns per nibble
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint32_t v = 0u;
#pragma unroll
                for (int b = 0; b < per; ++b)
                    v |= (low_bits8(run_set[(uint32_t)(q * 8 * per + j * per + b) * 64u + lane]) &
                          (LB == 0 ? 0x11111111u : 0x33333333u))
                         << ((1 << LB) * b);
                a[j] = v;
            }
            tr8(a);
#pragma unroll
            for (int r = 0; r < 8; ++r) out[r][q] = a[r];
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (r0 + (uint32_t)r >= nrows) continue;
            // the lane's kWords words at word (cl << LB) / 32 of the row
            uint32_t* __restrict__ ow = dense + (size_t)out_row[r0 + r] * wpr + ((cl << LB) >> 5);
            if constexpr (kWords >= 4) {
#pragma unroll
                for (int q = 0; q < kWords; q += 4)
                    reinterpret_cast<uint4*>(ow)[q / 4] =
                        make_uint4(out[r][q], out[r][q + 1], out[r][q + 2], out[r][q + 3]);
            } else if constexpr (kWords == 2) {
                reinterpret_cast<uint2*>(ow)[0] = make_uint2(out[r][0], out[r][1]);
            } else {
                ow[0] = out[r][0];
            }
        }
    }
    if (lane < 8u && r0 + lane < nrows) {
        const uint32_t w = (lane & 1u) ? ((lane & 2u) ? s3 : s2) : ((lane & 2u) ? s1 : s0);
        const size_t at = (size_t)(r0 + lane) * nch + ch;
        ck.xe[at] = (guess0 >> (4u * lane)) & 0xFu;
        ck.xs[at] = (E >> (4u * lane)) & 0xFu;
        ck.cc[at] = (lane & 4u) ? w >> 16 : w & 0xFFFFu;
    }
}

// The compact form on the wire and on disk: a move per column in `bits` =
// 1, 2 or 4 bits (every move of a graph whose out-degrees are <= 2^bits fits:
// a move indexes its column's out-list, and a wildcard run's lowest set bit
// is 0), ceil(n * bits / 32) words per row, rows back to back.  repack: any
// width to any width — the tables (stride words per row) to a file's packed
// rows on export, a file's rows to the tables on load when the widths differ
// (4-bit rows into a narrower index: each move must fit, which valid rows of
// the graph always do; *lost |= 1 when one does not).  One thread per output
// word; input past a row's s_words reads as 0.
__global__ __launch_bounds__(256) void repack_moves(const uint32_t* __restrict__ src,
                                                    uint32_t s_stride, uint32_t s_words,
                                                    uint32_t s_bits, uint32_t rows,
                                                    uint32_t* __restrict__ dst, uint32_t d_stride,
                                                    uint32_t d_words, uint32_t d_bits,
                                                    uint32_t* __restrict__ lost) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)rows * d_words) return;
    const uint32_t r = (uint32_t)(i / d_words), w = (uint32_t)(i % d_words);
    const uint32_t per = 32u / d_bits;  // columns per output word
    const uint32_t* __restrict__ in = src + (size_t)r * s_stride;
    auto at = [&](uint32_t k) { return k < s_words ? in[k] : 0u; };
    if (s_bits == 4u && d_bits == 2u && !lost) {  // nibble tables -> 2 bits (export, index)
        dst[(size_t)r * d_stride + w] = nib_to2(at(2u * w)) | (nib_to2(at(2u * w + 1u)) << 16);
        return;
    }
    if (s_bits == 4u && d_bits == 1u && !lost) {
        dst[(size_t)r * d_stride + w] = nib_to1(at(4u * w)) | (nib_to1(at(4u * w + 1u)) << 8) |
                                        (nib_to1(at(4u * w + 2u)) << 16) | (nib_to1(at(4u * w + 3u)) << 24);
        return;
    }
    if (s_bits == 2u && d_bits == 4u) {  // 2-bit rows -> nibble tables
        dst[(size_t)r * d_stride + w] = nib_from2(at(w >> 1) >> (16u * (w & 1u)));
        return;
    }
    if (s_bits == 1u && d_bits == 4u) {
        dst[(size_t)r * d_stride + w] = nib_from1(at(w >> 2) >> (8u * (w & 3u)));
        return;
    }
    const uint32_t smask = (1u << s_bits) - 1u, dmask = (1u << d_bits) - 1u;
    uint32_t o = 0, wide = 0;
    for (uint32_t k = 0; k < per; ++k) {
        const uint64_t bit = (uint64_t)(w * per + k) * s_bits;  // first bit in the input row
        const uint32_t sw = (uint32_t)(bit >> 5);
        const uint32_t v = sw < s_words ? (in[sw] >> (bit & 31u)) & smask : 0u;
        o |= (v & dmask) << (d_bits * k);
        wide |= v & ~dmask;
    }
    dst[(size_t)r * d_stride + w] = o;
    // a move that does not fit the output width (only rows from outside the
    // library can carry one): flagged, never silently truncated
    if (lost && __any(wide != 0u) && (threadIdx.x & 63u) == 0u) atomicOr(lost, 1u);
}

// Move tables -> RLE words, the inverse of rle_moves: a row's runs start at
// column 0 and at every column whose move differs from its left neighbour's,
// word = column << 4 | move (warthog rle_run32 [U]); columns >= n are
// ignored.  EMIT = false: counts[r] = the row's runs; EMIT = true: the runs at
// runs[off[r] - base].  A wave per row, 2048-column tiles left to right, runs
// staged per tile in LDS and stored coalesced.  Row r's table at
// dense + r * stride, 2^lb bits per column (Tbl).
template <bool EMIT>
__global__ __launch_bounds__(256) void moves_runs(const uint32_t* __restrict__ dense,
                                                  uint32_t stride, uint32_t lb, uint32_t n,
                                                  uint32_t nrows,
                                                  const uint64_t* __restrict__ off, uint64_t base,
                                                  uint32_t* __restrict__ runs,
                                                  uint32_t* __restrict__ counts) {
    __shared__ uint32_t stage_all[EMIT ? 4 * kTile : 1];
    const uint32_t row = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (row >= nrows) return;
    uint32_t* stage = stage_all + (EMIT ? (threadIdx.x >> 6) * kTile : 0u);
    const uint32_t* __restrict__ rowp = dense + (size_t)row * stride;
    uint32_t* __restrict__ out = EMIT ? runs + (off[row] - base) : nullptr;
    const uint32_t ntiles = (n + kTile - 1u) / kTile;
    uint32_t prev = 0x10u;  // no nibble: column 0 always starts a run
    uint32_t total = 0;
    // the next tile's columns are loaded while this one is scanned and
    // stored (one load in flight per wave left the kernel at ~3.6 TB/s)
    // (raw words in flight; widened to nibbles only when scanned, or the
    // widening would wait for the load right away)
    auto raw_load = [&](uint32_t g) {
        if (lb == 2u) return reinterpret_cast<const uint4*>(rowp)[g];
        if (lb == 1u) {
            const uint2 q = reinterpret_cast<const uint2*>(rowp)[g];
            return make_uint4(q.x, q.y, 0u, 0u);
        }
        return make_uint4(rowp[g], 0u, 0u, 0u);
    };
    uint4 rn = lane * kSeg < n ? raw_load(lane) : make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t t = 0; t < ntiles; ++t) {
        const uint32_t c0 = t * kTile + lane * kSeg;
        const uint4 r = rn;
        rn = (t + 1u < ntiles && c0 + kTile < n) ? raw_load((t + 1u) * 64u + lane)
                                                  : make_uint4(0u, 0u, 0u, 0u);
        uint32_t x[4];
        if (lb == 2u) {
            x[0] = r.x;
            x[1] = r.y;
            x[2] = r.z;
            x[3] = r.w;
        } else if (lb == 1u) {
            x[0] = nib_from2(r.x);
            x[1] = nib_from2(r.x >> 16);
            x[2] = nib_from2(r.y);
            x[3] = nib_from2(r.y >> 16);
        } else {
            x[0] = nib_from1(r.x);
            x[1] = nib_from1(r.x >> 8);
            x[2] = nib_from1(r.x >> 16);
            x[3] = nib_from1(r.x >> 24);
        }
        if (c0 >= n) x[0] = x[1] = x[2] = x[3] = 0u;
        uint32_t pl = (uint32_t)__shfl_up((int)(x[3] >> 28), 1, 64);
        if (lane == 0) pl = prev;
        uint32_t chg = 0;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const uint32_t mv = (x[k >> 3] >> (4 * (k & 7))) & 0xFu;
            const uint32_t pv = k == 0 ? pl : (x[(k - 1) >> 3] >> (4 * ((k - 1) & 7))) & 0xFu;
            chg |= (mv != pv ? 1u : 0u) << k;
        }
        if (c0 + kSeg > n) chg &= c0 >= n ? 0u : (uint32_t)((1ull << (n - c0)) - 1ull);
        const uint32_t cnt = (uint32_t)__builtin_popcount(chg);
        uint32_t incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        const uint32_t tile_total = (uint32_t)__shfl((int)incl, 63, 64);
        if (EMIT) {
            uint32_t p = incl - cnt;
            for (uint32_t b = chg; b; b &= b - 1u) {
                const uint32_t k = (uint32_t)__builtin_ctz(b);
                stage[p++] = ((c0 + k) << 4) | nib_at(x[0], x[1], x[2], x[3], k);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
            for (uint32_t i = lane; i < tile_total; i += 64u) out[total + i] = stage[i];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        total += tile_total;
        prev = (uint32_t)__shfl((int)(x[3] >> 28), 63, 64);
    }
    if (!EMIT && lane == 0) counts[row] = total;
}

// ---------------------------------------------------------------------------
// RLE count, chunked (4-bit sets; CPD_RLE_CH, default on).  rle_scan<false>
// gives each lane one 32-column segment of a 2048-column tile and guesses
// the state entering it (16 look-back columns), then rescans every segment
// whose guess was wrong — and a wave pays a whole rescan whenever any of
// its 64 lanes needs one — about 80 column steps per 32 useful ones.  Here a
// lane owns a chunk of CH consecutive segments of one row and scans them in
// order, so only the chunk's entry is guessed (16 look-back columns per
// CH x 32), and the guesses are checked afterwards by rle_fix, one wave per
// row, which rescans the rare chunk whose guess differs from its
// predecessor's exit.  A wave = 4 rows (one row group of the interleaved fm
// layout: its 4 lanes of a chunk read one 64-B sector) x 16 chunks.
// Per segment the lane keeps the entry state (RleState st, stored 8
// segments = 32 B at a time) and the run count (rc, stored 32 segments =
// 32 B at a time), per chunk its exit state and run count (xs / cc).
struct RleChunks {
    uint32_t* xs;  // [nrows][nch] exit state (h << 4 | S) of the chunk
    uint32_t* cc;  // [nrows][nch] runs ending inside the chunk
    uint32_t* xe;  // [nrows][nch] its guessed entry state (= its first segment's st):
                   // rle_fix reads the seams from here, 4 B per chunk, instead of
                   // one 4-B state per 128-B line of st (3.4 GB per 24576-row
                   // launch)
};

// the greedy scan over one 32-column segment (word v[c / 8], nibble c % 8)
// from (h, S); returns the runs that end inside it, updates (h, S)
__device__ __forceinline__ uint32_t seg_count4(const uint4& q, uint32_t c0, uint32_t& h,
                                               uint32_t& S) {
    const uint32_t v[4] = {q.x, q.y, q.z, q.w};
    uint32_t brk = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t word = v[w];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t f = word & 0xFu;
            word >>= 4;
            const uint32_t T = S & f;
            brk |= (T == 0u ? 1u : 0u) << (8 * w + j);
            S = T == 0u ? f : T;
        }
    }
    if (brk) h = c0 + 31u - (uint32_t)__builtin_clz(brk);
    return (uint32_t)__builtin_popcount(brk);
}

template <int CH>
__global__ __launch_bounds__(256) void rle_count_ch(const uint32_t* __restrict__ fm,
                                                    uint32_t npad, uint32_t nrows,
                                                    uint32_t* __restrict__ st,
                                                    uint8_t* __restrict__ rc, RleChunks rk) {
    static_assert(CH % 32 == 0, "whole 32-B count stores");
    const uint32_t nseg = npad / kSeg, nch = nseg / CH;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t rg = blockIdx.y * 4u + (threadIdx.x >> 6);  // row group of this wave
    const uint32_t row = rg * 4u + (lane & 3u);
    const uint32_t ch = blockIdx.x * 16u + (lane >> 2);
    if (row >= nrows || ch >= nch) return;
    const uint4* __restrict__ f4 = reinterpret_cast<const uint4*>(fm);
    const uint32_t s0 = ch * CH;
    uint32_t h = 0, S = 0xFu;  // entering column 0: head 0, wildcard set
    if (ch > 0) {  // the guess: the previous segment's last 16 columns from a fresh run
        const uint4 q = f4[fm4_piece(row, nseg, s0 - 1u)];
        const uint32_t v[2] = {q.z, q.w};
        const uint32_t c0 = s0 * kSeg - 16u;
        h = c0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t f = (v[k / 8] >> (4 * (k % 8))) & 0xFu;
            const uint32_t T = S & f;
            h = T == 0u ? c0 + (uint32_t)k : h;
            S = T == 0u ? f : T;
        }
    }
    uint32_t* __restrict__ stp = st + (size_t)row * nseg + s0;
    rk.xe[(size_t)row * nch + ch] = (h << 4) | S;
    uint32_t total = 0;
    uint4 nq = f4[fm4_piece(row, nseg, s0)];
    uint2 r0 = {}, r1 = {}, r2 = {};  // counts of segments 0-7, 8-15, 16-23 of 32
#pragma unroll 1
    for (uint32_t s = 0; s < (uint32_t)CH; s += 8u) {  // 8 segments: 32 B of states
        uint32_t sw[8];
        uint2 r8 = {0u, 0u};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t seg = s0 + s + (uint32_t)i;
            const uint4 q = nq;
            if (s + (uint32_t)i + 1u < (uint32_t)CH) nq = f4[fm4_piece(row, nseg, seg + 1u)];
            sw[i] = (h << 4) | S;
            const uint32_t k = seg_count4(q, seg * kSeg, h, S);
            total += k;
            if (i < 4) r8.x |= k << (8 * i);
            else r8.y |= k << (8 * (i - 4));
        }
        uint4* o = reinterpret_cast<uint4*>(stp + s);
        o[0] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
        o[1] = make_uint4(sw[4], sw[5], sw[6], sw[7]);
        switch ((s / 8u) & 3u) {  // the counts go out 32 segments (32 B) at a time
            case 0: r0 = r8; break;
            case 1: r1 = r8; break;
            case 2: r2 = r8; break;
            default: {
                uint4* orc = reinterpret_cast<uint4*>(rc + (size_t)row * nseg + s0 + s - 24u);
                orc[0] = make_uint4(r0.x, r0.y, r1.x, r1.y);
                orc[1] = make_uint4(r2.x, r2.y, r8.x, r8.y);
            }
        }
    }
    rk.xs[(size_t)row * nch + ch] = (h << 4) | S;
    rk.cc[(size_t)row * nch + ch] = total;
}

// Chunk seams of rle_count_ch, one wave per row: lane j holds chunk b + j's
// guessed entry state (its first segment's stored state), exit state and run
// count.  A chunk whose entry differs from its predecessor's exit is rescanned
// from the true state by its lane, segment by segment, rewriting the segment
// states and counts, until the state meets the stored one (from there on the
// stored states are the true ones); a chunk rescanned to its end passes a new
// exit state on.  The lowest such chunk is fixed first, so every fix starts
// from a true state.  counts[row] = the row's runs (+ the final one).
// A row whose rescans pass kFixBudget segments (runs far longer than the
// look-back — never on road graphs, where a run averages 1.6 columns, but a
// chain graph has a handful of runs per row) is given up: *hard = 1, and the
// host re-counts the batch with rle_scan<false>, which bounds that case.
constexpr uint32_t kFixBudget = 256;  // segments rescanned per row

template <int CH>
__global__ __launch_bounds__(64) void rle_fix(const uint32_t* __restrict__ fm, uint32_t npad,
                                              uint32_t nrows, uint32_t* __restrict__ st,
                                              uint8_t* __restrict__ rc, RleChunks rk,
                                              uint32_t* __restrict__ counts,
                                              uint32_t* __restrict__ hard) {
    const uint32_t row = blockIdx.x;
    if (row >= nrows) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nseg = npad / kSeg, nch = nseg / CH;
    uint32_t* __restrict__ str = st + (size_t)row * nseg;
    uint8_t* __restrict__ rcr = rc + (size_t)row * nseg;
    uint32_t* __restrict__ xs = rk.xs + (size_t)row * nch;
    const uint32_t* __restrict__ cc = rk.cc + (size_t)row * nch;
    const uint4* __restrict__ f4 = reinterpret_cast<const uint4*>(fm);
    uint32_t carry = 0xFu;  // entering column 0: head 0, wildcard set
    uint32_t total = 0, spent = 0;
    for (uint32_t b = 0; b < nch; b += 64u) {
        const uint32_t c = b + lane;
        const bool valid = c < nch;
        uint32_t in = valid ? rk.xe[(size_t)row * nch + c] : 0u;
        uint32_t ex = valid ? xs[c] : 0u;
        uint32_t cnt = valid ? cc[c] : 0u;
        for (;;) {
            uint32_t pred = __shfl_up(ex, 1, 64);
            if (lane == 0) pred = carry;
            const uint64_t m = __ballot(valid && pred != in);
            if (!m) break;
            const uint32_t j = (uint32_t)__builtin_ctzll(m);
            uint32_t nres = 0;
            if (lane == j) {
                uint32_t state = pred;
                int delta = 0;
                bool met = false;
                for (uint32_t s = c * CH; s < (c + 1u) * CH; ++s) {
                    if (state == str[s]) {
                        met = true;
                        break;
                    }
                    ++nres;
                    str[s] = state;
                    uint32_t hh = state >> 4, SS = state & 0xFu;
                    const uint32_t k = seg_count4(f4[fm4_piece(row, nseg, s)], s * kSeg, hh, SS);
                    delta += (int)k - (int)rcr[s];
                    rcr[s] = (uint8_t)k;
                    state = (hh << 4) | SS;
                }
                in = pred;
                cnt = (uint32_t)((int)cnt + delta);
                if (!met) {
                    ex = state;
                    xs[c] = state;
                }
            }
            spent += __shfl(nres, (int)j, 64);  // wave-uniform
            if (spent > kFixBudget) {
                if (lane == 0) *hard = 1u;
                return;
            }
        }
        uint32_t sum = cnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
        total += sum;
        carry = __shfl(ex, 63, 64);
    }
    if (lane == 0) counts[row] = total + 1u;  // + the final run
}

// ---------------------------------------------------------------------------
// Query batches on the GPU (cpd_query_prepare / cpd_query_fetch; VERDICT r03
// item 4): the caller's (s, t) node ids are mapped to columns and target rows,
// sorted by row (a radix sort of (row, query) pairs: stable, so the order is
// the host counting sort's) so that a wave's lanes walk the same row, and the
// per-query results go back to the caller's order by a scatter — no per-query
// host work.  bad |= 1: a node out of range, 2: a target without a row.
__global__ __launch_bounds__(256) void query_keys(const uint32_t* __restrict__ s,
                                                  const uint32_t* __restrict__ t, uint32_t nq,
                                                  uint32_t n, const uint32_t* __restrict__ order,
                                                  const uint32_t* __restrict__ row_of_col,
                                                  uint32_t* __restrict__ key,
                                                  uint32_t* __restrict__ val,
                                                  uint32_t* __restrict__ bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const uint32_t a = s[i], b = t[i];
    uint32_t f = 0, row = 0;
    if (a >= n || b >= n) {
        f = 1;
    } else {
        row = row_of_col[order[b]];
        if (row == INF) f = 2;
    }
    key[i] = f ? 0u : row;
    val[i] = i;
    if (f) atomicOr(bad, f);
}

__global__ __launch_bounds__(256) void query_gather(const uint32_t* __restrict__ s,
                                                    const uint32_t* __restrict__ t,
                                                    const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ key,
                                                    const uint32_t* __restrict__ val, uint32_t nq,
                                                    uint32_t* __restrict__ qs,
                                                    uint32_t* __restrict__ qt,
                                                    uint32_t* __restrict__ qrow) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const uint32_t q = val[i];
    qs[i] = order[s[q]];
    qt[i] = order[t[q]];
    qrow[i] = key[i];
}

// out[perm[i] * k + j] = in[i * k + j]: row-sorted results back to the
// caller's order (k values per query)
template <class T>
__global__ __launch_bounds__(256) void scatter_rows(const T* __restrict__ in,
                                                    const uint32_t* __restrict__ perm, uint32_t nq,
                                                    uint32_t k, T* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)nq * k) return;
    const uint32_t q = (uint32_t)(i / k), j = (uint32_t)(i % k);
    out[(size_t)perm[q] * k + j] = in[i];
}

// Table-search extraction (table_walk below).  cur/t are columns; the run for
// column cur is found by galloping from the previous hop's run (consecutive
// path nodes have nearby DFS columns), then binary search inside the bracket:
// the result is always the LAST run with start <= cur — the same run warthog's
// get_move binary search returns [U].  Edges come from a packed fixed-stride
// adjacency: edge k of column c is adj[(c << shift) + k] = (dst column, weight),
// dst = kNoEdge past the out-degree — one 8-B load per move, no row_ptr.

// Per-wave sums of (cost, moves, finished) added to agg[2], agg[1], agg[0].
__device__ void wave_stats(uint64_t cost, uint32_t hops, uint32_t fin,
                           unsigned long long* __restrict__ agg);

// Expand RLE rows into dense 4-bit move tables (8 columns per u32, column c at
// bits 4*(c&7) of word c>>3; column c's move = the move of the last run that
// starts at or before c — copied, never recomputed).
//
// Work is cut by RUNS, not columns: chunks of kExpandRuns consecutive runs of
// one row (chunk_first[row] = the row's first chunk, a prefix over rows of
// ceil(R / kExpandRuns)); a wave takes kExpandCpw consecutive chunks, loads each plus the next 8 runs (coalesced, into LDS)
// and writes the output words whose first column lies in the chunk:
// [ceil(start(r0) / 8), ceil(start(r1) / 8)) — the first chunk of a row from
// word 0, the last to the end of the row — a lane per word (the last staged
// run at or before its first column by binary search, then its 8 columns).
// A word's 8 columns are covered by at most 8 runs past r1, so the lookahead
// completes every owned word and each word has exactly one writer.  Round 2's
// form (wave per 2048-column tile, two ~20-step binary searches over the row's
// runs per wave) read 1.6x its algorithmic bytes at 0.12 of HBM peak; one
// chunk per wave (round 3's first form) ran 6.5M workgroups at 1M nodes (42.9 ms
// per 21504 rows; 4 chunks: 35.2; 16: 32.8).
// (A lane per RUN instead — each word written by the run holding its first
// column, interiors as a segmented fill — measured 100 ms against 39 for
// 21504 rows: five times as many lanes' worth of work as words.  A bitmap of
// the chunk's run starts with prefix popcounts in place of the binary
// search: 38.8 ms against 32.8.)
constexpr uint32_t kExpandRuns = 512;
constexpr uint32_t kExpandCpw = 16;

__global__ __launch_bounds__(256) void expand_rows(const uint64_t* __restrict__ offsets,
                                                   const uint32_t* __restrict__ runs,
                                                   const uint32_t* __restrict__ chunk_first,
                                                   uint32_t nrows, uint32_t total_chunks,
                                                   uint32_t words_per_row, uint32_t cpw,
                                                   uint32_t* __restrict__ dense) {
    constexpr uint32_t kLook = 8;
    __shared__ uint32_t cr_all[4][kExpandRuns + kLook];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t c_begin = (blockIdx.x * 4u + wv) * cpw;
    if (c_begin >= total_chunks) return;  // wave-uniform; no block barrier below
    const uint32_t c_end = min(total_chunks, c_begin + cpw);
    uint32_t* cr = cr_all[wv];
    // the first chunk's row: the last row whose first chunk is <= it (uniform)
    uint32_t lo = 0, hi = nrows;
    while (lo + 1 < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (chunk_first[mid] <= c_begin) lo = mid;
        else hi = mid;
    }
    uint32_t row = lo;
    for (uint32_t chunk = c_begin; chunk < c_end; ++chunk) {
        while (chunk_first[row + 1] <= chunk) ++row;  // rows of >= 1 chunk
        const uint64_t o0 = offsets[row];
        const uint32_t R = (uint32_t)(offsets[row + 1] - o0);
        const uint32_t r0 = (chunk - chunk_first[row]) * kExpandRuns;
        const uint32_t r1 = min(R, r0 + kExpandRuns);
        const uint32_t nl = min(R, r1 + kLook) - r0;  // runs staged
        const uint32_t* __restrict__ rr = runs + o0 + r0;
        __builtin_amdgcn_wave_barrier();  // the previous chunk's LDS reads are done
        for (uint32_t i = lane; i < nl; i += 64u) cr[i] = rr[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t w0 = r0 == 0 ? 0u : ((cr[0] >> 4) + 7u) >> 3;
        const uint32_t w1 = r1 == R ? words_per_row : ((cr[r1 - r0] >> 4) + 7u) >> 3;
        uint32_t* __restrict__ out = dense + (size_t)row * words_per_row;
        uint32_t a0 = 0;  // this lane's previous word's run: its next word starts there or later
        for (uint32_t w = w0 + lane; w < w1; w += 64u) {
            const uint32_t c0 = w * 8u;
            uint32_t a = a0, b = nl;  // last staged run with start <= c0
            while (a + 1 < b) {
                const uint32_t mid = (a + b) >> 1;
                if ((cr[mid] >> 4) > c0) b = mid;
                else a = mid;
            }
            a0 = a;
            uint32_t word = 0;
#pragma unroll
            for (uint32_t k = 0; k < 8u; ++k) {
                while (a + 1 < nl && (cr[a + 1] >> 4) <= c0 + k) ++a;
                word |= (cr[a] & 0xFu) << (4u * k);
            }
            out[w] = word;
        }
    }
}

// Row format check for rows loaded from outside the library (bucket files,
// host arrays), in expand_rows' run chunks: *bad |= 1 when a row does not
// start at column 0, its run columns do not strictly increase, or a column
// is >= n, or (mlimit < 16: rows bound for tables narrower than 4 bits) a
// move does not fit the table's field.  expand_rows and the binary searches rely on exactly these
// properties (a run's move is checked by the walk itself: a move naming no
// edge of its column stops the walk, so it is not checked here — a run that
// starts on a wildcard column may legally carry a move that column does not
// have).  Empty rows are refused on the host.
__global__ __launch_bounds__(256) void validate_rows(const uint64_t* __restrict__ offsets,
                                                     const uint32_t* __restrict__ runs,
                                                     const uint32_t* __restrict__ chunk_first,
                                                     uint32_t nrows, uint32_t total_chunks,
                                                     uint32_t n, uint32_t mlimit,
                                                     uint32_t* __restrict__ bad) {
    const uint32_t chunk = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (chunk >= total_chunks) return;
    uint32_t lo = 0, hi = nrows;
    while (lo + 1 < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (chunk_first[mid] <= chunk) lo = mid;
        else hi = mid;
    }
    const uint64_t o0 = offsets[lo];
    const uint32_t R = (uint32_t)(offsets[lo + 1] - o0);
    const uint32_t r0 = (chunk - chunk_first[lo]) * kExpandRuns;
    const uint32_t r1 = min(R, r0 + kExpandRuns);
    bool b = false;
    for (uint32_t i = r0 + lane; i < r1; i += 64u) {
        const uint32_t c = runs[o0 + i] >> 4;
        b |= c >= n;
        b |= (runs[o0 + i] & 0xFu) >= mlimit;
        if (i == 0) b |= c != 0u;
        else b |= c <= (runs[o0 + i - 1] >> 4);
    }
    if (__any(b) && lane == 0) atomicOr(bad, 1u);
}

// ---------------------------------------------------------------------------
// Table-search v2: the same walk, the same results, restructured for latency.
//
// (1) Adjacency co-fetch.  A hop's two loads — the move of column cur and the
//     packed edge (cur, move) — both depend only on cur, so for <= 4 slots per
//     column the whole adjacency row of cur (<= 32 B: one or two 16-B loads)
//     is fetched beside the move word and the edge is picked in registers: one
//     memory round trip per hop instead of two.  (Wider adjacency: the edge
//     load still follows the move.)
// (2) Lane refill.  Path lengths differ by several x inside a wave (s is
//     uniform over the graph), so a lane per query leaves most lanes idle
//     while the wave waits for its longest walk.  Here a wave owns `chunk`
//     consecutive queries of the target-sorted batch; a lane whose walk ends
//     stores its result and takes the next unstarted query of the chunk (rank
//     among the wave's finishing lanes by mbcnt, a wave-uniform cursor in an
//     SGPR), so lanes stay busy until the chunk runs dry.
// (3) ILP walks per lane, issued together: more loads in flight per wave.
// qrow[q] = the row of query q's target (host-computed with the sort).
constexpr uint32_t kIdleQ = 0xFFFFFFFFu;

struct DenseRows {
    const uint32_t* __restrict__ dense;
    uint32_t wpr;  // words per row
    Tbl tb;        // bits per column
};

struct RleRows {
    const uint64_t* __restrict__ off;
    const uint32_t* __restrict__ runs;
};

struct WalkState {
    uint32_t q, cur, t, hops, pos, R;
    uint64_t cost;
    const uint32_t* row;  // dense words / RLE runs of the query's row
    bool bad;             // a move past the out-degree (malformed row): stop
};

__device__ __forceinline__ void walk_begin(WalkState& w, uint32_t q, const uint32_t* __restrict__ qs,
                                           const uint32_t* __restrict__ qt,
                                           const uint32_t* __restrict__ qrow, const DenseRows& d) {
    w.q = q;
    w.cur = qs[q];
    w.t = qt[q];
    w.row = d.dense + (size_t)qrow[q] * d.wpr;
    w.hops = 0;
    w.cost = 0;
    w.bad = false;
}

__device__ __forceinline__ void walk_begin(WalkState& w, uint32_t q, const uint32_t* __restrict__ qs,
                                           const uint32_t* __restrict__ qt,
                                           const uint32_t* __restrict__ qrow, const RleRows& r) {
    w.q = q;
    w.cur = qs[q];
    w.t = qt[q];
    const uint32_t row = qrow[q];
    const uint64_t o0 = r.off[row], o1 = r.off[row + 1];
    w.row = r.runs + o0;
    w.R = (uint32_t)(o1 - o0);
    w.pos = 0;
    w.hops = 0;
    w.cost = 0;
    w.bad = false;
}

__device__ __forceinline__ const uint32_t* rows_base(const DenseRows& d) { return d.dense; }
__device__ __forceinline__ const uint32_t* rows_base(const RleRows& r) { return r.runs; }

__device__ __forceinline__ uint32_t walk_move(WalkState& w, const DenseRows& d) {
    return d.tb.move(w.row, w.cur);
}

// The last run with start <= cur, galloping from the previous hop's run.
__device__ __forceinline__ uint32_t walk_move(WalkState& w, const RleRows&) {
    const uint32_t* __restrict__ rr = w.row;
    const uint32_t cur = w.cur, R = w.R, pos = w.pos;
    uint32_t lo, hi;  // invariant: start(lo) <= cur < start(hi) (hi == R: +inf)
    if ((rr[pos] >> 4) <= cur) {
        lo = pos;
        uint32_t step = 1;
        hi = pos + 1;
        while (hi < R && (rr[hi] >> 4) <= cur) {
            lo = hi;
            step <<= 1;
            hi = lo + step;
        }
        if (hi > R) hi = R;
    } else {
        hi = pos;
        uint32_t step = 1;
        lo = pos >= 1 ? pos - 1 : 0;
        while (lo > 0 && (rr[lo] >> 4) > cur) {
            hi = lo;
            step <<= 1;
            lo = hi > step ? hi - step : 0;
        }
    }
    while (lo + 1 < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if ((rr[mid] >> 4) > cur) hi = mid;
        else lo = mid;
    }
    w.pos = lo;
    return rr[lo] & 0xFu;
}

// One hop of a walking lane.  SHIFT <= 2: the adjacency row of cur is loaded
// before the move is known (co-fetch); otherwise the edge load follows it.
template <int SHIFT, class Rows>
__device__ __forceinline__ void walk_hop(WalkState& w, const uint2* __restrict__ adj,
                                         const Rows& rows) {
    uint32_t ex, ew;
    if (SHIFT == 2) {
        const uint4* a4 = reinterpret_cast<const uint4*>(adj) + 2u * (size_t)w.cur;
        const uint4 p0 = a4[0], p1 = a4[1];
        const uint32_t mv = walk_move(w, rows);
        const uint4 p = (mv & 2u) ? p1 : p0;
        ex = (mv & 1u) ? p.z : p.x;
        ew = (mv & 1u) ? p.w : p.y;
        if (mv > 3u) ex = kNoEdge;
    } else if (SHIFT == 1) {
        const uint4 p = reinterpret_cast<const uint4*>(adj)[w.cur];
        const uint32_t mv = walk_move(w, rows);
        ex = (mv & 1u) ? p.z : p.x;
        ew = (mv & 1u) ? p.w : p.y;
        if (mv > 1u) ex = kNoEdge;
    } else if (SHIFT == 0) {
        const uint2 p = adj[w.cur];
        const uint32_t mv = walk_move(w, rows);
        ex = mv == 0u ? p.x : kNoEdge;
        ew = p.y;
    } else {  // wide adjacency: the edge load follows the move
        const uint32_t mv = walk_move(w, rows);
        if (mv >> SHIFT) {  // names no slot of cur: malformed row
            w.bad = true;
            return;
        }
        const uint2 e = adj[((size_t)w.cur << SHIFT) + mv];
        ex = e.x;
        ew = e.y;
    }
    if (ex == kNoEdge) {
        w.bad = true;
        return;
    }
    w.cost += ew;
    w.cur = ex;
    ++w.hops;
}

// Dense rows, all ILP walks of a lane at once: every slot's move word and
// adjacency row are loaded unconditionally (an idle slot keeps a valid column
// and row pointer), then the walking slots step — the loads of the ILP walks
// are in flight together instead of one branch region after another.
template <int SHIFT, int ILP>
__device__ __forceinline__ void walk_hops(WalkState (&w)[ILP], const uint2* __restrict__ adj,
                                          const DenseRows& d) {
    constexpr int NQ = SHIFT == 2 ? 2 : 1;  // 16-B pieces of an adjacency row
    const uint32_t wsh = 5u - d.tb.lb, cm = 31u >> d.tb.lb, mm = (1u << (1u << d.tb.lb)) - 1u;
    uint32_t word[ILP];
    uint4 p[ILP][NQ];
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
        word[i] = w[i].row[w[i].cur >> wsh];
        if (SHIFT <= 2) {
            if (SHIFT == 0) {
                const uint2 e = adj[w[i].cur];
                p[i][0] = make_uint4(e.x, e.y, kNoEdge, 0u);
            } else {
                const uint4* a4 = reinterpret_cast<const uint4*>(adj) + (size_t)w[i].cur * NQ;
#pragma unroll
                for (int k = 0; k < NQ; ++k) p[i][k] = a4[k];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
        if (w[i].q == kIdleQ || w[i].cur == w[i].t) continue;
        const uint32_t mv = (word[i] >> ((w[i].cur & cm) << d.tb.lb)) & mm;
        uint32_t ex, ew;
        if (SHIFT <= 2) {
            const uint4 q = (NQ == 2 && (mv & 2u)) ? p[i][NQ - 1] : p[i][0];
            ex = (mv & 1u) ? q.z : q.x;
            ew = (mv & 1u) ? q.w : q.y;
            if (mv >> SHIFT) ex = kNoEdge;
        } else {
            if (mv >> SHIFT) {
                w[i].bad = true;
                continue;
            }
            const uint2 e = adj[((size_t)w[i].cur << SHIFT) + mv];
            ex = e.x;
            ew = e.y;
        }
        if (ex == kNoEdge) {
            w[i].bad = true;
            continue;
        }
        w[i].cost += ew;
        w[i].cur = ex;
        ++w[i].hops;
    }
}

template <int SHIFT, int ILP>
__device__ __forceinline__ void walk_hops(WalkState (&w)[ILP], const uint2* __restrict__ adj,
                                          const RleRows& rows) {
#pragma unroll
    for (int i = 0; i < ILP; ++i)
        if (w[i].q != kIdleQ && w[i].cur != w[i].t) walk_hop<SHIFT>(w[i], adj, rows);
}

template <int SHIFT, int ILP, class Rows>
__global__ __launch_bounds__(256) void table_walk(
    const uint2* __restrict__ adj, Rows rows, const uint32_t* __restrict__ qs,
    const uint32_t* __restrict__ qt, const uint32_t* __restrict__ qrow, uint32_t nq,
    uint32_t chunk, uint32_t limit, uint64_t* __restrict__ cost_out,
    uint32_t* __restrict__ hops_out, uint8_t* __restrict__ fin_out,
    unsigned long long* __restrict__ agg) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t q0l = wave * chunk;
    const uint32_t q0 = q0l < nq ? (uint32_t)q0l : nq;
    const uint32_t q1 = (uint32_t)min((uint64_t)nq, q0l + chunk);
    uint64_t sum_cost = 0;
    uint32_t sum_hops = 0, sum_fin = 0;
    WalkState w[ILP];
    uint32_t next = q0;  // wave-uniform: first query of the chunk not yet started
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
        const uint32_t q = next + (uint32_t)i * 64u + lane;
        w[i].q = kIdleQ;  // idle: column 0 of row 0 stays loadable
        w[i].cur = 0;
        w[i].t = 0;
        w[i].hops = 0;
        w[i].bad = false;
        w[i].cost = 0;
        w[i].pos = 0;
        w[i].R = 0;
        w[i].row = rows_base(rows);
        if (q < q1) walk_begin(w[i], q, qs, qt, qrow, rows);
    }
    next = min(q1, next + 64u * ILP);
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    for (;;) {
        // retire finished walks; their lanes take the next queries of the chunk
        bool live = false;
#pragma unroll
        for (int i = 0; i < ILP; ++i) {
            const bool idle = w[i].q == kIdleQ;
            const bool done = !idle && (w[i].cur == w[i].t || w[i].hops >= limit || w[i].bad);
            const uint64_t m = __ballot(done);
            if (m) {
                if (done) {
                    const uint32_t fin = w[i].cur == w[i].t ? 1u : 0u;
                    cost_out[w[i].q] = w[i].cost;
                    hops_out[w[i].q] = w[i].hops;
                    fin_out[w[i].q] = (uint8_t)fin;
                    sum_cost += w[i].cost;
                    sum_hops += w[i].hops;
                    sum_fin += fin;
                    const uint32_t nqi = next + (uint32_t)__builtin_popcountll(m & lt_mask);
                    if (nqi < q1) walk_begin(w[i], nqi, qs, qt, qrow, rows);
                    else w[i].q = kIdleQ;
                }
                next = min(q1, next + (uint32_t)__builtin_popcountll(m));
            }
            live |= w[i].q != kIdleQ;
        }
        if (!__any(live)) break;
        walk_hops<SHIFT, ILP>(w, adj, rows);  // one hop of every walking slot
    }
    wave_stats(sum_cost, sum_hops, sum_fin, agg);
}

__device__ void wave_stats(uint64_t cost, uint32_t hops, uint32_t fin,
                           unsigned long long* __restrict__ agg) {
    // wave reduction, one atomic per wave per counter
    unsigned long long c = cost, h = hops, f = fin;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        c += __shfl_xor(c, off, 64);
        h += __shfl_xor(h, off, 64);
        f += __shfl_xor(f, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&agg[0], f);
        atomicAdd(&agg[1], h);
        atomicAdd(&agg[2], c);
    }
}

// ---------------------------------------------------------------------------
// CPD-heuristic search (semantics restated in
// oracle/cpd_oracle.c ora_cpd_search, [U]).
//
// One lane per query, lanes refilled from the wave's chunk of the
// target-sorted batch (as table_walk).  Each lane slot owns a workspace in
// HBM: an open-addressing hash of the columns met (2C slots, at most C used),
// a binary heap of C entries keyed (f, column, g) — the oracle's order — and
// a walk stack of C entries.  A hash entry is
//   Ent {tag, column, g lo, g hi}       tag = query + 1; g = INF: not (yet) in
//                                       the search (only walked)
//   Memo {hf lo, hf hi, cw lo, cw hi}   the CPD path from the column to t:
//                                       free-flow cost, cost under the
//                                       selected weights (INF: no path)
//   Aux {depth, lw | state << 30}       search depth; the path's moves; state
//                                       1 = walked, 2 = on the current walk
// The heuristic and incumbent values come from memoised CPD walks over the
// dense move row of t (the oracle's ora_walk): a walk follows moves until it
// meets a walked column (or t, walked with zeros), then assigns every column
// it passed its suffix cost, popping the walk stack; meeting a column of the
// current walk again (a zero-weight cycle) or a move that names no edge gives
// the whole walk INF.  Nothing is precomputed per row, so an index of any
// size can be searched (round 2 kept 20 B per column per row of tables).
// A search whose columns (walked or searched) outgrow C stops unfinished and
// is counted in agg[7] (overflow) — never silently wrong.
// Time limit (process_query.py:149-160 `time`, ns): checked with the stop
// conditions at every pop; elapsed = wall clock since the search began
// (s_memrealtime, 100 MHz) or, with a virtual tick (tests), tick x (expanded
// + touched) so far — the oracle's deterministic restatement.
constexpr uint64_t kInf64 = 0xFFFFFFFFFFFFFFFFull;
constexpr uint32_t kOnWalk = 2u, kWalked = 1u;

// Per-row tables (the TABLES form of the search): per index row r (target
// t), over the columns, computed from the dense move table by pointer
// jumping over the CPD's next-hop tree — the CPD walk from every column at
// once, in log2(n) + 1 doubling rounds:
//   hrow[r][c] = free-flow cost of the CPD path c -> t (the heuristic),
//   crow[r][c] = its cost under the selected weights (the incumbent bound),
//   lrow[r][c] = its moves;  INF (hrow, crow) when the walk never reaches t.
// Jump state per (row, column): next column (kJumpBad = no path), cf, cw,
// lw; t points to itself with zero cost (absorbing).
constexpr uint32_t kJumpBad = 0xFFFFFFFFu;

struct JumpState {
    uint32_t* next;
    uint64_t* cf;
    uint64_t* cw;
    uint32_t* lw;
};

__global__ __launch_bounds__(256) void jump_init(const uint32_t* __restrict__ dense,
                                                 uint32_t wpr, Tbl tbl, const uint2* __restrict__ adj_f,
                                                 const uint2* __restrict__ adj_w, uint32_t shift,
                                                 const uint32_t* __restrict__ tcol, uint32_t rows,
                                                 uint32_t n, JumpState js) {
    const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (j >= (uint64_t)rows * n) return;
    const uint32_t r = (uint32_t)(j / n), c = (uint32_t)(j - (uint64_t)r * n);
    uint32_t nx = kJumpBad, l = 0;
    uint64_t f = 0, w = 0;
    if (c == tcol[r]) {
        nx = c;
    } else {
        const uint32_t mv = tbl.move(dense + (size_t)r * wpr, c);
        if (!(mv >> shift)) {
            const size_t e = ((size_t)c << shift) + mv;
            const uint2 ef = adj_f[e];
            if (ef.x != kNoEdge) {
                nx = ef.x;
                f = ef.y;
                w = adj_w[e].y;
                l = 1;
            }
        }
    }
    js.next[j] = nx;
    js.cf[j] = f;
    js.cw[j] = w;
    js.lw[j] = l;
}

// One doubling round a -> b: b(c) = a(c) followed by a(next(c)).
__global__ __launch_bounds__(256) void jump_round(JumpState a, JumpState b,
                                                  const uint32_t* __restrict__ tcol, uint32_t rows,
                                                  uint32_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (j >= (uint64_t)rows * n) return;
    const uint32_t r = (uint32_t)(j / n);
    const uint32_t nx = a.next[j];
    uint32_t o = nx;
    uint64_t f = a.cf[j], w = a.cw[j];
    uint32_t l = a.lw[j];
    if (nx != kJumpBad && nx != tcol[r]) {
        const uint64_t k = (uint64_t)r * n + nx;
        o = a.next[k];
        if (o != kJumpBad) {
            f += a.cf[k];
            w += a.cw[k];
            l += a.lw[k];
        }
    }
    b.next[j] = o;
    b.cf[j] = f;
    b.cw[j] = w;
    b.lw[j] = l;
}

__global__ __launch_bounds__(256) void jump_final(JumpState a, const uint32_t* __restrict__ tcol,
                                                  uint32_t rows, uint32_t n,
                                                  uint64_t* __restrict__ hrow,
                                                  uint64_t* __restrict__ crow,
                                                  uint32_t* __restrict__ lrow, int write_h) {
    const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (j >= (uint64_t)rows * n) return;
    const uint32_t r = (uint32_t)(j / n);
    const bool ok = a.next[j] == tcol[r];
    if (write_h) hrow[j] = ok ? a.cf[j] : kInf64;
    crow[j] = ok ? a.cw[j] : kInf64;
    lrow[j] = ok ? a.lw[j] : 0u;
}


struct SearchWs {
    uint32_t cap;   // C (power of 2)
    // slot s's arrays lie together in one block at base + s * stride: the
    // heap (C + K entries: f lo, f hi, column, hash slot), ent and aux (2C
    // each), then with walks memo (2C) and the walk stack (C: hash slot, w
    // free, w selected, -) — a search touches one contiguous region of a few
    // MB, not six spread over the workspace (array-major blocks measured
    // 1-5% slower in round 5 and were removed in round 6)
    char* base;
    uint64_t stride;
    uint32_t lpw;  // lanes per wave that search (64 / 32 / 16 / 8)
};

struct SearchOpt {
    double hscale, fscale;
    int32_t kmoves;
    int64_t itrs;
    uint64_t time_ns;     // 0 = none
    uint64_t tick_ns;     // 0 = wall clock, else the virtual clock's tick
};

__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) {
    return ((uint64_t)hi << 32) | lo;
}

// Hash probe: slot of column c (found = true) or the free slot to insert it
// in (2C slots, at most C used: probes end).
__device__ __forceinline__ uint32_t hprobe(const uint4* __restrict__ ent, uint32_t mask,
                                           uint32_t tag, uint32_t c, bool& found) {
    uint32_t i = (c * 0x9E3779B1u) & mask;
    for (;;) {
        const uint4 e = ent[i];
        if (e.x != tag) {
            found = false;
            return i;
        }
        if (e.y == c) {
            found = true;
            return i;
        }
        i = (i + 1u) & mask;
    }
}

// hprobe with the first slot's entry already loaded (e = ent[hash(c)]); the
// slot found is returned with its entry in e
__device__ __forceinline__ uint32_t hprobe_from(const uint4* __restrict__ ent, uint32_t mask,
                                                uint32_t tag, uint32_t c, bool& found, uint4& e) {
    uint32_t i = (c * 0x9E3779B1u) & mask;
    for (;;) {
        if (e.x != tag) {
            found = false;
            return i;
        }
        if (e.y == c) {
            found = true;
            return i;
        }
        i = (i + 1u) & mask;
        e = ent[i];
    }
}

// The search heap: kHeapK-ary (children of i at K i + 1 .. K i + K), so a
// pop descends log_K of the size in levels whose K child loads go out
// together — a binary heap's dependent round trips / log2 K.  An entry is
// one 16-B word, (f lo, f hi, column, hash slot of the column): the slot
// rides with the entry, so a pop finds its column's hash entry without
// probing (slots never move within a search; a resumed search's are probed
// again once).  The array starts K - 1 entries into its block (128-B
// aligned), so the K children of every entry are one aligned 128-B line.
// The oracle orders its heap by (f, column, g); g is implied by (f,
// column): f = g + h(column) with h fixed per column, and a column is pushed
// again only with a strictly smaller g — so (f, column) is a total order
// over the entries a search holds, its pops (and every counter) those of the
// oracle's binary heap, and a popped entry is stale exactly when its f
// exceeds the column's current g + h.
constexpr uint32_t kHeapK = 8;

__device__ __forceinline__ uint64_t hkey_f(const uint4& e) { return u64of(e.x, e.y); }

// (f, column) lexicographic, without branches (the heap loops compare eight
// children at once; short-circuit forms compiled to a branch each)
__device__ __forceinline__ bool hkey_less(const uint4& a, const uint4& b) {
    const uint64_t fa = hkey_f(a), fb = hkey_f(b);
    return (fa < fb) | ((fa == fb) & (a.z < b.z));
}

__device__ __forceinline__ uint4 hkey_make(uint64_t f, uint32_t col, uint32_t slot) {
    return make_uint4((uint32_t)f, (uint32_t)(f >> 32), col, slot);
}

// component-wise select (a select of whole vectors became a select of their
// addresses, which put the children arrays in scratch)
__device__ __forceinline__ uint4 sel4(bool t, const uint4& a, const uint4& b) {
    return make_uint4(t ? a.x : b.x, t ? a.y : b.y, t ? a.z : b.z, t ? a.w : b.w);
}

__device__ __forceinline__ void heap_push(uint4* __restrict__ hk, uint32_t& size, const uint4 e) {
    uint32_t i = size++;
    while (i) {
        const uint32_t p = (i - 1u) / kHeapK;
        const uint4 pe = hk[p];
        if (!hkey_less(e, pe)) break;
        hk[i] = pe;
        i = p;
    }
    hk[i] = e;
}

// The pop, in two steps so that its descent starts one round trip early.
// heap_pick (the caller, with the root's children and the last entry in
// registers, before the pop is decided): the root's least live child (be at
// position bk; nk live children) and that child's own children group
// loaded (e2: nc2 live) — beside the expansion's other loads.  heap_pop_pre
// then moves the last entry down from the root with no load for its first
// two levels.
struct HeapPick {
    uint4 be;
    uint32_t bk, nk, nc2;
};

__device__ __forceinline__ HeapPick heap_pick(const uint4* __restrict__ hk, uint32_t size,
                                              const uint4 (&e1)[kHeapK], uint4 (&e2)[kHeapK]) {
    HeapPick p;
    const uint32_t sz = size - 1u;  // after the pop
    p.nk = sz ? min(kHeapK, sz - 1u) : 0u;  // live children of the root (< sz)
    p.be = e1[0];
    p.bk = 1;
#pragma unroll
    for (uint32_t j = 1; j < kHeapK; ++j) {
        const bool t = (j < p.nk) & hkey_less(e1[j], p.be);
        p.be = sel4(t, e1[j], p.be);
        p.bk = t ? 1u + j : p.bk;
    }
    const uint32_t k0 = kHeapK * p.bk + 1u;
    p.nc2 = (p.nk && k0 < sz) ? min(kHeapK, sz - k0) : 0u;
    if (p.nc2) {  // the whole group: in bounds (k0 < size, the array is C + K long)
#pragma unroll
        for (uint32_t j = 0; j < kHeapK; ++j) e2[j] = hk[k0 + j];
    }
    return p;
}

__device__ __forceinline__ void heap_pop_pre(uint4* __restrict__ hk, uint32_t& size,
                                             const HeapPick& p, const uint4 (&e2)[kHeapK],
                                             const uint4 le) {
    --size;
    if (!size) return;
    if (!p.nk || !hkey_less(p.be, le)) {
        hk[0] = le;
        return;
    }
    hk[0] = p.be;
    uint32_t i = p.bk;
    if (p.nc2) {  // the second level from registers
        const uint32_t k0 = kHeapK * i + 1u;
        uint4 ce = e2[0];
        uint32_t ck = k0;
#pragma unroll
        for (uint32_t j = 1; j < kHeapK; ++j) {
            const bool t = (j < p.nc2) & hkey_less(e2[j], ce);
            ce = sel4(t, e2[j], ce);
            ck = t ? k0 + j : ck;
        }
        if (hkey_less(ce, le)) {
            hk[i] = ce;
            i = ck;
            for (;;) {
                const uint32_t k1 = kHeapK * i + 1u;
                if (k1 >= size) break;
                const uint32_t nc = min(kHeapK, size - k1);
                uint4 e[kHeapK];
#pragma unroll
                for (uint32_t j = 0; j < kHeapK; ++j) e[j] = hk[k1 + j];  // in bounds (k1 < size)
                uint4 me = e[0];
                uint32_t mk = k1;
#pragma unroll
                for (uint32_t j = 1; j < kHeapK; ++j) {
                    const bool t = (j < nc) & hkey_less(e[j], me);
                    me = sel4(t, e[j], me);
                    mk = t ? k1 + j : mk;
                }
                if (!hkey_less(me, le)) break;
                hk[i] = me;
                i = mk;
            }
        }
    }
    hk[i] = le;
}

// The expansion's pushes (one per out-edge at most, `valid`), their parents
// loaded together: a new entry no less than its parent stays where it lands
// (the rule in A* with a consistent heuristic: children's f are no smaller);
// the first that must rise goes through heap_push, and so do the ones after
// it (their parents may have moved).  The heap ends as valid as pushing one
// by one, and pops depend only on the keys.
template <int N>
__device__ __forceinline__ void heap_push_n(uint4* __restrict__ hk, uint32_t& size,
                                            const bool (&valid)[N], const uint4 (&e)[N]) {
    const uint32_t s0 = size;
    uint4 pe[N];
    uint32_t at = s0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (valid[k]) {
            const uint32_t p = at ? (at - 1u) / kHeapK : 0u;
            if (at && p < s0) pe[k] = hk[p];
            ++at;
        }
    }
    bool slow = false;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (!valid[k]) continue;
        const uint32_t i = size;
        const uint32_t p = i ? (i - 1u) / kHeapK : 0u;
        if (!slow && (i == 0 || (p < s0 && !hkey_less(e[k], pe[k])))) {
            hk[i] = e[k];
            ++size;
        } else {
            slow = true;
            heap_push(hk, size, e[k]);
        }
    }
}

struct Lane {
    uint32_t q, s, t, tag, hsize, used, best_len;
    uint64_t ub, t0;
    uint32_t expanded, inserted, touched, updated, surplus;
    bool done, overflow, spilled;
};

// Resumable overflow.  A search checks, before each
// pop, that the expansion cannot outgrow its workspace: at most 2^SHIFT new
// columns and heap entries (the tables form), or — the walks form, whose
// walks add any number — the heads' walks done first and the heap's room.
// When it could, the search stops there with its state whole and, given a
// spill pool, copies it out as a record: the heap verbatim, then every
// column it holds (column, g, depth, moves | state, and with walks the memo)
// — ~20-36 B per column, not the 72-120 B per column of capacity a
// workspace costs.  The next pass (4x the capacity) rebuilds the hash from
// the record and continues from the same pop: the heap keys (f, column, g)
// are a total order, so pops, counters and results are those of one
// uninterrupted search.  Record (u32 words): hsize, used, ub lo/hi,
// best_len, the five counters, elapsed ticks lo/hi, entries, 0 | heap
// hsize x (f lo, f hi, column) | entries x (column, g lo, g hi, depth,
// moves | state [, memo x4]).
struct SearchSpill {
    const unsigned long long* resume;  // [nq] record of query q in rin, ~0 = fresh (null: all)
    const uint32_t* rin;
    unsigned long long* at;            // [nq] record written for a spilled query (fin 3)
    uint32_t* rout;                    // the pool records go to (null: no spilling)
    unsigned long long* top;           // its bump counter, words
    unsigned long long cap;            // its size, words
};
constexpr uint32_t kSpillHead = 14;

// The lane's workspace (one slot's arrays).
struct LaneWs {
    uint4* __restrict__ ent;
    uint4* __restrict__ memo;
    uint2* __restrict__ aux;
    uint4* __restrict__ hk;
    uint4* __restrict__ stk;
    uint32_t C, mask;
    Tbl tb;  // the move tables' bits per column
};

// Insert column c (absent: slot i from hprobe) as walked-only; false on
// overflow (more than C columns).
__device__ __forceinline__ bool ws_insert(Lane& L, const LaneWs& W, uint32_t i, uint32_t c,
                                          uint32_t state) {
    if (L.used >= W.C) return false;
    ++L.used;
    W.ent[i] = make_uint4(L.tag, c, 0xFFFFFFFFu, 0xFFFFFFFFu);
    W.aux[i] = make_uint2(0u, state << 30);
    return true;
}

// A walk that overflowed: the columns it marked "on the walk" (the stack and
// the column in hand) go back to "not walked", so the search's state stays
// whole — it is spilled and resumed, or restarted, from there.
__device__ __forceinline__ void walk_abandon(const LaneWs& W, uint32_t sp, uint32_t xi) {
    W.aux[xi].y &= 0x3FFFFFFFu;
    for (uint32_t j = 0; j < sp; ++j) W.aux[W.stk[j].x].y &= 0x3FFFFFFFu;
}

// Memoised CPD walk from column v (ora_walk): afterwards v's entry (returned
// slot) is walked; false on overflow (walk_abandon: nothing half-walked).
template <int SHIFT>
__device__ bool cpd_walk(Lane& L, const LaneWs& W, const uint2* __restrict__ adj_f,
                         const uint2* __restrict__ adj_w, const uint32_t* __restrict__ row,
                         uint32_t v, uint32_t& vslot) {
    bool found;
    uint32_t i = hprobe(W.ent, W.mask, L.tag, v, found);
    if (found && (W.aux[i].y >> 30) == kWalked) {
        vslot = i;
        return true;
    }
    if (!found && !ws_insert(L, W, i, v, 0u)) return false;
    vslot = i;
    uint32_t sp = 0, x = v, xi = i;
    bool bad = false;
    // per step, everything that depends only on the column x — its first
    // hash slot (entry and aux), its move word and its adjacency rows — is
    // loaded together: one round trip per step when the probe hits at once
    uint32_t auy = W.aux[xi].y;
    for (;;) {
        const uint32_t st = auy >> 30;
        if (st == kWalked) break;
        if (st == kOnWalk) {  // a cycle: no path to t
            bad = true;
            break;
        }
        W.aux[xi].y = (auy & 0x3FFFFFFFu) | (kOnWalk << 30);
        uint2 ef = make_uint2(kNoEdge, 0u), ew = make_uint2(kNoEdge, 0u);
        if (SHIFT <= 2) {
            constexpr int ND = 1 << (SHIFT <= 2 ? SHIFT : 0);
            uint2 af[ND], aw[ND];
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                af[k] = adj_f[((size_t)x << SHIFT) + k];
                aw[k] = adj_w[((size_t)x << SHIFT) + k];
            }
            const uint32_t mv = W.tb.move(row, x);
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                if (mv == (uint32_t)k) {
                    ef = af[k];
                    ew = aw[k];
                }
            }
        } else {
            const uint32_t mv = W.tb.move(row, x);
            if (!(mv >> SHIFT)) {
                ef = adj_f[((size_t)x << SHIFT) + mv];
                ew = adj_w[((size_t)x << SHIFT) + mv];
            }
        }
        if (sp >= W.C) {
            walk_abandon(W, sp, xi);
            return false;
        }
        W.stk[sp++] = make_uint4(xi, ef.y, ew.y, 0u);
        if (ef.x == kNoEdge) {  // names no edge of x
            bad = true;
            break;
        }
        x = ef.x;
        const uint32_t h = (x * 0x9E3779B1u) & W.mask;
        uint4 e = W.ent[h];
        const uint2 au = W.aux[h];
        xi = hprobe_from(W.ent, W.mask, L.tag, x, found, e);
        if (!found) {
            if (!ws_insert(L, W, xi, x, 0u)) {
                walk_abandon(W, sp, W.stk[sp - 1u].x);  // sp >= 1: the column just left
                return false;
            }
            auy = 0u;  // what ws_insert wrote: not walked
        } else {
            auy = xi == h ? au.y : W.aux[xi].y;
        }
    }
    uint64_t hf = kInf64, cw = kInf64;
    uint32_t lw = 0;
    if (!bad) {
        const uint4 m = W.memo[xi];
        hf = u64of(m.x, m.y);
        cw = u64of(m.z, m.w);
        lw = W.aux[xi].y & 0x3FFFFFFFu;
    }
    while (sp) {
        const uint4 e = W.stk[--sp];
        if (hf != kInf64) {
            hf += e.y;
            cw += e.z;
            lw += 1u;
        }
        W.memo[e.x] = make_uint4((uint32_t)hf, (uint32_t)(hf >> 32), (uint32_t)cw,
                                 (uint32_t)(cw >> 32));
        W.aux[e.x].y = (hf == kInf64 ? 0u : lw) | (kWalked << 30);
    }
    return true;
}

// h = (uint64_t)(hscale * (double)hu), the oracle's expression; with hscale
// 1 (a kernel-uniform test) and hu < 2^53 it is hu exactly, and the double
// conversions (~25 instructions a push) are skipped
__device__ __forceinline__ uint64_t hval(const SearchOpt& opt, uint64_t hu) {
    if (opt.hscale == 1.0 && hu < (1ull << 53)) return hu;
    return (uint64_t)(opt.hscale * (double)hu);
}

// the stop rule (double)f * (1 + fscale) >= (double)ub; at fscale 0 with
// both below 2^53 (or ub INF) the integer compare is the same
__device__ __forceinline__ bool f_stops(const SearchOpt& opt, uint64_t f, uint64_t ub) {
    if (opt.fscale == 0.0 && f < (1ull << 53) && (ub < (1ull << 53) || ub == kInf64))
        return f >= ub;
    return (double)f * (1.0 + opt.fscale) >= (double)ub;
}

// TABLES: the CPD path values come from the per-row tables (hrow / crow /
// lrow, n per row) instead of memoised walks; the workspace then holds only
// the searched columns (no memo, no walk stack).  Same results and counters.
struct SearchTables {
    const uint64_t* hrow;
    const uint64_t* crow;
    const uint32_t* lrow;
    uint32_t n;
};

template <int SHIFT, bool TABLES>
// (one wave per SIMD: the register budget of 512 leaves the children arrays in
// registers; 1024 one-wave workgroups fill the 1024 SIMDs)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void cpd_search(
    const uint2* __restrict__ adj_f, const uint2* __restrict__ adj_w,
    const uint32_t* __restrict__ dense, uint32_t wpr, uint32_t lb, SearchTables tb,
    const uint32_t* __restrict__ qs,
    const uint32_t* __restrict__ qt, const uint32_t* __restrict__ qrow, uint32_t nq,
    uint32_t chunk, SearchOpt opt, SearchWs ws, SearchSpill sp, uint64_t* __restrict__ cost_out,
    uint32_t* __restrict__ plen_out, uint8_t* __restrict__ fin_out,
    uint32_t* __restrict__ qstats, unsigned long long* __restrict__ agg) {
    constexpr uint32_t KD = 1u << SHIFT;  // most new columns / heap entries of one expansion
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    // ws.lpw lanes per wave search (64, or fewer when few searches are left:
    // more waves, each issuing for fewer divergent lanes); the others idle
    const uint32_t lpw = ws.lpw;
    const bool active = lane < lpw;
    const uint64_t slot = wave * lpw + (active ? lane : 0u);  // this lane's workspace
    const uint64_t q0l = wave * chunk;
    const uint32_t q0 = q0l < nq ? (uint32_t)q0l : nq;
    const uint32_t q1 = (uint32_t)min((uint64_t)nq, q0l + chunk);
    const uint32_t C = ws.cap;
    // the slot's block = the heap (C + K entries), ent, aux, then memo and
    // stk with walks.  The heap pointer starts K - 1 entries in (aligned
    // child groups).
    char* const lb0 = ws.base + slot * ws.stride;
    const uint64_t C2 = 2ull * C, CH = (uint64_t)C + kHeapK;
    const LaneWs W{reinterpret_cast<uint4*>(lb0 + CH * 16ull),
                   TABLES ? nullptr : reinterpret_cast<uint4*>(lb0 + CH * 16ull + C2 * 24ull),
                   reinterpret_cast<uint2*>(lb0 + CH * 16ull + C2 * 16ull),
                   reinterpret_cast<uint4*>(lb0) + (kHeapK - 1u),
                   TABLES ? nullptr : reinterpret_cast<uint4*>(lb0 + CH * 16ull + C2 * 40ull), C,
                   2u * C - 1u, Tbl{lb}};
    unsigned long long s_exp = 0, s_ins = 0, s_tou = 0, s_upd = 0, s_sur = 0, s_len = 0,
                       s_fin = 0, s_ovf = 0;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    // tag = query index + 1 of the search that wrote a slot; cleared once per
    // launch so stale tags never match
    if (active)
        for (uint32_t i = 0; i < 2u * C; ++i) W.ent[i] = make_uint4(0u, 0u, 0u, 0u);

    Lane L;
    L.q = kIdleQ;
    L.done = false;
    const uint32_t* row = dense;
    size_t rb = 0;  // TABLES: the query row's first table entry
    auto begin = [&](uint32_t q) {
        L.q = q;
        L.s = qs[q];
        L.t = qt[q];
        L.tag = q + 1u;
        L.hsize = 0;
        L.used = 0;
        L.ub = kInf64;
        L.best_len = 0;
        L.expanded = L.inserted = L.touched = L.updated = L.surplus = 0;
        L.done = false;
        L.overflow = false;
        L.spilled = false;
        L.t0 = __builtin_amdgcn_s_memrealtime();
        row = dense + (size_t)qrow[q] * wpr;
        rb = (size_t)qrow[q] * tb.n;
        if (sp.resume && sp.resume[q] != ~0ull) {  // a spilled search: its state back
            const uint32_t* __restrict__ r = sp.rin + sp.resume[q];
            L.hsize = r[0];
            L.used = r[1];
            L.ub = u64of(r[2], r[3]);
            L.best_len = r[4];
            L.expanded = r[5];
            L.inserted = r[6];
            L.touched = r[7];
            L.updated = r[8];
            L.surplus = r[9];
            L.t0 -= u64of(r[10], r[11]);
            const uint32_t ne = r[12];
            const uint32_t* __restrict__ h = r + kSpillHead;
            constexpr uint32_t per = TABLES ? 5u : 9u;
            const uint32_t* __restrict__ en = h + 3ull * L.hsize;
            for (uint32_t k = 0; k < ne; ++k) {
                const uint32_t* __restrict__ o = en + (size_t)per * k;
                bool f;
                const uint32_t i = hprobe(W.ent, W.mask, L.tag, o[0], f);
                W.ent[i] = make_uint4(L.tag, o[0], o[1], o[2]);
                W.aux[i] = make_uint2(o[3], o[4]);
                if (!TABLES) W.memo[i] = make_uint4(o[5], o[6], o[7], o[8]);
            }
            // the heap after the hash: its entries' slots in this workspace
            for (uint32_t i = 0; i < L.hsize; ++i) {
                bool f;
                const uint32_t c = h[3u * i + 2u];
                W.hk[i] = make_uint4(h[3u * i], h[3u * i + 1u], c, hprobe(W.ent, W.mask, L.tag, c, f));
            }
            return;
        }
        bool found;
        uint32_t si;
        uint64_t hs;
        if (TABLES) {
            hs = tb.hrow[rb + L.s];
            si = hprobe(W.ent, W.mask, L.tag, L.s, found);
            if (hs != kInf64) ws_insert(L, W, si, L.s, 0u);
        } else {  // t walked with zeros, then the walk from s
            const uint32_t ti = hprobe(W.ent, W.mask, L.tag, L.t, found);
            ws_insert(L, W, ti, L.t, kWalked);
            W.memo[ti] = make_uint4(0u, 0u, 0u, 0u);
            if (!cpd_walk<SHIFT>(L, W, adj_f, adj_w, row, L.s, si)) {
                L.overflow = L.done = true;
                return;
            }
            const uint4 m = W.memo[si];
            hs = u64of(m.x, m.y);
        }
        if (hs != kInf64) {
            W.ent[si].z = 0u;
            W.ent[si].w = 0u;
            W.aux[si].x = 0u;
            L.inserted = 1;
            heap_push(W.hk, L.hsize, hkey_make(hval(opt, hs), L.s, si));
        }
    };
    // a search stopped before a pop that could outgrow the workspace: its
    // record into the spill pool (false: no pool, or the pool is full — the
    // search then restarts from scratch at the next capacity)
    auto spill = [&]() -> bool {
        if (!sp.rout) return false;
        constexpr uint32_t per = TABLES ? 5u : 9u;
        const unsigned long long words =
            kSpillHead + 3ull * L.hsize + (unsigned long long)per * L.used;
        const unsigned long long off = atomicAdd(sp.top, words);
        if (off + words > sp.cap) return false;
        uint32_t* __restrict__ r = sp.rout + off;
        uint32_t* __restrict__ h = r + kSpillHead;
        for (uint32_t i = 0; i < L.hsize; ++i) {
            const uint4 e = W.hk[i];
            h[3u * i] = e.x;
            h[3u * i + 1u] = e.y;
            h[3u * i + 2u] = e.z;
        }
        uint32_t* __restrict__ en = h + 3ull * L.hsize;
        uint32_t k = 0;
        for (uint32_t i = 0; i < 2u * C && k < L.used; ++i) {
            const uint4 e = W.ent[i];
            if (e.x != L.tag) continue;
            const uint2 a = W.aux[i];
            uint32_t* __restrict__ o = en + (size_t)per * k++;
            o[0] = e.y;
            o[1] = e.z;
            o[2] = e.w;
            o[3] = a.x;
            o[4] = a.y;
            if (!TABLES) {
                const uint4 mm = W.memo[i];
                o[5] = mm.x;
                o[6] = mm.y;
                o[7] = mm.z;
                o[8] = mm.w;
            }
        }
        const uint64_t el = __builtin_amdgcn_s_memrealtime() - L.t0;
        r[0] = L.hsize;
        r[1] = L.used;
        r[2] = (uint32_t)L.ub;
        r[3] = (uint32_t)(L.ub >> 32);
        r[4] = L.best_len;
        r[5] = L.expanded;
        r[6] = L.inserted;
        r[7] = L.touched;
        r[8] = L.updated;
        r[9] = L.surplus;
        r[10] = (uint32_t)el;
        r[11] = (uint32_t)(el >> 32);
        r[12] = k;
        r[13] = 0u;
        sp.at[L.q] = off;
        return true;
    };
    uint32_t next = q0;
    // the first round hands every searching lane its first query through the
    // refill below: one call site of begin() (which holds a walk and the
    // resume loops), not two
    bool want = active;
    for (;;) {
        // retire finished searches, refill from the chunk
        const bool fin_now = L.q != kIdleQ && (L.done || L.hsize == 0);
        const bool take = fin_now || want;
        const uint64_t m = __ballot(take);
        want = false;
        if (m) {
            if (fin_now) {
                const bool found = L.ub != kInf64 && !L.overflow;
                cost_out[L.q] = found ? L.ub : 0ull;
                plen_out[L.q] = found ? L.best_len : 0u;
                // 2: stopped on the workspace (restarts), 3: spilled (resumes)
                fin_out[L.q] = found ? 1u : L.overflow ? (L.spilled ? 3u : 2u) : 0u;
                uint32_t* st = qstats + 5ull * L.q;
                st[0] = L.expanded;
                st[1] = L.inserted;
                st[2] = L.touched;
                st[3] = L.updated;
                st[4] = L.surplus;
                // a spilled search's counters are summed when it completes
                const uint32_t keep = L.spilled ? 0u : 1u;
                s_exp += keep * L.expanded;
                s_ins += keep * L.inserted;
                s_tou += keep * L.touched;
                s_upd += keep * L.updated;
                s_sur += keep * L.surplus;
                s_len += found ? L.best_len : 0u;
                s_fin += found ? 1u : 0u;
                s_ovf += L.overflow ? 1u : 0u;
            }
            if (take) {
                const uint32_t nqi = next + (uint32_t)__builtin_popcountll(m & lt_mask);
                if (nqi < q1) begin(nqi);
                else L.q = kIdleQ;
            }
            next = min(q1, next + (uint32_t)__builtin_popcountll(m));
        }
        if (!__any(L.q != kIdleQ)) break;
        if (L.q == kIdleQ || L.done || L.hsize == 0) continue;
        // one pop of this lane's search: the top, looked at first (it is
        // popped once the expansion is known to fit the workspace)
        uint64_t f;
        uint32_t v, hi;
        uint4 e1[kHeapK], lst;  // the root's children and the last entry (heap_pick)
        {
            const uint4 top = W.hk[0];
            f = hkey_f(top);
            v = top.z;
            hi = top.w;  // v's hash slot
#pragma unroll
            for (uint32_t j = 0; j < kHeapK; ++j) e1[j] = W.hk[1u + j];  // positions 1..K: in bounds
            lst = W.hk[L.hsize - 1u];
        }
        // what the expansion reads and nothing in it writes — v's out-edges,
        // its hash entry and, per-row tables, its incumbent values — is
        // loaded together, one round trip for all of it
        constexpr int ND = SHIFT <= 2 ? (1 << SHIFT) : 1;
        uint2 ed[ND];
        if (SHIFT <= 2) {
#pragma unroll
            for (int k = 0; k < ND; ++k) ed[k] = adj_w[((size_t)v << SHIFT) + k];
        }
        uint64_t cw_t = 0, hv;
        uint32_t lw_t = 0;
        if (TABLES) {
            cw_t = tb.crow[rb + v];
            lw_t = tb.lrow[rb + v];
            hv = tb.hrow[rb + v];
        } else {
            const uint4 mv = W.memo[hi];  // walked when it was inserted
            hv = u64of(mv.x, mv.y);
        }
        const uint4 ev = W.ent[hi];
        const uint2 av = W.aux[hi];
        uint4 e2[kHeapK];  // the pop's second level (heap_pick)
        const HeapPick hp = heap_pick(W.hk, L.hsize, e1, e2);
        // the entry's g is the column's current one unless the entry is
        // stale (its f above current g + h: a better g came later)
        const uint64_t g = u64of(ev.z, ev.w);
        if (f > g + hval(opt, hv)) {  // stale entry
            heap_pop_pre(W.hk, L.hsize, hp, e2, lst);
            ++L.surplus;
            continue;
        }
        const uint64_t elapsed =
            opt.tick_ns ? opt.tick_ns * ((uint64_t)L.expanded + L.touched)
                        : 10ull * (__builtin_amdgcn_s_memrealtime() - L.t0);
        if (f_stops(opt, f, L.ub) ||
            (opt.itrs >= 0 && (int64_t)L.expanded >= opt.itrs) ||
            (opt.time_ns && elapsed > opt.time_ns)) {
            L.done = true;
            continue;
        }
        // room for the expansion: <= KD heap entries (and, tables, columns);
        // with walks the heads are walked first (the expansion would walk
        // exactly these; their memo does not depend on the search)
        bool room = L.hsize - 1u + KD <= C && (!TABLES || L.used + KD <= C);
        if (room && !TABLES) {
            if (SHIFT <= 2) {
                // one walk call site, not one per unrolled edge (the walk is
                // large): the heads picked by index from registers
#pragma unroll 1
                for (int k = 0; k < ND && room; ++k) {
                    uint32_t u = ed[0].x;
#pragma unroll
                    for (int j = 1; j < ND; ++j) u = k == j ? ed[j].x : u;
                    if (u == kNoEdge) break;  // edges are packed first
                    uint32_t ui;
                    room = cpd_walk<SHIFT>(L, W, adj_f, adj_w, row, u, ui);
                }
            } else {
#pragma unroll 1
                for (uint32_t k = 0; k < KD && room; ++k) {
                    const uint32_t u = adj_w[((size_t)v << SHIFT) + k].x;
                    if (u == kNoEdge) break;
                    uint32_t ui;
                    room = cpd_walk<SHIFT>(L, W, adj_f, adj_w, row, u, ui);
                }
            }
        }
        if (!room) {  // stop whole, before the pop: spilled, or restarted
            L.overflow = L.done = true;
            L.spilled = spill();
            continue;
        }
        // the heads' first hash slots and (per-row tables) heuristics,
        // issued with the pop's descent: they arrive together
        uint4 e0[ND];
        uint64_t hr[ND];
        if (SHIFT <= 2) {
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                if (TABLES && ed[k].x != kNoEdge) {
                    e0[k] = W.ent[(ed[k].x * 0x9E3779B1u) & W.mask];
                    hr[k] = tb.hrow[rb + ed[k].x];
                } else if (ed[k].x != kNoEdge) {
                    e0[k] = W.ent[(ed[k].x * 0x9E3779B1u) & W.mask];
                }
            }
        }
        heap_pop_pre(W.hk, L.hsize, hp, e2, lst);
        ++L.expanded;
        const uint32_t dv = av.x;
        {
            uint64_t cw;
            uint32_t lw;
            if (TABLES) {
                cw = cw_t;
                lw = lw_t;
            } else {
                const uint4 mv = W.memo[hi];
                cw = u64of(mv.z, mv.w);
                lw = W.aux[hi].y & 0x3FFFFFFFu;
            }
            if (cw != kInf64 && (opt.kmoves < 0 || lw <= (uint32_t)opt.kmoves)) {
                const uint64_t cand = g + cw;
                if (cand < L.ub) {
                    L.ub = cand;
                    L.best_len = dv + lw;
                }
            }
        }
if (SHIFT <= 2) {
            uint32_t wr[ND];  // slot this expansion wrote for edge k
            bool pv[ND];      // edge k's push (heap_push_n after the edges)
            uint4 pk[ND];     // its heap entry
            uint32_t np = 0;
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                wr[k] = 0xFFFFFFFFu;
                pv[k] = false;
            }
#pragma unroll
        for (int k = 0; k < ND; ++k) {
            const uint2 e = ed[k];
            if (e.x == kNoEdge) break;  // edges are packed first
            ++L.touched;
            const uint32_t u = e.x;
            const uint64_t ng = g + e.y;
            bool fu;
            uint4 eu = e0[k];
            // the first slot again if this expansion wrote it for an earlier
            // edge (or a memoised walk may have written anything)
            bool dirty = !TABLES && k > 0;
#pragma unroll
            for (int j = 0; j < k; ++j) dirty |= wr[j] == ((u * 0x9E3779B1u) & W.mask);
            if (dirty) eu = W.ent[(u * 0x9E3779B1u) & W.mask];
            uint32_t ui = hprobe_from(W.ent, W.mask, L.tag, u, fu, eu);
            const bool seen = fu && !(eu.z == 0xFFFFFFFFu && eu.w == 0xFFFFFFFFu);
            if (!seen) {
                uint64_t hu;
                if (TABLES) {
                    hu = hr[k];
                    if (hu == kInf64) continue;
                    if (!ws_insert(L, W, ui, u, 0u)) {
                        L.overflow = L.done = true;
                        break;
                    }
                } else {
                    // walked (and so in the hash) by the room check above:
                    // its memo is final; no walk here (a second inlined walk
                    // per edge only grew the kernel)
                    if (!fu) {  // cannot happen: the heads were all walked
                        L.overflow = L.done = true;
                        break;
                    }
                    const uint4 mu = W.memo[ui];
                    hu = u64of(mu.x, mu.y);
                    if (hu == kInf64) continue;
                }
                if (L.hsize + np >= C) {
                    L.overflow = L.done = true;
                    break;
                }
                W.ent[ui].z = (uint32_t)ng;
                W.ent[ui].w = (uint32_t)(ng >> 32);
                W.aux[ui].x = dv + 1u;
                wr[k] = ui;
                ++L.inserted;
                pv[k] = true;
                pk[k] = hkey_make(ng + hval(opt, hu), u, ui);
                ++np;
            } else if (ng < u64of(eu.z, eu.w)) {
                if (L.hsize + np >= C) {
                    L.overflow = L.done = true;
                    break;
                }
                W.ent[ui].z = (uint32_t)ng;
                W.ent[ui].w = (uint32_t)(ng >> 32);
                W.aux[ui].x = dv + 1u;
                wr[k] = ui;
                ++L.updated;
                const uint64_t hu = TABLES ? hr[k] : u64of(W.memo[ui].x, W.memo[ui].y);
                pv[k] = true;
                pk[k] = hkey_make(ng + hval(opt, hu), u, ui);
                ++np;
            }
        }
        heap_push_n<ND>(W.hk, L.hsize, pv, pk);
        } else {
#pragma unroll 1
        for (int k = 0; k < (1 << SHIFT); ++k) {
            const uint2 e = adj_w[((size_t)v << SHIFT) + k];
            if (e.x == kNoEdge) break;  // edges are packed first
            ++L.touched;
            const uint32_t u = e.x;
            const uint64_t ng = g + e.y;
            bool fu;
            uint32_t ui = hprobe(W.ent, W.mask, L.tag, u, fu);
            const bool seen = fu && !(W.ent[ui].z == 0xFFFFFFFFu && W.ent[ui].w == 0xFFFFFFFFu);
            if (!seen) {
                uint64_t hu;
                if (TABLES) {
                    hu = tb.hrow[rb + u];
                    if (hu == kInf64) continue;
                    if (!ws_insert(L, W, ui, u, 0u)) {
                        L.overflow = L.done = true;
                        break;
                    }
                } else {
                    // walked (and so in the hash) by the room check above:
                    // its memo is final; no walk here (a second inlined walk
                    // per edge only grew the kernel)
                    if (!fu) {  // cannot happen: the heads were all walked
                        L.overflow = L.done = true;
                        break;
                    }
                    const uint4 mu = W.memo[ui];
                    hu = u64of(mu.x, mu.y);
                    if (hu == kInf64) continue;
                }
                if (L.hsize >= C) {
                    L.overflow = L.done = true;
                    break;
                }
                W.ent[ui].z = (uint32_t)ng;
                W.ent[ui].w = (uint32_t)(ng >> 32);
                W.aux[ui].x = dv + 1u;
                ++L.inserted;
                heap_push(W.hk, L.hsize, hkey_make(ng + hval(opt, hu), u, ui));
            } else if (ng < u64of(W.ent[ui].z, W.ent[ui].w)) {
                if (L.hsize >= C) {
                    L.overflow = L.done = true;
                    break;
                }
                W.ent[ui].z = (uint32_t)ng;
                W.ent[ui].w = (uint32_t)(ng >> 32);
                W.aux[ui].x = dv + 1u;
                ++L.updated;
                const uint64_t hu = TABLES ? tb.hrow[rb + u]
                                           : u64of(W.memo[ui].x, W.memo[ui].y);
                heap_push(W.hk, L.hsize, hkey_make(ng + hval(opt, hu), u, ui));
            }
        }
        }
    }
    // wave sums, one atomic per wave per counter
    unsigned long long v8[8] = {s_exp, s_ins, s_tou, s_upd, s_sur, s_len, s_fin, s_ovf};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v8[i] += __shfl_xor(v8[i], o, 64);
    }
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < 8; ++i) atomicAdd(&agg[i], v8[i]);
}

}  // namespace kern

// ---------------------------------------------------------------------------
// Launchers (host side of this translation unit).  Each launch goes through
// hipExtLaunchKernelGGL so that, when the caller armed a start/stop event pair
// (set_launch_events), the timestamps ride on the dispatch packet itself: exact
// kernel time without extra barrier packets between launches.

namespace {
thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;

template <typename... Args, typename F>
void launch_shm(F kernel, dim3 grid, dim3 block, size_t shm, hipStream_t s, Args... args) {
    hipEvent_t a = g_ev_start, b = g_ev_stop;
    g_ev_start = g_ev_stop = nullptr;
    hipExtLaunchKernelGGL(kernel, grid, block, shm, s, a, b, 0, args...);
}
template <typename... Args, typename F>
void launch(F kernel, dim3 grid, dim3 block, hipStream_t s, Args... args) {
    launch_shm(kernel, grid, block, 0, s, args...);
}
}  // namespace

void set_launch_events(hipEvent_t start, hipEvent_t stop) {
    g_ev_start = start;
    g_ev_stop = stop;
}

// CPD_XCD=0 turns the XCD-aware block remap off (A/B measurements).
uint32_t xcd_remap() {
    static const uint32_t on = [] {
        const char* e = std::getenv("CPD_XCD");
        return (e && *e == '0') ? 0u : 1u;
    }();
    return on;
}

// Tuning knobs for A/B runs: waves per workgroup of the down-sweep and of
// first_moves (CPD_DOWN_WPB, CPD_FM_WPB: 1, 2 or 4; a workgroup covers
// 256 x wpb targets), columns per gather group of first_moves (CPD_FM_G).
// Defaults = the fastest measured on the 1M-node bench (MI355X, 16k rows):
// down 4 waves (1: +5 %, 2: +8 %), first_moves 2 waves (4: +11 %), G = 2
// (1: +4 %, 4: +14 %).
uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = std::getenv(name);
    return (e && *e) ? (uint32_t)std::strtoul(e, nullptr, 10) : dflt;
}
uint32_t down_wpb() {
    static const uint32_t v = env_u32("CPD_DOWN_WPB", 4);
    return v;
}
uint32_t down8_wpb() {  // CPD_DOWN8_WPB: 1, 2 or 4 waves per narrow down-sweep workgroup
    static const uint32_t v = [] {
        const uint32_t w = env_u32("CPD_DOWN8_WPB", 2);
        return w == 1 ? 1u : (w == 4 ? 4u : 2u);
    }();
    return v;
}
uint32_t fm_wpb() {
    static const uint32_t v = env_u32("CPD_FM_WPB", 2);
    return v;
}
// narrow rows, 4-slot adjacency: first_moves_n4 (the generic
// first_moves<4, 2, true> measured slower and is not launched)
uint32_t fm_n4() { return 1u; }

void launch_sweep(bool ascend, const uint32_t* nodes, const uint32_t* arc_off,
                  const uint32_t* arcs32, uint32_t slot0, uint32_t count, uint32_t* dist,
                  uint32_t* up, uint32_t ubase, const uint32_t* uidx, const uint32_t* tgt,
                  uint32_t B, uint32_t slabs, const uint32_t* asc_nodes,
                  const uint32_t* asc_off, const uint32_t* asc_arcs, uint32_t* live,
                  const uint32_t* tmask, const uint32_t* adj, uint32_t shift, uint16_t* fmleaf,
                  NarrowRows nr, const uint32_t* desc, hipStream_t s) {
    const uint4* t4 = reinterpret_cast<const uint4*>(tgt);
    const uint2* arcs = reinterpret_cast<const uint2*>(arcs32);
    const kern::Closed cf{asc_nodes, asc_off, reinterpret_cast<const uint2*>(asc_arcs)};
    const kern::LeafFm lf{reinterpret_cast<const uint2*>(adj), shift, ascend ? nullptr : fmleaf};
    if (ascend && live) {
        // one block per node on wide levels; narrow levels split the slabs
        const uint32_t nsplit = std::max(1u, std::min(slabs, 2048u / std::max(count, 1u)));
        const uint32_t active = slabs >= 32 ? 0xFFFFFFFFu : ((1u << slabs) - 1u);
        launch(kern::sweep_up_sparse, dim3(count * nsplit * kern::kUpQ), dim3(64), s, nodes, arc_off, arcs,
               slot0, count, nsplit, xcd_remap(), up, ubase, t4, B / 4u, cf, live, tmask, active);
    } else if (ascend) {
        launch(kern::sweep_level<true>, dim3(count * slabs), dim3(256), s, nodes, arc_off, arcs,
               slot0, count, xcd_remap(), dist, up, ubase, uidx, t4, B / 4u, cf,
               (const uint32_t*)nullptr, lf);
    } else {
        const uint32_t tpb = 64u * down_wpb();  // a workgroup covers 4 * tpb targets
        const dim3 grid(count * slabs * (256u / tpb)), blk(tpb);
        if (nr.d16) {
            // 8 targets per lane: a workgroup of 64 x wpb8 lanes covers 512 x wpb8
            // targets (wpb8 = 2: one 1024-target slab)
            // (4 waves = 2048 targets: only when the slab count is even)
            const uint32_t wpb8 = down8_wpb() == 4 && slabs % 2 ? 2u : down8_wpb();
            const uint32_t tpb8 = 64u * wpb8;
            const dim3 g8(count * slabs * 2u / wpb8), b8(tpb8);
            launch(kern::sweep_down8, g8, b8, s, reinterpret_cast<const uint4*>(desc), arcs, slot0,
                   count, xcd_remap(), (const uint32_t*)up, t4, B / 4u, cf, (const uint32_t*)live,
                   fmleaf, nr);
        } else
            launch(kern::sweep_level<false>, grid, blk, s, nodes, arc_off, arcs, slot0, count,
                   xcd_remap(), dist, up, ubase, uidx, t4, B / 4u, cf, (const uint32_t*)live, lf);
    }
}

static uint32_t up_init_blocks() { return 2048u; }  // the init's grid (grid-stride, one wave each)

void launch_sweep_up_init(const uint32_t* slots, uint32_t nslots, const uint32_t* nodes,
                          uint32_t* up, uint32_t ubase, const uint32_t* tgt, uint32_t B,
                          uint32_t slabs, uint32_t* live, const uint32_t* tmask, hipStream_t s) {
    if (!nslots) return;
    const uint32_t active = slabs >= 32 ? 0xFFFFFFFFu : ((1u << slabs) - 1u);
    const uint32_t total = nslots * slabs * kern::kUpQ;
    launch(kern::sweep_up_init, dim3(std::min(total, up_init_blocks())), dim3(64), s, slots,
           nslots, total, nodes, up, ubase, reinterpret_cast<const uint4*>(tgt), B / 4u, live,
           tmask, active);
}

void launch_sweep_up_chunks(const uint32_t* items, uint32_t nitems, const uint32_t* arcs32,
                            uint32_t* up, uint32_t ubase, const uint32_t* tgt, uint32_t B,
                            uint32_t slabs, const uint32_t* asc_nodes, const uint32_t* asc_off,
                            const uint32_t* asc_arcs, uint32_t* live, const uint32_t* tmask,
                            hipStream_t s) {
    if (!nitems) return;
    const uint32_t active = slabs >= 32 ? 0xFFFFFFFFu : ((1u << slabs) - 1u);
    const kern::Closed cf{asc_nodes, asc_off, reinterpret_cast<const uint2*>(asc_arcs)};
    launch(kern::sweep_up_chunks, dim3(nitems * slabs * kern::kUpQ), dim3(64), s,
           reinterpret_cast<const uint4*>(items), nitems, xcd_remap(),
           reinterpret_cast<const uint2*>(arcs32), up, ubase, reinterpret_cast<const uint4*>(tgt),
           B / 4u, cf, live, tmask, active);
}


uint32_t sweep_chunk_arcs() { return (uint32_t)kern::kChunk; }
uint32_t down_desc_arcs() { return kern::kDescArcs; }

void launch_target_mask(const uint32_t* tgt, uint32_t B, uint32_t* tmask, hipStream_t s) {
    launch(kern::target_mask, dim3((B + 63u) / 64u), dim3(64), s, tgt, B, tmask);
}

void launch_live_stats(bool ascend, const uint32_t* nodes, const uint32_t* arc_off,
                       const uint32_t* arcs32, const uint32_t* lvl_of, uint32_t slot0,
                       uint32_t slot1, uint32_t ubase, const uint32_t* uidx,
                       const uint32_t* live, unsigned int* stat, hipStream_t s) {
    if (slot1 <= slot0) return;
    const dim3 grid((slot1 - slot0 + 255u) / 256u);
    const uint2* arcs = reinterpret_cast<const uint2*>(arcs32);
    if (ascend)
        launch(kern::live_stats<true>, grid, dim3(256), s, nodes, arc_off, arcs, lvl_of, slot0,
               slot1, ubase, uidx, live, stat);
    else
        launch(kern::live_stats<false>, grid, dim3(256), s, nodes, arc_off, arcs, lvl_of, slot0,
               slot1, ubase, uidx, live, stat);
}

// segments per first_moves_n4 workgroup, one after another (CPD_FM_SPW: 1,
// 2, 4, ..., 64).  At 7 waves per SIMD 8 measured 418.6-423.4k rows/s
// against 413.2-419.1k for one (profiles/up_store_ab/r06n_*, r06o_*); at 8
// waves per SIMD, whose workgroups hold every slot the up-sweep beside them
// needs, shorter workgroups hand slots over sooner: 2 measured 440.5-441.2k
// against 435.3-435.4k for 8 and 435.7-436.0k for 1 (r06ee_*)
static uint32_t fm_spw() {
    static const uint32_t v = [] {
        const char* e = std::getenv("CPD_FM_SPW");
        const uint32_t x = e && *e ? (uint32_t)std::atoi(e) : 2u;
        return (x && x <= 64u && !(x & (x - 1u))) ? x : 1u;
    }();
    return v;
}

uint32_t fm_bits(uint32_t shift) { return shift <= 2 ? 4u : (1u << shift); }

template <bool NARROW>
static void launch_first_moves_t(const uint2* adj, uint32_t shift, const uint32_t* dist,
                                 const uint32_t* tgt, uint32_t B, uint32_t n, uint32_t npad,
                                 uint32_t* fm, const uint32_t* leafbits, const uint16_t* fmleaf,
                                 NarrowRows nr, dim3 grid, dim3 blk, hipStream_t s) {
    const uint32_t r = xcd_remap();
    switch (shift) {  // SLOTS = 2^shift edges per column; G columns per gather group
        case 0: launch(kern::first_moves<1, 4, NARROW>, grid, blk, s, adj, dist, tgt, B, n, npad, r, fm, leafbits, fmleaf, nr); break;
        case 1: launch(kern::first_moves<2, 2, NARROW>, grid, blk, s, adj, dist, tgt, B, n, npad, r, fm, leafbits, fmleaf, nr); break;
        case 2: launch(kern::first_moves<4, 2, NARROW>, grid, blk, s, adj, dist, tgt, B, n, npad, r, fm, leafbits, fmleaf, nr); break;
        case 3: launch(kern::first_moves<8, 1, NARROW>, grid, blk, s, adj, dist, tgt, B, n, npad, r, fm, leafbits, fmleaf, nr); break;
        default: launch(kern::first_moves<16, 1, NARROW>, grid, blk, s, adj, dist, tgt, B, n, npad, r, fm, leafbits, fmleaf, nr); break;
    }
}

void launch_first_moves(const uint32_t* adj32, uint32_t shift, const uint32_t* dist,
                        const uint32_t* tgt, uint32_t B, uint32_t rows, uint32_t n,
                        uint32_t npad, uint32_t* fm, const uint32_t* leafbits,
                        const uint16_t* fmleaf, NarrowRows nr, hipStream_t s,
                        const uint32_t* seg_order) {
    const uint32_t tpb = 64u * fm_wpb();  // a workgroup covers 4 * tpb targets
    const dim3 grid((npad / kern::kSeg) * ((rows + 1023u) / 1024u) * (256u / tpb)), blk(tpb);
    const uint2* adj = reinterpret_cast<const uint2*>(adj32);
    if (nr.d16 && shift == 2 && fm_n4()) {
        const uint32_t spw = fm_spw();
        launch_shm(kern::first_moves_n4<2>, dim3(grid.x / spw), blk, 64u * tpb, s, adj, dist, tgt,
                   B, n, npad, xcd_remap(), fm, leafbits, fmleaf, nr, seg_order, spw);
    } else if (nr.d16)
        launch_first_moves_t<true>(adj, shift, dist, tgt, B, n, npad, fm, leafbits, fmleaf, nr,
                                   grid, blk, s);
    else
        launch_first_moves_t<false>(adj, shift, dist, tgt, B, n, npad, fm, leafbits, fmleaf, nr,
                                    grid, blk, s);
}

bool first_moves_reads_own(uint32_t shift, bool narrow) {
    return !(narrow && shift == 2 && fm_n4());  // only the generic kernel reads it
}

void launch_rle_count(const uint32_t* fm, uint32_t fmb, uint32_t npad, uint32_t nrows,
                      uint32_t* counts, uint32_t* st, uint8_t* rc, hipStream_t s,
                      const uint32_t* gate) {
    if (!nrows) return;
    const dim3 grid((nrows + 3u) / 4u), block(256);
    const kern::RleState rs{st, rc};
    switch (fmb) {
        case 4: launch(kern::rle_scan<4>, grid, block, s, fm, npad, nrows, counts, rs, gate); break;
        case 8: launch(kern::rle_scan<8>, grid, block, s, fm, npad, nrows, counts, rs, gate); break;
        default: launch(kern::rle_scan<16>, grid, block, s, fm, npad, nrows, counts, rs, gate); break;
    }
}

// the chunked count's chunks: 32 segments each (rle_count_ch<32>)
uint32_t rle_count_chunks(uint32_t npad) { return npad / kern::kSeg / 32u; }

void launch_rle_count_ch(const uint32_t* fm, uint32_t npad, uint32_t nrows, uint32_t* st,
                         uint8_t* rc, uint32_t* xs, uint32_t* cc, hipStream_t s) {
    if (!nrows) return;
    const uint32_t nch = rle_count_chunks(npad);
    const kern::RleChunks rk{xs, cc, xs + (size_t)nrows * nch};
    const dim3 grid((nch + 15u) / 16u, (nrows + 15u) / 16u), blk(256);
    launch(kern::rle_count_ch<32>, grid, blk, s, fm, npad, nrows, st, rc, rk);
}

void launch_rle_fix(const uint32_t* fm, uint32_t npad, uint32_t nrows, uint32_t* st,
                    uint8_t* rc, uint32_t* xs, uint32_t* cc, uint32_t* counts, uint32_t* hard,
                    hipStream_t s) {
    if (!nrows) return;
    const kern::RleChunks rk{xs, cc, xs + (size_t)nrows * rle_count_chunks(npad)};
    launch(kern::rle_fix<32>, dim3(nrows), dim3(64), s, fm, npad, nrows, st, rc, rk, counts,
           hard);
}

uint32_t rle_emit_chunks(uint32_t npad) {
    const uint32_t ntiles = npad / kern::kTile;
    return (ntiles + kern::kEmitTiles - 1u) / kern::kEmitTiles;
}

void launch_rle_emit(const uint32_t* fm, uint32_t npad, uint32_t nrows, const uint32_t* out_row,
                     uint32_t lb, uint32_t* dense, uint32_t* xe, uint32_t* xs, uint32_t* cc,
                     uint32_t* counts, hipStream_t s) {
    if (!nrows) return;
    const kern::EmitChunks ck{xe, xs, cc};
    const dim3 grid(rle_emit_chunks(npad) * ((nrows + 7u) / 8u));
    if (lb == 2u)
        launch(kern::rle_emit8<2>, grid, dim3(64), s, fm, npad, nrows, out_row, dense, ck, xcd_remap());
    else if (lb == 1u)
        launch(kern::rle_emit8<1>, grid, dim3(64), s, fm, npad, nrows, out_row, dense, ck, xcd_remap());
    else
        launch(kern::rle_emit8<0>, grid, dim3(64), s, fm, npad, nrows, out_row, dense, ck, xcd_remap());
    launch(kern::rle_emit_fix, dim3(nrows), dim3(64), s, fm, npad, nrows, out_row, lb, dense, ck,
           counts);
}

void launch_rle_moves(const uint32_t* fm, uint32_t fmb, uint32_t npad, uint32_t nrows,
                      const uint32_t* st, const uint8_t* rc, const uint32_t* out_row,
                      uint32_t lb, uint32_t* dense, hipStream_t s) {
    if (!nrows) return;
    const uint32_t ntiles = npad / kern::kTile;
    const dim3 grid((ntiles + kern::kMoveTiles - 1u) / kern::kMoveTiles, (nrows + 3u) / 4u),
        block(256);
    switch (fmb) {
        case 4: launch(kern::rle_moves4, grid, block, s, fm, npad, nrows, st, rc, out_row, lb, dense); break;
        case 8: launch(kern::rle_moves<8>, grid, block, s, fm, npad, nrows, st, rc, out_row, lb, dense); break;
        default: launch(kern::rle_moves<16>, grid, block, s, fm, npad, nrows, st, rc, out_row, lb, dense); break;
    }
}

void launch_repack_moves(const uint32_t* src, uint32_t s_stride, uint32_t s_words,
                         uint32_t s_bits, uint32_t rows, uint32_t* dst, uint32_t d_stride,
                         uint32_t d_words, uint32_t d_bits, hipStream_t s, uint32_t* lost) {
    const uint64_t items = (uint64_t)rows * d_words;
    if (!items) return;
    launch(kern::repack_moves, dim3((uint32_t)((items + 255u) / 256u)), dim3(256), s, src,
           s_stride, s_words, s_bits, rows, dst, d_stride, d_words, d_bits, lost);
}

void launch_moves_count(const uint32_t* dense, uint32_t stride, uint32_t lb, uint32_t n,
                        uint32_t nrows, uint32_t* counts, hipStream_t s) {
    if (!nrows) return;
    launch(kern::moves_runs<false>, dim3((nrows + 3u) / 4u), dim3(256), s, dense, stride, lb, n,
           nrows, (const uint64_t*)nullptr, (uint64_t)0, (uint32_t*)nullptr, counts);
}

void launch_moves_runs(const uint32_t* dense, uint32_t stride, uint32_t lb, uint32_t n,
                       uint32_t nrows, const uint64_t* off, uint64_t base, uint32_t* runs,
                       hipStream_t s) {
    if (!nrows) return;
    launch(kern::moves_runs<true>, dim3((nrows + 3u) / 4u), dim3(256), s, dense, stride, lb, n,
           nrows, off, base, runs, (uint32_t*)nullptr);
}

void launch_validate_rows(const uint64_t* offsets, const uint32_t* runs,
                          const uint32_t* chunk_first, uint32_t nrows, uint32_t total_chunks,
                          uint32_t n, uint32_t mlimit, uint32_t* bad, hipStream_t s) {
    if (!nrows || !total_chunks) return;
    launch(kern::validate_rows, dim3((total_chunks + 3u) / 4u), dim3(256), s, offsets, runs,
           chunk_first, nrows, total_chunks, n, mlimit, bad);
}

uint32_t expand_chunk_runs() { return kern::kExpandRuns; }

void launch_expand_rows(const uint64_t* offsets, const uint32_t* runs, const uint32_t* chunk_first,
                        uint32_t nrows, uint32_t total_chunks, uint32_t npad, uint32_t* dense,
                        hipStream_t s) {
    if (!nrows || !total_chunks) return;
    constexpr uint32_t cpw = kern::kExpandCpw;
    const uint32_t waves = (total_chunks + cpw - 1u) / cpw;
    launch(kern::expand_rows, dim3((waves + 3u) / 4u), dim3(256), s, offsets, runs, chunk_first,
           nrows, total_chunks, npad / 8u, cpw, dense);
}

// Table-search chunking (launch parameters only; results are identical under
// every setting): the batch is cut into chunks of ceil(nq / waves) queries (a
// multiple of 64, at most 1024 for dense rows), CPD_TS_WAVES
// overriding the wave count.  Measured on the 1M-node bench (1M queries,
// MI355X, tools_scripts/query_ab.py): dense walks want few waves that each
// refill their lanes ~16 times (waves 1024: 88M q/s; 8192 waves, i.e. no
// refill: 60M; round 1's lane per query: 43.7M), RLE walks — a chain of
// dependent loads per hop — want every wave slot filled (8192).  Two walks
// per lane (ILP 2) was slower in both forms; it and round 1's lane-per-query
// kernels were removed in round 3.
uint32_t ts_waves(uint32_t dflt) {
    static const uint32_t v = env_u32("CPD_TS_WAVES", 0);
    return v ? v : dflt;
}

template <class Rows>
static void launch_walk(const uint2* adj, uint32_t shift, const Rows& rows, const uint32_t* qs,
                        const uint32_t* qt, const uint32_t* qrow, uint32_t nq, uint32_t limit,
                        uint64_t* cost, uint32_t* hops, uint8_t* fin, unsigned long long* agg,
                        uint32_t waves_target, uint32_t chunk_max, hipStream_t s,
                        uint32_t wpb_default) {
    constexpr uint32_t unit = 64u;
    uint64_t chunk = ((uint64_t)nq + waves_target - 1u) / waves_target;
    chunk = std::min<uint64_t>(chunk, std::max(unit, chunk_max));
    chunk = std::max<uint64_t>(unit, (chunk + unit - 1u) / unit * unit);
    const uint64_t waves = ((uint64_t)nq + chunk - 1u) / chunk;
    // waves per workgroup: dense walks 1 (their ~1000 waves spread over every
    // CU: 92.3M against 90.3M q/s with 4), RLE walks 4 (8192 one-wave
    // workgroups ran out of workgroup slots: 8.2M against 11.4M);
    // CPD_TS_WPB overrides both (A/B, profiles/walk_wpb_ab/)
    static const uint32_t wpb_env = env_u32("CPD_TS_WPB", 0);
    const uint32_t wpb = std::min(4u, std::max(1u, wpb_env ? wpb_env : wpb_default));
    const dim3 grid((uint32_t)std::max<uint64_t>(1u, (waves + wpb - 1u) / wpb)), blk(64u * wpb);
    const uint32_t c = (uint32_t)chunk;
#define CPD_WALK(SH, IL)                                                                       \
    launch(kern::table_walk<SH, IL, Rows>, grid, blk, s, adj, rows, qs, qt, qrow, nq, c, limit, \
           cost, hops, fin, agg)
    switch (shift) {
        case 0: CPD_WALK(0, 1); break;
        case 1: CPD_WALK(1, 1); break;
        case 2: CPD_WALK(2, 1); break;
        case 3: CPD_WALK(3, 1); break;
        default: CPD_WALK(4, 1); break;
    }
#undef CPD_WALK
}

static uint32_t walk_limit(int32_t kmoves, uint32_t n) {
    return kmoves >= 0 ? std::min((uint32_t)kmoves, n) : n;
}

void launch_table_search_dense(const uint32_t* adj, uint32_t shift, const uint32_t* row_of_col,
                               const uint32_t* dense, uint32_t npad, uint32_t lb,
                               const uint32_t* qs, const uint32_t* qt, const uint32_t* qrow,
                               uint32_t nq, int32_t kmoves, uint32_t n, uint64_t* cost,
                               uint32_t* hops, uint8_t* fin, unsigned long long* agg,
                               hipStream_t s) {
    const kern::DenseRows rows{dense, npad >> (5u - lb), kern::Tbl{lb}};
    launch_walk(reinterpret_cast<const uint2*>(adj), shift, rows, qs, qt, qrow, nq,
                walk_limit(kmoves, n), cost, hops, fin, agg, ts_waves(1024), 1024u, s,
                1u);
}

void launch_table_search(const uint32_t* adj, uint32_t shift, const uint32_t* row_of_col,
                         const uint64_t* offsets, const uint32_t* runs, const uint32_t* qs,
                         const uint32_t* qt, const uint32_t* qrow, uint32_t nq, int32_t kmoves,
                         uint32_t n, uint64_t* cost, uint32_t* hops, uint8_t* fin,
                         unsigned long long* agg, hipStream_t s) {
    launch_walk(reinterpret_cast<const uint2*>(adj), shift, kern::RleRows{offsets, runs}, qs, qt,
                qrow, nq, walk_limit(kmoves, n), cost, hops, fin, agg, ts_waves(8192),
                1u << 30, s, 4u);
}


// Lane slots for nq searches: at most CPD_SEARCH_WAVES (1024) one-wave
// workgroups (64k lanes: 3,389 q/s at fscale 0 on the 1M graph against
// 1,657 with 256 waves, profiles/search_lanes_ab/), a whole wave each
uint32_t search_slots(uint32_t nq) {
    static const uint32_t waves = std::max(1u, env_u32("CPD_SEARCH_WAVES", 1024));
    const uint32_t want = (nq + 63u) / 64u;
    return 64u * std::max(1u, std::min(waves, want));
}

void launch_search_tables(const uint32_t* dense, uint32_t npad, uint32_t lb, const uint32_t* adj_f,
                          const uint32_t* adj_w, uint32_t shift, const uint32_t* tcol,
                          uint32_t rows, uint32_t n, void* scratch, uint32_t chunk_rows,
                          uint64_t* hrow, uint64_t* crow, uint32_t* lrow, int write_h,
                          hipStream_t s) {
    uint32_t rounds = 1;
    while ((1ull << (rounds - 1)) < (uint64_t)n + 1ull) ++rounds;  // 2^(rounds-1) > n hops
    const size_t per = (size_t)chunk_rows * n;
    char* base = static_cast<char*>(scratch);
    auto state = [&](int k) {
        char* p = base + (size_t)k * per * 24u;
        return kern::JumpState{reinterpret_cast<uint32_t*>(p),
                               reinterpret_cast<uint64_t*>(p + per * 4u),
                               reinterpret_cast<uint64_t*>(p + per * 12u),
                               reinterpret_cast<uint32_t*>(p + per * 20u)};
    };
    const kern::JumpState A = state(0), Bs = state(1);
    const uint2* af = reinterpret_cast<const uint2*>(adj_f);
    const uint2* aw = reinterpret_cast<const uint2*>(adj_w);
    for (uint32_t r0 = 0; r0 < rows; r0 += chunk_rows) {
        const uint32_t R = std::min(chunk_rows, rows - r0);
        const uint64_t items = (uint64_t)R * n;
        const dim3 grid((uint32_t)((items + 255u) / 256u)), blk(256);
        const uint32_t wpr = npad >> (5u - lb);
        launch(kern::jump_init, grid, blk, s, dense + (size_t)r0 * wpr, wpr, kern::Tbl{lb}, af, aw,
               shift, tcol + r0, R, n, A);
        kern::JumpState a = A, b = Bs;
        for (uint32_t k = 0; k < rounds; ++k) {
            launch(kern::jump_round, grid, blk, s, a, b, tcol + r0, R, n);
            std::swap(a, b);
        }
        launch(kern::jump_final, grid, blk, s, a, tcol + r0, R, n, hrow + (size_t)r0 * n,
               crow + (size_t)r0 * n, lrow + (size_t)r0 * n, write_h);
    }
}

void launch_cpd_search(const uint32_t* adj_f, const uint32_t* adj_w, uint32_t shift,
                       const uint32_t* dense, uint32_t npad, uint32_t lb, const uint64_t* hrow,
                       const uint64_t* crow, const uint32_t* lrow, uint32_t n,
                       const uint32_t* qs, const uint32_t* qt, const uint32_t* qrow, uint32_t nq,
                       double hscale, double fscale, int32_t kmoves, int64_t itrs,
                       uint64_t time_ns, uint64_t tick_ns, void* ws, uint32_t cap,
                       uint32_t slots, const SearchSpillArgs& spill, uint64_t* cost,
                       uint32_t* plen, uint8_t* fin, uint32_t* qstats, unsigned long long* agg,
                       hipStream_t s) {
    const bool tables = hrow != nullptr;
    // Few searches left (a late pass): fewer lanes per wave, more waves —
    // each wave issues for fewer divergent lanes, and the SIMDs a full-wave
    // launch would leave idle take the rest (CPD_SEARCH_LPW_MIN: the fewest
    // lanes per wave allowed, default 8; 64 = off — profiles/search_heap_ab/
    // r05aj: fscale 0 5.51-5.69k against 5.03k q/s)
    static const uint32_t lpw_min = std::max(8u, std::min(64u, env_u32("CPD_SEARCH_LPW_MIN", 8)));
    // (the fewest lanes, a multiple of 8, at which the slots' waves still fit
    // one per SIMD: 1024 one-wave workgroups; more waves queued behind the
    // resident ones lost their A/B in round 5, profiles/search_resident_ab/)
    constexpr uint32_t resident = 1024u;
    const uint32_t fit = (uint32_t)(((uint64_t)slots + resident - 1u) / resident);
    const uint32_t lpw = std::max(lpw_min, std::min(64u, (fit + 7u) / 8u * 8u));
    const uint32_t waves = slots / lpw;  // waves x lpw <= slots workspaces
    kern::SearchWs w;
    w.cap = cap;
    // lane-major blocks: search_ws_bytes_per_slot each, 128-B aligned; the
    // heap first
    w.base = static_cast<char*>(ws);
    w.stride = search_ws_bytes_per_slot(cap, tables);
    w.lpw = lpw;
    const kern::SearchOpt o{hscale, fscale, kmoves, itrs, time_ns, tick_ns};
    const kern::SearchTables tb{hrow, crow, lrow, n};
    const kern::SearchSpill sp{spill.resume, spill.rin, spill.at, spill.rout, spill.top,
                               spill.cap_words};
    // a wave per workgroup: the searches are latency chains, and 256 waves
    // as 64 four-wave workgroups sat on a quarter of the CUs (their L1s and
    // address units shared four ways) while the rest idled
    const dim3 grid(waves), blk(64);  // every wave has a workspace slot
    const uint32_t c2 = (uint32_t)(((uint64_t)nq + waves - 1u) / waves);
    const uint2* af = reinterpret_cast<const uint2*>(adj_f);
    const uint2* aw = reinterpret_cast<const uint2*>(adj_w);
    const uint32_t wpr = npad >> (5u - lb);
#define CPD_SEARCH(SH, T)                                                                    \
    launch(kern::cpd_search<SH, T>, grid, blk, s, af, aw, dense, wpr, lb, tb, qs, qt, qrow, nq, c2, \
           o, w, sp, cost, plen, fin, qstats, agg)
#define CPD_SEARCH_T(SH)          \
    if (tables) CPD_SEARCH(SH, true); \
    else CPD_SEARCH(SH, false)
    switch (shift) {
        case 0: CPD_SEARCH_T(0); break;
        case 1: CPD_SEARCH_T(1); break;
        case 2: CPD_SEARCH_T(2); break;
        case 3: CPD_SEARCH_T(3); break;
        default: CPD_SEARCH_T(4); break;
    }
#undef CPD_SEARCH_T
#undef CPD_SEARCH
}

void launch_query_keys(const uint32_t* s, const uint32_t* t, uint32_t nq, uint32_t n,
                       const uint32_t* order, const uint32_t* row_of_col, uint32_t* key,
                       uint32_t* val, uint32_t* bad, hipStream_t st) {
    if (!nq) return;
    launch(kern::query_keys, dim3((nq + 255u) / 256u), dim3(256), st, s, t, nq, n, order,
           row_of_col, key, val, bad);
}

size_t query_sort_bytes(uint32_t nq) {
    size_t b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (int)nq, 0, 32, (hipStream_t)0);
    return b;
}

void launch_query_sort(void* tmp, size_t tmp_bytes, const uint32_t* key_in, uint32_t* key_out,
                       const uint32_t* val_in, uint32_t* val_out, uint32_t nq, uint32_t nrows,
                       hipStream_t st) {
    if (!nq) return;
    int bits = 1;
    while (bits < 32 && (1ull << bits) < (uint64_t)nrows) ++bits;
    size_t b = tmp_bytes;
    (void)hipcub::DeviceRadixSort::SortPairs(tmp, b, key_in, key_out, val_in, val_out, (int)nq, 0,
                                             bits, st);
}

void launch_query_gather(const uint32_t* s, const uint32_t* t, const uint32_t* order,
                         const uint32_t* key, const uint32_t* val, uint32_t nq, uint32_t* qs,
                         uint32_t* qt, uint32_t* qrow, hipStream_t st) {
    if (!nq) return;
    launch(kern::query_gather, dim3((nq + 255u) / 256u), dim3(256), st, s, t, order, key, val, nq,
           qs, qt, qrow);
}

template <class T>
static void scatter_t(const T* in, const uint32_t* perm, uint32_t nq, uint32_t k, T* out,
                      hipStream_t st) {
    if (!nq) return;
    const uint64_t items = (uint64_t)nq * k;
    launch(kern::scatter_rows<T>, dim3((uint32_t)((items + 255u) / 256u)), dim3(256), st, in, perm,
           nq, k, out);
}
void launch_scatter_u64(const uint64_t* in, const uint32_t* perm, uint32_t nq, uint64_t* out,
                        hipStream_t st) {
    scatter_t(in, perm, nq, 1u, out, st);
}
void launch_scatter_u32(const uint32_t* in, const uint32_t* perm, uint32_t nq, uint32_t k,
                        uint32_t* out, hipStream_t st) {
    scatter_t(in, perm, nq, k, out, st);
}
void launch_scatter_u8(const uint8_t* in, const uint32_t* perm, uint32_t nq, uint8_t* out,
                       hipStream_t st) {
    scatter_t(in, perm, nq, 1u, out, st);
}

// Workspace per lane slot and column of capacity: hash entries 2 x (16 + 8),
// heap 16 (f, column, hash slot), and for memoised walks the memo (2 x 16)
// and walk stack (16).  Per slot: ent 32C, aux 16C (+ memo 32C, stk 16C with
// walks) and the heap, 16 (C + kHeapK) B; a multiple of 128 B (aligned
// lane-major blocks)
uint64_t search_ws_bytes_per_slot(uint32_t cap, bool tables) {
    const uint64_t b = (tables ? 64ull : 112ull) * cap + 16ull * kern::kHeapK;
    return (b + 127u) / 128u * 128u;
}

// a record: the head, <= cap heap entries of 3 words, <= cap columns of 5
// (tables) or 9 (walks) words
uint64_t search_spill_words(uint32_t cap, bool tables) {
    return kern::kSpillHead + (tables ? 8ull : 12ull) * cap;
}

}  // namespace cpd

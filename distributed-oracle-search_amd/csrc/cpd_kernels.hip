// HIP kernels for gfx950 (MI355X, CDNA4).  Integer/byte work, HBM-bound: no
// MFMA.  Every kernel is written for wave64 and 256-thread workgroups.
//
// Data layout in HBM (column space = DFS-preorder position of a node):
//   dist  [col][B]   u32   one batch row of B targets per column; a wave's
//                          16-B/lane access covers 256 targets = 1 KiB
//   fm    [row][npad] u16  first-move sets, row-major for the RLE scan;
//                          columns >= n are padded with the wildcard
//   runs  [row][cap]  u32  RLE scratch, compacted afterwards
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cpd_kernels.hpp"

namespace cpd {
namespace kern {

constexpr uint32_t INF = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t sat_add(uint32_t d, uint32_t w) {
    uint32_t s = d + w;
    return (s < d) ? INF : s;  // d == INF or overflow -> INF
}

__device__ __forceinline__ void min4(uint4& acc, const uint4 d, uint32_t w) {
    acc.x = min(acc.x, sat_add(d.x, w));
    acc.y = min(acc.y, sat_add(d.y, w));
    acc.z = min(acc.z, sat_add(d.z, w));
    acc.w = min(acc.w, sat_add(d.w, w));
}

// One CH sweep level.  Block (x = slot in the level, y = 1024-target slab):
// node v = nodes[slot]; its arcs (col, w) are wave-uniform (scalar loads); each
// lane owns 4 consecutive targets.  ASCEND: upward sweep, init 0 at the lane's
// own target else INF.  !ASCEND: downward sweep, init = current dist (the
// upward value).  Then acc = min(acc, w + dist[arc.col]) over the arcs.
template <bool ASCEND>
__global__ __launch_bounds__(256) void sweep_level(const uint32_t* __restrict__ nodes,
                                                   const uint32_t* __restrict__ arc_off,
                                                   const uint2* __restrict__ arcs,
                                                   uint32_t slot0,
                                                   uint32_t* __restrict__ dist,
                                                   const uint4* __restrict__ tgt4,
                                                   uint32_t B4) {
    const uint32_t slot = slot0 + blockIdx.x;
    const uint32_t l4 = blockIdx.y * 256u + threadIdx.x;
    const uint32_t v = nodes[slot];
    const uint32_t a0 = arc_off[slot], a1 = arc_off[slot + 1];
    uint4* __restrict__ d4 = reinterpret_cast<uint4*>(dist);
    uint4 acc;
    if (ASCEND) {
        const uint4 t = tgt4[l4];
        acc.x = (t.x == v) ? 0u : INF;
        acc.y = (t.y == v) ? 0u : INF;
        acc.z = (t.z == v) ? 0u : INF;
        acc.w = (t.w == v) ? 0u : INF;
    } else {
        acc = d4[(size_t)v * B4 + l4];
    }
    uint32_t a = a0;
    for (; a + 4 <= a1; a += 4) {
        const uint2 e0 = arcs[a], e1 = arcs[a + 1], e2 = arcs[a + 2], e3 = arcs[a + 3];
        const uint4 x0 = d4[(size_t)e0.x * B4 + l4];
        const uint4 x1 = d4[(size_t)e1.x * B4 + l4];
        const uint4 x2 = d4[(size_t)e2.x * B4 + l4];
        const uint4 x3 = d4[(size_t)e3.x * B4 + l4];
        min4(acc, x0, e0.y);
        min4(acc, x1, e1.y);
        min4(acc, x2, e2.y);
        min4(acc, x3, e3.y);
    }
    for (; a < a1; ++a) {
        const uint2 e = arcs[a];
        min4(acc, d4[(size_t)e.x * B4 + l4], e.y);
    }
    d4[(size_t)v * B4 + l4] = acc;
}

// First-move sets.  Block (x = 64-column tile, y = 256-target slab); thread =
// one target, walks the tile's 64 columns: fm = bits k with
// w_k + d(dst_k) == d(c) (wildcard at the target and unreachable columns),
// then writes the 128-B row segment fm[target][c0 .. c0+64).
__global__ __launch_bounds__(256) void first_moves(const uint32_t* __restrict__ row_ptr,
                                                   const uint32_t* __restrict__ dst,
                                                   const uint32_t* __restrict__ w,
                                                   const uint32_t* __restrict__ dist,
                                                   const uint32_t* __restrict__ tgt,
                                                   uint32_t B, uint32_t n, uint32_t npad,
                                                   uint16_t* __restrict__ fm) {
    const uint32_t j = blockIdx.y * 256u + threadIdx.x;
    const uint32_t c0 = blockIdx.x * 64u;
    const uint32_t tcol = tgt[j];
    uint32_t packed[32];
#pragma unroll
    for (int p = 0; p < 32; ++p) {
        uint32_t two = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = c0 + 2u * p + h;
            uint32_t f = 0xFFFFu;
            if (c < n) {
                const uint32_t dn = dist[(size_t)c * B + j];
                const uint32_t e0 = row_ptr[c], e1 = row_ptr[c + 1];
                uint32_t bits = 0;
                for (uint32_t e = e0; e < e1; ++e) {
                    const uint32_t dv = dist[(size_t)dst[e] * B + j];
                    bits |= (sat_add(dv, w[e]) == dn ? 1u : 0u) << (e - e0);
                }
                f = (c == tcol || dn == INF) ? 0xFFFFu : bits;
            }
            two |= f << (16 * h);
        }
        packed[p] = two;
    }
    uint4* out = reinterpret_cast<uint4*>(fm + (size_t)j * npad + c0);
#pragma unroll
    for (int q = 0; q < 8; ++q)
        out[q] = make_uint4(packed[4 * q], packed[4 * q + 1], packed[4 * q + 2], packed[4 * q + 3]);
}

__device__ __forceinline__ uint32_t pick8(const uint32_t (&v)[8], int j) {
    uint32_t r = v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) r = (j == k) ? v[k] : r;
    return r;
}

// Greedy RLE of one row per wave (warthog graph_oracle::add_row [U]).  A chunk
// is 512 columns: lane l holds columns 8l..8l+7 (one 16-B load).  Given the
// running intersection S, the first column where S & AND(cols) becomes 0 is
// found with a lane-local prefix AND, a wave-wide exclusive AND-scan of the
// lane totals and a ballot; the run is emitted, S restarts at that column and
// the chunk is rescanned past it.  Output: runs[row*cap + i], counts[row]
// (the true count, even past `cap`; the host re-runs overflowing rows).
__global__ __launch_bounds__(256) void rle_rows(const uint16_t* __restrict__ fm,
                                                uint32_t npad, uint32_t nrows,
                                                uint32_t* __restrict__ runs,
                                                uint32_t cap,
                                                uint32_t* __restrict__ counts) {
    const uint32_t row = blockIdx.x * 4u + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= nrows) return;
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(fm + (size_t)row * npad);
    uint32_t* __restrict__ out = runs + (size_t)row * cap;
    uint32_t S = 0xFFFFu, head = 0, cnt = 0;
    const uint32_t nchunks = npad / 512u;
    uint4 q = src[lane];
    for (uint32_t ch = 0; ch < nchunks; ++ch) {
        const uint4 cur = q;
        if (ch + 1 < nchunks) q = src[(size_t)(ch + 1) * 64u + lane];
        uint32_t v[8] = {cur.x & 0xFFFFu, cur.x >> 16, cur.y & 0xFFFFu, cur.y >> 16,
                         cur.z & 0xFFFFu, cur.z >> 16, cur.w & 0xFFFFu, cur.w >> 16};
        int p = 0;  // first local column not yet consumed
        for (;;) {
            uint32_t P[8];
            uint32_t acc = 0xFFFFu;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t val = (lane * 8 + j < p) ? 0xFFFFu : v[j];
                acc &= val;
                P[j] = acc;
            }
            uint32_t x = acc;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, 64);
                if (lane >= off) x &= y;
            }
            uint32_t E = __shfl_up(x, 1, 64);
            if (lane == 0) E = 0xFFFFu;
            const uint32_t base = S & E;
            const unsigned long long mask = __ballot((base & acc) == 0u);
            if (mask == 0ull) {
                S &= __shfl(x, 63, 64);
                break;
            }
            const int L = __ffsll(mask) - 1;
            int j0 = 7;
            uint32_t before = base;
#pragma unroll
            for (int j = 7; j >= 0; --j)
                if ((base & P[j]) == 0u) j0 = j;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < j0) before = base & P[j];
            const uint32_t bval = pick8(v, j0);
            j0 = __shfl(j0, L, 64);
            before = __shfl(before, L, 64);
            const uint32_t newS = __shfl(bval, L, 64);
            const int bl = L * 8 + j0;
            if (lane == 0 && cnt < cap) out[cnt] = (head << 4) | (uint32_t)__builtin_ctz(before);
            ++cnt;
            head = ch * 512u + (uint32_t)bl;
            S = newS;
            p = bl + 1;
            if (p >= 512) break;
        }
    }
    if (lane == 0) {
        if (cnt < cap) out[cnt] = (head << 4) | (uint32_t)__builtin_ctz(S);
        ++cnt;
        counts[row] = cnt;
    }
}

// Copy each row's runs from the scratch slab to its compact offset.
__global__ __launch_bounds__(256) void compact_rows(const uint32_t* __restrict__ scratch,
                                                    uint32_t cap,
                                                    const uint64_t* __restrict__ off,
                                                    uint32_t* __restrict__ out) {
    const uint32_t row = blockIdx.x;
    const uint64_t b = off[row], e = off[row + 1];
    const uint32_t len = (uint32_t)(e - b);
    const uint32_t* s = scratch + (size_t)row * cap;
    for (uint32_t i = threadIdx.x; i < len; i += 256u) out[b + i] = s[i];
}

// Table-search extraction, one lane per query.  cur/t are columns; the run for
// column cur is found by galloping from the previous hop's run (consecutive
// path nodes have nearby DFS columns), then binary search inside the bracket:
// the result is always the LAST run with start <= cur — the same run warthog's
// get_move binary search returns [U].
__global__ __launch_bounds__(256) void table_search(
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ dst,
    const uint32_t* __restrict__ w, const uint32_t* __restrict__ row_of_col,
    const uint64_t* __restrict__ offsets, const uint32_t* __restrict__ runs,
    const uint32_t* __restrict__ qs, const uint32_t* __restrict__ qt, uint32_t nq,
    int32_t kmoves, uint32_t n, uint64_t* __restrict__ cost_out,
    uint32_t* __restrict__ hops_out, uint8_t* __restrict__ fin_out,
    unsigned long long* __restrict__ agg) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    uint64_t cost = 0;
    uint32_t hops = 0, fin = 0;
    if (q < nq) {
        const uint32_t t = qt[q];
        uint32_t cur = qs[q];
        const uint32_t row = row_of_col[t];
        const uint32_t* __restrict__ rr = runs + offsets[row];
        const uint32_t R = (uint32_t)(offsets[row + 1] - offsets[row]);
        const uint32_t limit = kmoves >= 0 ? (uint32_t)kmoves : n;
        uint32_t pos = 0;
        while (cur != t && hops < limit && hops < n) {
            uint32_t lo, hi;  // invariant: start(lo) <= cur < start(hi) (hi==R: +inf)
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
            pos = lo;
            const uint32_t mv = rr[lo] & 0xFu;
            const uint32_t e0 = row_ptr[cur];
            if (mv >= row_ptr[cur + 1] - e0) break;
            cost += w[e0 + mv];
            cur = dst[e0 + mv];
            ++hops;
        }
        fin = (cur == t) ? 1u : 0u;
        cost_out[q] = cost;
        hops_out[q] = hops;
        fin_out[q] = (uint8_t)fin;
    }
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

}  // namespace kern

// ---------------------------------------------------------------------------
// Launchers (host side of this translation unit).

void launch_sweep(bool ascend, const uint32_t* nodes, const uint32_t* arc_off,
                  const uint32_t* arcs32, uint32_t slot0, uint32_t count, uint32_t* dist,
                  const uint32_t* tgt, uint32_t B, uint32_t slabs, hipStream_t s) {
    dim3 grid(count, slabs);
    const uint4* t4 = reinterpret_cast<const uint4*>(tgt);
    const uint2* arcs = reinterpret_cast<const uint2*>(arcs32);
    if (ascend)
        kern::sweep_level<true><<<grid, 256, 0, s>>>(nodes, arc_off, arcs, slot0, dist, t4, B / 4u);
    else
        kern::sweep_level<false><<<grid, 256, 0, s>>>(nodes, arc_off, arcs, slot0, dist, t4, B / 4u);
}

void launch_first_moves(const uint32_t* row_ptr, const uint32_t* dst, const uint32_t* w,
                        const uint32_t* dist, const uint32_t* tgt, uint32_t B,
                        uint32_t rows, uint32_t n, uint32_t npad, uint16_t* fm,
                        hipStream_t s) {
    dim3 grid(npad / 64u, (rows + 255u) / 256u);
    kern::first_moves<<<grid, 256, 0, s>>>(row_ptr, dst, w, dist, tgt, B, n, npad, fm);
}

void launch_rle(const uint16_t* fm, uint32_t npad, uint32_t nrows, uint32_t* runs,
                uint32_t cap, uint32_t* counts, hipStream_t s) {
    kern::rle_rows<<<(nrows + 3u) / 4u, 256, 0, s>>>(fm, npad, nrows, runs, cap, counts);
}

void launch_compact(const uint32_t* scratch, uint32_t cap, const uint64_t* off,
                    uint32_t nrows, uint32_t* out, hipStream_t s) {
    kern::compact_rows<<<nrows, 256, 0, s>>>(scratch, cap, off, out);
}

void launch_table_search(const uint32_t* row_ptr, const uint32_t* dst, const uint32_t* w,
                         const uint32_t* row_of_col, const uint64_t* offsets,
                         const uint32_t* runs, const uint32_t* qs, const uint32_t* qt,
                         uint32_t nq, int32_t kmoves, uint32_t n, uint64_t* cost,
                         uint32_t* hops, uint8_t* fin, unsigned long long* agg,
                         hipStream_t s) {
    kern::table_search<<<(nq + 255u) / 256u, 256, 0, s>>>(row_ptr, dst, w, row_of_col, offsets,
                                                          runs, qs, qt, nq, kmoves, n, cost,
                                                          hops, fin, agg);
}

}  // namespace cpd

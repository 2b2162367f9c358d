// GPU contraction of the hierarchy (driven by ch_gpu.cpp): ch.cpp's parallel
// independent-set contraction, step for step, with every decision made the
// same way — the priority key, the independent set, the witness searches (a
// bounded Dijkstra whose binary heap replays libstdc++'s push_heap /
// pop_heap, so that ties settle in the same order and a settle limit cuts a
// search at the same node), the lightest-arc merge of the shortcuts.  The
// hierarchy it yields is the host's, arc for arc (tests/test_ch_gpu.py).
//
// Work is integer and latency-bound (a witness search is a chain of
// dependent loads): one lane per search, lanes refilled grid-stride, the
// search's hash table and heap in an HBM workspace per lane; nothing here is
// GEMM-shaped.  The searches dominate: a 1M-node road graph needs ~10M of
// them over ~200 rounds.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "ch_kernels.hpp"

namespace cpd {
namespace chk {
namespace {

constexpr uint32_t kTgtBit = 0x80000000u;
constexpr uint64_t kInf = ~0ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ch.cpp Contractor::less_key (ids are the original ids here)
__device__ __forceinline__ bool less_key(uint32_t a, uint32_t b, const int64_t* prio) {
    const int64_t pa = prio[a], pb = prio[b];
    if (pa != pb) return pa < pb;
    const uint64_t ha = mix64(a), hb = mix64(b);
    if (ha != hb) return ha < hb;
    return a < b;
}

__device__ __forceinline__ uint32_t gid() { return blockIdx.x * blockDim.x + threadIdx.x; }

__global__ void k_pick(const uint32_t* __restrict__ rem, uint32_t R, Overlay g,
                       const int64_t* __restrict__ prio, uint32_t* __restrict__ flag) {
    const uint32_t i = gid();
    if (i > R) return;
    if (i == R) {
        flag[R] = 0;
        return;
    }
    const uint32_t v = rem[i];
    const uint2* arcs = reinterpret_cast<const uint2*>(g.arcs);
    bool ok = true;
    for (uint32_t k = 0, o = g.ooff[v], d = g.odeg[v]; k < d; ++k)
        if (!less_key(v, arcs[o + k].x, prio)) {
            ok = false;
            break;
        }
    if (ok)
        for (uint32_t k = 0, o = g.ioff[v], d = g.ideg[v]; k < d; ++k)
            if (!less_key(v, arcs[o + k].x, prio)) {
                ok = false;
                break;
            }
    flag[i] = ok ? 1u : 0u;
}

__global__ void k_split(const uint32_t* __restrict__ in, const uint32_t* __restrict__ flag,
                        const uint32_t* __restrict__ pos, uint32_t n, uint32_t* __restrict__ sel,
                        uint32_t* __restrict__ rej) {
    const uint32_t i = gid();
    if (i >= n) return;
    if (flag[i])
        sel[pos[i]] = in[i];
    else
        rej[i - pos[i]] = in[i];
}

__global__ void k_sel_counts(const uint32_t* __restrict__ S, uint32_t nS, Overlay g,
                             uint8_t* __restrict__ state, uint32_t* c0, uint32_t* c1,
                             uint32_t* c2, uint32_t* c3) {
    const uint32_t i = gid();
    if (i > nS) return;
    if (i == nS) {
        c0[i] = c1[i] = c2[i] = c3[i] = 0;
        return;
    }
    const uint32_t v = S[i];
    const uint32_t od = g.odeg[v], id = g.ideg[v];
    state[v] = 1;
    c0[i] = od ? id : 0u;
    c1[i] = od ? id * od : 0u;
    c2[i] = od;
    c3[i] = id;
}

__global__ void k_make_pairs(const uint32_t* __restrict__ list, uint32_t k, Overlay g,
                             const uint32_t* __restrict__ pbase, const uint32_t* __restrict__ sbase,
                             uint4* __restrict__ pairs) {
    const uint32_t i = gid();
    if (i >= k) return;
    const uint32_t v = list[i];
    const uint32_t od = g.odeg[v];
    if (!od) return;
    const uint32_t id = g.ideg[v], p0 = pbase[i], s0 = sbase ? sbase[i] : 0u;
    for (uint32_t j = 0; j < id; ++j) pairs[p0 + j] = make_uint4(v, j, s0 + j * od, 0u);
}

// ---------------------------------------------------------------------------
// Witness search.  Workspace per lane: hash[caps.hash] (tag, node | target
// bit, dist lo, dist hi), heap[caps.heap] (dist lo, dist hi, node, -),
// tgt[caps.tgt] (via lo, via hi, node, -) sorted by via descending, tset[caps.tgt]
// (1 = that target has settled).  Entries are valid when their tag is the
// search's (tags are never reused within a workspace), so nothing is cleared.

constexpr uint32_t kRelax = 8;  // arcs of a settled node relaxed per group

struct Lane {
    uint4* hash;
    uint4* heap;
    uint4* tgt;
    uint32_t* tset;
    uint32_t hmask, hcap_fill, heap_cap;
    uint32_t tag, hn, L;
    bool ovf;

    __device__ __forceinline__ uint32_t slot0(uint32_t node) const {
        return (node * 0x9E3779B1u) & hmask;
    }
    // slot of node, or hmask + 1 + (free slot) when absent
    __device__ __forceinline__ uint32_t find(uint32_t node) const {
        uint32_t s = slot0(node);
        for (;;) {
            const uint4 e = hash[s];
            if (e.x != tag) return hmask + 1u + s;
            if ((e.y & ~kTgtBit) == node) return s;
            s = (s + 1u) & hmask;
        }
    }
    __device__ __forceinline__ uint64_t get(uint32_t node) const {
        const uint32_t s = find(node);
        if (s > hmask) return kInf;
        const uint4 e = hash[s];
        return ((uint64_t)e.w << 32) | e.z;
    }
    // set dist of node (inserted if absent, keeping a target bit)
    __device__ __forceinline__ void set_at(uint32_t s, uint32_t node, uint64_t d) {
        if (s > hmask) {
            s -= hmask + 1u;
            if (++hn > hcap_fill) {
                ovf = true;
                return;
            }
            hash[s] = make_uint4(tag, node, (uint32_t)d, (uint32_t)(d >> 32));
            return;
        }
        uint4 e = hash[s];
        e.z = (uint32_t)d;
        e.w = (uint32_t)(d >> 32);
        hash[s] = e;
    }
    __device__ __forceinline__ static uint64_t hd(uint4 e) { return ((uint64_t)e.y << 32) | e.x; }
    // libstdc++ __push_heap(first, hole, 0, value) with comp(a, b) = a.d > b.d
    __device__ __forceinline__ void sift_up(int64_t hole, uint4 value) {
        const uint64_t vd = hd(value);
        int64_t parent = (hole - 1) / 2;
        while (hole > 0) {
            const uint4 p = heap[parent];
            if (!(hd(p) > vd)) break;
            heap[hole] = p;
            hole = parent;
            parent = (hole - 1) / 2;
        }
        heap[hole] = value;
    }
    __device__ __forceinline__ void push(uint64_t d, uint32_t node) {
        if (L >= heap_cap) {
            ovf = true;
            return;
        }
        const uint4 value = make_uint4((uint32_t)d, (uint32_t)(d >> 32), node, 0u);
        ++L;
        sift_up((int64_t)L - 1, value);
    }
    // std::pop_heap + back() + pop_back()
    __device__ __forceinline__ uint4 pop() {
        if (L > 1) {
            const int64_t len = (int64_t)L - 1;
            const uint4 value = heap[len];
            heap[len] = heap[0];
            int64_t hole = 0, second = 0;
            const int64_t lim = (len - 1) / 2;
            // libstdc++'s descent, two levels per round trip: a step loads
            // the two children of the hole and their four children together
            // (the lane's heap is private: nothing else writes it meanwhile)
            while (second < lim) {
                const int64_t c = 2 * (second + 1);
                const uint4 a0 = heap[c - 1], a1 = heap[c];
                uint4 gc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int64_t gi = 2 * c - 1 + q;
                    gc[q] = gi < len ? heap[gi] : make_uint4(0u, 0u, 0u, 0u);
                }
                second = c;
                uint4 up = a1;
                if (hd(a1) > hd(a0)) {
                    --second;
                    up = a0;
                }
                heap[hole] = up;
                hole = second;
                if (!(second < lim)) break;
                const int64_t c2 = 2 * (second + 1);
                const bool left = second == c - 1;
                const uint4 b0 = left ? gc[0] : gc[2], b1 = left ? gc[1] : gc[3];
                second = c2;
                up = b1;
                if (hd(b1) > hd(b0)) {
                    --second;
                    up = b0;
                }
                heap[hole] = up;
                hole = second;
            }
            if ((len & 1) == 0 && second == (len - 2) / 2) {
                second = 2 * (second + 1);
                heap[hole] = heap[second - 1];
                hole = second - 1;
            }
            sift_up(hole, value);
        }
        --L;
        return heap[L];
    }
};

__global__ __launch_bounds__(256) void k_witness(
    const uint4* __restrict__ pairs, const uint32_t* __restrict__ plist, uint32_t np, Overlay g,
    const uint8_t* __restrict__ state, uint32_t contract, uint32_t settle, uint8_t* ws,
    WitnessCaps caps, uint64_t lane_bytes, uint32_t tag_base, uint32_t step_cap,
    uint4* __restrict__ slots, uint32_t* __restrict__ sflag, uint32_t* __restrict__ sc,
    uint32_t* __restrict__ ovf, uint32_t* __restrict__ ovf_n, uint32_t* __restrict__ err) {
    const uint32_t lane = gid();
    const uint32_t stride = gridDim.x * blockDim.x;
    uint8_t* base = ws + lane_bytes * lane;
    Lane W;
    W.hash = reinterpret_cast<uint4*>(base);
    W.heap = W.hash + caps.hash;
    W.tgt = W.heap + caps.heap;
    W.tset = reinterpret_cast<uint32_t*>(W.tgt + caps.tgt);
    W.hmask = caps.hash - 1u;
    W.hcap_fill = caps.hash - caps.hash / 4u;
    W.heap_cap = caps.heap;
    const uint2* arcs = reinterpret_cast<const uint2*>(g.arcs);
    for (uint32_t i = lane; i < np; i += stride) {
        const uint32_t p = plist ? plist[i] : i;
        const uint4 pr = pairs[p];
        const uint32_t v = pr.x;
        const uint2 a = arcs[g.ioff[v] + pr.y];  // (u, w(u, v))
        const uint32_t oo = g.ooff[v], od = g.odeg[v];
        W.tag = tag_base + i + 1u;  // never 0: the workspace starts zeroed
        W.hn = 0;
        W.L = 0;
        W.ovf = false;
        // targets (via, x) for x in out(v) \ {u}, via descending (insertion sort)
        uint32_t T = 0;
        for (uint32_t k = 0; k < od; ++k) {
            const uint2 b = arcs[oo + k];
            if (b.x == a.x) continue;
            if (T >= caps.tgt) {
                W.ovf = true;
                break;
            }
            const uint64_t via = (uint64_t)a.y + b.y;
            int64_t j = T;
            while (j > 0) {
                const uint4 t = W.tgt[j - 1];
                const uint64_t tv = ((uint64_t)t.y << 32) | t.x;
                if (tv > via || (tv == via && t.z < b.x)) break;
                W.tgt[j] = t;
                --j;
            }
            W.tgt[j] = make_uint4((uint32_t)via, (uint32_t)(via >> 32), b.x, 0u);
            ++T;
        }
        if (!W.ovf && T) {
            for (uint32_t j = 0; j < T && !W.ovf; ++j) {  // tstamp[t] = cur
                W.tset[j] = 0;
                const uint32_t x = W.tgt[j].z;
                const uint32_t s = W.find(x);  // absent: targets are distinct
                if (++W.hn > W.hcap_fill) {
                    W.ovf = true;
                    break;
                }
                W.hash[s - (W.hmask + 1u)] = make_uint4(W.tag, x | kTgtBit, 0xFFFFFFFFu, 0xFFFFFFFFu);
            }
            if (!W.ovf) {
                W.set_at(W.find(a.x), a.x, 0);
                W.push(0, a.x);
            }
            uint32_t settled = 0, open = 0, steps = 0;
            while (W.L && !W.ovf) {
                // a search past step_cap pops + relaxations is handed on
                // (ovf) to a wave, so that no lane holds its wave for long
                if (++steps > step_cap) {
                    W.ovf = true;
                    break;
                }
                const uint4 top = W.pop();
                const uint64_t d = Lane::hd(top);
                const uint32_t x = top.z;
                const uint32_t sx = W.find(x);
                const uint4 ex = W.hash[sx];  // x is present: it was pushed
                if (d != (((uint64_t)ex.w << 32) | ex.z)) continue;
                if (open == T) break;
                const uint64_t vo = ((uint64_t)W.tgt[open].y << 32) | W.tgt[open].x;
                if (d > vo || ++settled > settle) break;
                if (ex.y & kTgtBit) {  // a target settles
                    for (uint32_t j = 0; j < T; ++j)
                        if (W.tgt[j].z == x) {
                            if (!W.tset[j]) {
                                W.tset[j] = 1;
                                while (open < T && W.tset[open]) ++open;
                            }
                            break;
                        }
                }
                const uint32_t dx = g.odeg[x];
                steps += dx;
                // arcs in groups of kRelax: the group's arcs, avoid flags and
                // home hash slots are loaded together (independent: the arcs
                // of one list name distinct nodes), then applied in arc order
                // — the sequential search's sets and pushes, in its order
                const uint32_t o = g.ooff[x];
                for (uint32_t k0 = 0; k0 < dx && !W.ovf; k0 += kRelax) {
                    const uint32_t kn = min(kRelax, dx - k0);
                    uint2 e[kRelax];
                    bool live[kRelax];
#pragma unroll
                    for (uint32_t j = 0; j < kRelax; ++j)
                        e[j] = j < kn ? arcs[o + k0 + j] : make_uint2(v, 0u);
#pragma unroll
                    for (uint32_t j = 0; j < kRelax; ++j)
                        live[j] = e[j].x != v && !(contract && state[e[j].x] == 1);
                    uint4 h[kRelax];
#pragma unroll
                    for (uint32_t j = 0; j < kRelax; ++j)
                        h[j] = live[j] ? W.hash[W.slot0(e[j].x)] : make_uint4(0u, 0u, 0u, 0u);
                    uint32_t ins[kRelax];  // slots inserted by this group
                    uint32_t nins = 0;
                    for (uint32_t j = 0; j < kn; ++j) {
                        if (!live[j]) continue;
                        const uint32_t y = e[j].x;
                        // resolve the probe from the preloaded home entry
                        uint32_t sy = W.slot0(y);
                        uint4 ey = h[j];
                        bool present = false;
                        for (;;) {
                            bool taken = ey.x == W.tag;
                            if (!taken)  // free when loaded: an insert of this group may have taken it
                                for (uint32_t q = 0; q < nins; ++q) taken |= ins[q] == sy;
                            if (!taken) break;
                            if (ey.x == W.tag && (ey.y & ~kTgtBit) == y) {
                                present = true;
                                break;
                            }
                            sy = (sy + 1u) & W.hmask;
                            ey = W.hash[sy];
                        }
                        const uint64_t nd = d + e[j].y;
                        const uint64_t cur = present ? (((uint64_t)ey.w << 32) | ey.z) : kInf;
                        if (nd < cur) {
                            if (present) {
                                W.set_at(sy, y, nd);
                            } else {
                                W.set_at(W.hmask + 1u + sy, y, nd);
                                ins[nins++] = sy;
                            }
                            W.push(nd, y);
                            if (W.ovf) break;
                        }
                    }
                }
            }
        }
        if (W.ovf) {
            ovf[atomicAdd(ovf_n, 1u)] = p;
            continue;
        }
        uint32_t count = 0;
        for (uint32_t k = 0; k < od; ++k) {
            const uint2 b = arcs[oo + k];
            bool need = false;
            uint64_t via = 0;
            if (b.x != a.x) {
                via = (uint64_t)a.y + b.y;
                need = !(W.get(b.x) <= via);
            }
            count += need;
            if (contract) {
                if (need && via >= 0xFFFFFFFFull) atomicOr(err, 1u);
                slots[pr.z + k] = need ? make_uint4(a.x, b.x, (uint32_t)via, 1u) : make_uint4(0, 0, 0, 0);
                sflag[pr.z + k] = need;
            }
        }
        if (!contract && count) atomicAdd(&sc[v], count);
    }
}

// ---------------------------------------------------------------------------
// Wave-cooperative witness search (the core rounds: few searches, high
// degrees, hundreds of settled nodes each).  One wave per search, hash and
// heap in LDS.  The heap operations are the lane search's (every lane runs
// them in step on the same LDS words), while the arcs of a settled node are
// relaxed one per lane: their hash probes and inserts run in parallel (the
// arcs of one list name distinct nodes, so no two lanes touch one key, and
// 64-bit compare-and-swap of (tag, node) claims free slots), and the
// improving arcs are then pushed in arc order — the host's push order, so
// the heap, and every tie it breaks, stays the host's.
// LDS of one wave's search: kWH hash slots, kWP heap slots, kWT targets
// (two sizes: 27 KB, five workgroups per CU, then 55 KB for what outgrows it)
template <uint32_t kWH, uint32_t kWP, uint32_t kWT>
struct WaveLds {
    unsigned long long key[kWH];  // (node | target bit) << 32 | tag
    unsigned long long hdist[kWH];
    unsigned long long pd[kWP];  // heap: dist
    uint32_t pn[kWP];            //       node
    unsigned long long tv[kWT];  // targets: via (descending), node, settled
    uint32_t tn[kWT];
    uint32_t ts[kWT];
    uint32_t hn, ovf;
};

template <uint32_t kWH>
__device__ __forceinline__ uint32_t wslot0(uint32_t node) { return (node * 0x9E3779B1u) & (kWH - 1u); }

// probe for node (tag): slot index, found flag
template <uint32_t kWH, uint32_t kWP, uint32_t kWT>
__device__ __forceinline__ uint32_t wfind(const WaveLds<kWH, kWP, kWT>& S, uint32_t node, uint32_t tag,
                                          bool& found) {
    uint32_t s = wslot0<kWH>(node);
    for (;;) {
        const unsigned long long k = S.key[s];
        if ((uint32_t)k != tag) {
            found = false;
            return s;
        }
        if (((uint32_t)(k >> 32) & ~kTgtBit) == node) {
            found = true;
            return s;
        }
        s = (s + 1u) & (kWH - 1u);
    }
}

// insert an absent node (parallel-safe for distinct nodes): the slot, or
// kWH when the table is full
template <uint32_t kWH, uint32_t kWP, uint32_t kWT>
__device__ __forceinline__ uint32_t winsert(WaveLds<kWH, kWP, kWT>& S, uint32_t nodebits, uint32_t tag,
                                            uint32_t s) {
    const unsigned long long mine = ((unsigned long long)nodebits << 32) | tag;
    for (uint32_t probes = 0; probes < kWH; ++probes) {
        const unsigned long long k = S.key[s];
        if ((uint32_t)k != tag) {
            if (atomicCAS(&S.key[s], k, mine) == k) {
                if (atomicAdd(&S.hn, 1u) + 1u > kWH - kWH / 4u) S.ovf = 1u;
                return s;
            }
            continue;  // lost the slot: look at it again
        }
        s = (s + 1u) & (kWH - 1u);
    }
    S.ovf = 1u;
    return kWH;
}

template <uint32_t kWH, uint32_t kWP, uint32_t kWT>
__device__ __forceinline__ void wsift_up(WaveLds<kWH, kWP, kWT>& S, int64_t hole, unsigned long long vd,
                                         uint32_t vn) {
    int64_t parent = (hole - 1) / 2;
    while (hole > 0) {
        const unsigned long long p = S.pd[parent];
        if (!(p > vd)) break;
        S.pd[hole] = p;
        S.pn[hole] = S.pn[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    S.pd[hole] = vd;
    S.pn[hole] = vn;
}

template <uint32_t kWH, uint32_t kWP, uint32_t kWT>
__global__ __launch_bounds__(64) void k_witness_wave(
    const uint4* __restrict__ pairs, const uint32_t* __restrict__ plist, uint32_t np, Overlay g,
    const uint8_t* __restrict__ state, uint32_t contract, uint32_t settle, uint4* __restrict__ slots,
    uint32_t* __restrict__ sflag, uint32_t* __restrict__ sc, uint32_t* __restrict__ ovf,
    uint32_t* __restrict__ ovf_n, uint32_t* __restrict__ err) {
    extern __shared__ unsigned long long lds_raw[];
    using WL = WaveLds<kWH, kWP, kWT>;
    WL& S = *reinterpret_cast<WL*>(lds_raw);
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < kWH; i += 64u) S.key[i] = 0ull;  // tag 0: empty
    const uint2* arcs = reinterpret_cast<const uint2*>(g.arcs);
    for (uint32_t i = blockIdx.x; i < np; i += gridDim.x) {
        const uint32_t p = plist ? plist[i] : i;
        const uint4 pr = pairs[p];
        const uint32_t v = pr.x;
        const uint2 a = arcs[g.ioff[v] + pr.y];  // (u, w(u, v))
        const uint32_t oo = g.ooff[v], od = g.odeg[v];
        const uint32_t tag = i + 1u;
        if (lane == 0) {
            S.hn = 0;
            S.ovf = 0;
        }
        __syncthreads();
        // targets: out(v) \ {u}, via descending (rank of each by counting)
        uint32_t T = 0;
        for (uint32_t k0 = 0; k0 < od; k0 += 64u) {
            const uint32_t k = k0 + lane;
            const bool on = k < od && arcs[oo + k].x != a.x;
            const unsigned long long m = __ballot(on);
            if (on) {
                const uint2 b = arcs[oo + k];
                const uint32_t j = T + __popcll(m & ((1ull << lane) - 1ull));
                if (j < kWT) {
                    S.tv[j] = (unsigned long long)a.y + b.y;
                    S.tn[j] = b.x;
                    S.ts[j] = 0;
                }
            }
            T += __popcll(m);
        }
        __syncthreads();
        bool bad = T > kWT;
        if (!bad && T) {
            // sort (via desc, node asc) by rank: T <= 128, two entries per lane
            unsigned long long rv[2];
            uint32_t rn[2], rk[2];
            for (int h = 0; h < 2; ++h) {
                const uint32_t j = lane + 64u * h;
                rk[h] = 0xFFFFFFFFu;
                if (j < T) {
                    rv[h] = S.tv[j];
                    rn[h] = S.tn[j];
                    uint32_t r = 0;
                    for (uint32_t q = 0; q < T; ++q) {
                        const unsigned long long qv = S.tv[q];
                        r += qv > rv[h] || (qv == rv[h] && S.tn[q] < rn[h]);
                    }
                    rk[h] = r;
                }
            }
            __syncthreads();
            for (int h = 0; h < 2; ++h)
                if (rk[h] != 0xFFFFFFFFu) {
                    S.tv[rk[h]] = rv[h];
                    S.tn[rk[h]] = rn[h];
                }
            __syncthreads();
            // tstamp: every target enters the table unreached
            for (uint32_t j = lane; j < T; j += 64u) {
                bool f;
                const uint32_t s = wfind(S, S.tn[j], tag, f);
                const uint32_t s2 = winsert(S, S.tn[j] | kTgtBit, tag, s);
                if (s2 < kWH) S.hdist[s2] = ~0ull;
            }
            __syncthreads();
            if (lane == 0) {
                bool f;
                const uint32_t s = wfind(S, a.x, tag, f);
                const uint32_t s2 = winsert(S, a.x, tag, s);
                if (s2 < kWH) S.hdist[s2] = 0ull;
            }
            __syncthreads();
            bad = S.ovf != 0u;
            uint32_t L = 0;
            if (!bad) {
                S.pd[0] = 0ull;  // every lane writes the same words
                S.pn[0] = a.x;
                L = 1;
            }
            uint32_t settled = 0, open = 0;
            while (L && !bad) {
                // pop (std::pop_heap + back + pop_back), in step on every lane
                if (L > 1) {
                    const int64_t len = (int64_t)L - 1;
                    const unsigned long long vd = S.pd[len];
                    const uint32_t vn = S.pn[len];
                    const unsigned long long td = S.pd[0];
                    const uint32_t tn0 = S.pn[0];
                    __syncthreads();
                    S.pd[len] = td;
                    S.pn[len] = tn0;
                    int64_t hole = 0, second = 0;
                    while (second < (len - 1) / 2) {
                        second = 2 * (second + 1);
                        if (S.pd[second] > S.pd[second - 1]) --second;
                        const unsigned long long cd = S.pd[second];
                        const uint32_t cn = S.pn[second];
                        __syncthreads();
                        S.pd[hole] = cd;
                        S.pn[hole] = cn;
                        hole = second;
                    }
                    if ((len & 1) == 0 && second == (len - 2) / 2) {
                        second = 2 * (second + 1);
                        const unsigned long long cd = S.pd[second - 1];
                        const uint32_t cn = S.pn[second - 1];
                        __syncthreads();
                        S.pd[hole] = cd;
                        S.pn[hole] = cn;
                        hole = second - 1;
                    }
                    __syncthreads();
                    wsift_up(S, hole, vd, vn);
                }
                __syncthreads();
                --L;
                const unsigned long long d = S.pd[L];
                const uint32_t x = S.pn[L];
                bool fx;
                const uint32_t sx = wfind(S, x, tag, fx);
                const unsigned long long kx = S.key[sx];
                if (d != S.hdist[sx]) continue;
                if (open == T) break;
                if (d > S.tv[open] || ++settled > settle) break;
                if ((uint32_t)(kx >> 32) & kTgtBit) {  // a target settles
                    for (uint32_t j = 0; j < T; ++j)
                        if (S.tn[j] == x) {
                            if (!S.ts[j]) {
                                __syncthreads();
                                if (lane == 0) S.ts[j] = 1u;
                                __syncthreads();
                                while (open < T && S.ts[open]) ++open;
                            }
                            break;
                        }
                }
                const uint32_t ox = g.ooff[x], dx = g.odeg[x];
                for (uint32_t k0 = 0; k0 < dx && !bad; k0 += 64u) {
                    const uint32_t k = k0 + lane;
                    bool imp = false;
                    unsigned long long nd = 0;
                    uint32_t y = 0;
                    if (k < dx) {
                        const uint2 e = arcs[ox + k];
                        y = e.x;
                        if (!(e.x == v || (contract && state[e.x] == 1))) {
                            nd = d + e.y;
                            bool f;
                            const uint32_t s = wfind(S, e.x, tag, f);
                            if (!f || nd < S.hdist[s]) {
                                imp = true;
                                if (f) {
                                    S.hdist[s] = nd;
                                } else {
                                    const uint32_t s2 = winsert(S, e.x, tag, s);
                                    if (s2 < kWH) S.hdist[s2] = nd;
                                }
                            }
                        }
                    }
                    __syncthreads();
                    bad = S.ovf != 0u;
                    unsigned long long m = __ballot(imp);
                    if (!bad && L + __popcll(m) > kWP) bad = true;
                    while (m && !bad) {  // pushes in arc order, in step on every lane
                        const uint32_t j = __builtin_ctzll(m);
                        m &= m - 1ull;
                        const unsigned long long jd = __shfl(nd, j, 64);
                        const uint32_t jn = __shfl(y, j, 64);
                        ++L;
                        wsift_up(S, (int64_t)L - 1, jd, jn);
                        __syncthreads();
                    }
                }
            }
        }
        if (bad) {
            if (lane == 0) ovf[atomicAdd(ovf_n, 1u)] = p;
            __syncthreads();
            continue;
        }
        uint32_t count = 0;
        for (uint32_t k0 = 0; k0 < od; k0 += 64u) {
            const uint32_t k = k0 + lane;
            bool need = false;
            if (k < od) {
                const uint2 b = arcs[oo + k];
                unsigned long long via = 0;
                if (b.x != a.x) {
                    via = (unsigned long long)a.y + b.y;
                    bool f;
                    const uint32_t s = wfind(S, b.x, tag, f);
                    need = !(f && S.hdist[s] <= via);
                }
                if (contract) {
                    if (need && via >= 0xFFFFFFFFull) atomicOr(err, 1u);
                    slots[pr.z + k] = need ? make_uint4(a.x, b.x, (uint32_t)via, 1u) : make_uint4(0, 0, 0, 0);
                    sflag[pr.z + k] = need;
                }
            }
            count += __popcll(__ballot(need));
        }
        if (!contract && count && lane == 0) atomicAdd(&sc[v], count);
        __syncthreads();
    }
}

__global__ void k_record(const uint32_t* __restrict__ S, uint32_t nS, uint32_t rank0, Overlay g,
                         const uint32_t* __restrict__ upos, const uint32_t* __restrict__ dpos,
                         uint64_t ubase, uint64_t dbase, uint32_t* __restrict__ rank,
                         uint32_t* __restrict__ rec_v, uint64_t* __restrict__ rec_uo,
                         uint32_t* __restrict__ rec_un, uint64_t* __restrict__ rec_do,
                         uint32_t* __restrict__ rec_dn, uint2* __restrict__ upool,
                         uint2* __restrict__ dpool, uint32_t* deleted, uint32_t* depth,
                         uint32_t* aff, uint8_t* state) {
    const uint32_t i = gid();
    if (i >= nS) return;
    const uint32_t v = S[i], r = rank0 + i;
    const uint2* arcs = reinterpret_cast<const uint2*>(g.arcs);
    rank[v] = r;
    rec_v[r] = v;
    const uint32_t oo = g.ooff[v], od = g.odeg[v], io = g.ioff[v], id = g.ideg[v];
    const uint64_t uo = ubase + upos[i], dn = dbase + dpos[i];
    rec_uo[r] = uo;
    rec_un[r] = od;
    rec_do[r] = dn;
    rec_dn[r] = id;
    const uint32_t dv = depth[v] + 1u;  // v's depth is not written this round
    for (uint32_t k = 0; k < od; ++k) {
        const uint2 e = arcs[oo + k];
        upool[uo + k] = e;
        atomicAdd(&deleted[e.x], 1u);
        atomicMax(&depth[e.x], dv);
        aff[e.x] = 1u;
    }
    for (uint32_t k = 0; k < id; ++k) {
        const uint2 e = arcs[io + k];
        dpool[dn + k] = e;
        atomicAdd(&deleted[e.x], 1u);
        atomicMax(&depth[e.x], dv);
        aff[e.x] = 1u;
    }
    state[v] = 2;
}

__global__ void k_compact_shortcuts(const uint4* __restrict__ slots, const uint32_t* __restrict__ sflag,
                                    const uint32_t* __restrict__ spos, uint32_t nslots,
                                    uint4* __restrict__ sc, uint32_t* cnt_o, uint32_t* cnt_i,
                                    uint32_t* aff) {
    const uint32_t i = gid();
    if (i >= nslots || !sflag[i]) return;
    const uint4 e = slots[i];
    sc[spos[i]] = make_uint4(e.x, e.y, e.z, 0u);
    atomicAdd(&cnt_o[e.x], 1u);
    atomicAdd(&cnt_i[e.y], 1u);
    aff[e.x] = 1u;
    aff[e.y] = 1u;
}

__global__ void k_aff_counts(const uint32_t* __restrict__ A, uint32_t nA, Overlay g,
                             const uint32_t* __restrict__ cnt_o, const uint32_t* __restrict__ cnt_i,
                             uint32_t* c0, uint32_t* c1, uint32_t* c2, uint32_t* c3) {
    const uint32_t i = gid();
    if (i > nA) return;
    if (i == nA) {
        c0[i] = c1[i] = c2[i] = c3[i] = 0;
        return;
    }
    const uint32_t u = A[i];
    c0[i] = g.odeg[u] + cnt_o[u];
    c1[i] = g.ideg[u] + cnt_i[u];
    c2[i] = cnt_o[u];
    c3[i] = cnt_i[u];
}

__global__ void k_bucket_starts(const uint32_t* __restrict__ A, uint32_t nA,
                                const uint32_t* __restrict__ s2, const uint32_t* __restrict__ s3,
                                uint32_t* bo_o, uint32_t* bo_i) {
    const uint32_t i = gid();
    if (i >= nA) return;
    const uint32_t u = A[i];
    bo_o[u] = s2[i];
    bo_i[u] = s3[i];
}

__global__ void k_fill_buckets(const uint4* __restrict__ sc, uint32_t nsc,
                               const uint32_t* __restrict__ bo_o, const uint32_t* __restrict__ bo_i,
                               uint32_t* cur_o, uint32_t* cur_i, uint2* __restrict__ bucket_o,
                               uint2* __restrict__ bucket_i) {
    const uint32_t i = gid();
    if (i >= nsc) return;
    const uint4 e = sc[i];  // (u, x, w)
    bucket_o[bo_o[e.x] + atomicAdd(&cur_o[e.x], 1u)] = make_uint2(e.y, e.z);
    bucket_i[bo_i[e.y] + atomicAdd(&cur_i[e.y], 1u)] = make_uint2(e.x, e.z);
}

// old list (minus done nodes) merged with the sorted bucket, lightest per key
__device__ uint32_t merge_one(const uint2* old, uint32_t nold, uint2* bk, uint32_t nb,
                              const uint8_t* state, uint2* out) {
    for (uint32_t j = 1; j < nb; ++j) {  // insertion sort by (key, w)
        const uint2 x = bk[j];
        uint32_t k = j;
        while (k > 0) {
            const uint2 y = bk[k - 1];
            if (y.x < x.x || (y.x == x.x && y.y <= x.y)) break;
            bk[k] = y;
            --k;
        }
        bk[k] = x;
    }
    uint32_t n = 0, i = 0, j = 0;
    while (true) {
        while (i < nold && state[old[i].x] == 2) ++i;
        const bool hi = i < nold, hj = j < nb;
        if (!hi && !hj) break;
        uint2 e;
        if (hi && (!hj || old[i].x < bk[j].x)) {
            e = old[i++];
        } else if (!hi || bk[j].x < old[i].x) {
            e = bk[j++];
        } else {  // same neighbour: the lighter arc
            e = old[i++];
            e.y = min(e.y, bk[j].y);
            ++j;
        }
        while (j < nb && bk[j].x == e.x) ++j;  // heavier duplicates of this key
        out[n++] = e;
    }
    return n;
}

__global__ void k_merge(const uint32_t* __restrict__ A, uint32_t nA, uint32_t* ooff, uint32_t* odeg,
                        uint32_t* ioff, uint32_t* ideg, uint2* arcs, const uint8_t* __restrict__ state,
                        const uint32_t* __restrict__ s0, const uint32_t* __restrict__ s1,
                        uint32_t obase, uint32_t ibase, const uint32_t* __restrict__ bo_o,
                        const uint32_t* __restrict__ bo_i, const uint32_t* __restrict__ cnt_o,
                        const uint32_t* __restrict__ cnt_i, uint2* bucket_o, uint2* bucket_i,
                        uint32_t* maxdeg) {
    const uint32_t t = gid();
    if (t >= 2u * nA) return;
    const uint32_t i = t >> 1;
    const uint32_t u = A[i];
    uint32_t d;
    if (t & 1u) {
        const uint32_t no = ibase + s1[i];
        d = merge_one(arcs + ioff[u], ideg[u], bucket_i + bo_i[u], cnt_i[u], state, arcs + no);
        ioff[u] = no;
        ideg[u] = d;
    } else {
        const uint32_t no = obase + s0[i];
        d = merge_one(arcs + ooff[u], odeg[u], bucket_o + bo_o[u], cnt_o[u], state, arcs + no);
        ooff[u] = no;
        odeg[u] = d;
    }
    atomicMax(maxdeg, d);
}

__global__ void k_sim_counts(const uint32_t* __restrict__ list, uint32_t k, Overlay g, uint32_t* c0,
                             uint32_t* sc) {
    const uint32_t i = gid();
    if (i > k) return;
    if (i == k) {
        c0[i] = 0;
        return;
    }
    const uint32_t u = list[i];
    c0[i] = g.odeg[u] ? g.ideg[u] : 0u;
    sc[u] = 0;
}

__global__ void k_prio(const uint32_t* __restrict__ list, uint32_t k, Overlay g,
                       const uint32_t* __restrict__ sc, const uint32_t* __restrict__ deleted,
                       const uint32_t* __restrict__ depth, int64_t a, int64_t b, int64_t c,
                       int64_t* prio, uint32_t* aff, uint32_t* cnt_o, uint32_t* cnt_i,
                       uint32_t* cur_o, uint32_t* cur_i) {
    const uint32_t i = gid();
    if (i >= k) return;
    const uint32_t u = list[i];
    const int64_t ed = (int64_t)sc[u] - (int64_t)g.ideg[u] - (int64_t)g.odeg[u];
    prio[u] = a * ed + b * (int64_t)deleted[u] + c * (int64_t)depth[u];
    aff[u] = 0;
    cnt_o[u] = cnt_i[u] = cur_o[u] = cur_i[u] = 0;
}

__global__ void k_compact_lists(const uint32_t* __restrict__ list, uint32_t k, uint32_t* ooff,
                                const uint32_t* __restrict__ odeg, uint32_t* ioff,
                                const uint32_t* __restrict__ ideg, const uint2* __restrict__ old,
                                uint2* __restrict__ nw, const uint32_t* __restrict__ s0,
                                const uint32_t* __restrict__ s1, uint32_t ibase) {
    const uint32_t i = gid();
    if (i >= k) return;
    const uint32_t u = list[i];
    const uint32_t o = ooff[u], no = s0[i];
    for (uint32_t j = 0, d = odeg[u]; j < d; ++j) nw[no + j] = old[o + j];
    ooff[u] = no;
    const uint32_t io = ioff[u], nio = ibase + s1[i];
    for (uint32_t j = 0, d = ideg[u]; j < d; ++j) nw[nio + j] = old[io + j];
    ioff[u] = nio;
}

__global__ void k_deg_counts(const uint32_t* __restrict__ list, uint32_t k, Overlay g, uint32_t* c0,
                             uint32_t* c1) {
    const uint32_t i = gid();
    if (i > k) return;
    if (i == k) {
        c0[i] = c1[i] = 0;
        return;
    }
    const uint32_t u = list[i];
    c0[i] = g.odeg[u];
    c1[i] = g.ideg[u];
}

__global__ void k_gather_flag(const uint32_t* __restrict__ list, uint32_t k,
                              const uint32_t* __restrict__ f, uint32_t* __restrict__ flag) {
    const uint32_t i = gid();
    if (i > k) return;
    flag[i] = i == k ? 0u : (f[list[i]] ? 1u : 0u);
}

inline dim3 grid_for(uint64_t n, uint32_t block = 256) {
    return dim3((uint32_t)((n + block - 1) / block));
}

}  // namespace

uint64_t witness_lane_bytes(WitnessCaps c) {
    const uint64_t b = 16ull * c.hash + 16ull * c.heap + 16ull * c.tgt + 4ull * c.tgt;
    return (b + 255ull) & ~255ull;
}

void scan_u32(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
              hipStream_t s) {
    (void)hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, in, out, (int)n, s);
}

void launch_pick(const uint32_t* rem, uint32_t R, Overlay g, const int64_t* prio, uint32_t* flag,
                 hipStream_t s) {
    hipLaunchKernelGGL(k_pick, grid_for(R + 1ull), dim3(256), 0, s, rem, R, g, prio, flag);
}

void launch_split(const uint32_t* in, const uint32_t* flag, const uint32_t* pos, uint32_t n,
                  uint32_t* sel, uint32_t* rej, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_split, grid_for(n), dim3(256), 0, s, in, flag, pos, n, sel, rej);
}

void launch_sel_counts(const uint32_t* S, uint32_t nS, Overlay g, uint8_t* state, uint32_t* c0,
                       uint32_t* c1, uint32_t* c2, uint32_t* c3, hipStream_t s) {
    hipLaunchKernelGGL(k_sel_counts, grid_for(nS + 1ull), dim3(256), 0, s, S, nS, g, state, c0,
                       c1, c2, c3);
}

void launch_make_pairs(const uint32_t* list, uint32_t k, Overlay g, const uint32_t* pbase,
                       const uint32_t* sbase, uint32_t* pairs, hipStream_t s) {
    if (!k) return;
    hipLaunchKernelGGL(k_make_pairs, grid_for(k), dim3(256), 0, s, list, k, g, pbase, sbase,
                       reinterpret_cast<uint4*>(pairs));
}

void launch_witness(const uint32_t* pairs, const uint32_t* plist, uint32_t np, Overlay g,
                    const uint8_t* state, bool contract, uint32_t settle, void* ws,
                    WitnessCaps caps, uint32_t lanes, uint32_t tag_base, uint32_t step_cap,
                    uint32_t* slots, uint32_t* sflag, uint32_t* sc, uint32_t* ovf,
                    uint32_t* ovf_n, uint32_t* err, hipStream_t s) {
    if (!np) return;
    // lanes: a multiple of 64 (whole waves; 256-thread blocks when it allows)
    const uint32_t l = std::min<uint32_t>(lanes, ((np + 63u) / 64u) * 64u);
    const uint32_t tpb = l % 256u == 0 ? 256u : 64u;
    hipLaunchKernelGGL(k_witness, dim3(l / tpb), dim3(tpb), 0, s,
                       reinterpret_cast<const uint4*>(pairs), plist, np, g, state,
                       contract ? 1u : 0u, settle, static_cast<uint8_t*>(ws), caps,
                       witness_lane_bytes(caps), tag_base, step_cap,
                       reinterpret_cast<uint4*>(slots), sflag, sc, ovf, ovf_n, err);
}

template <uint32_t H, uint32_t P, uint32_t T>
void launch_ww(const uint32_t* pairs, const uint32_t* plist, uint32_t np, Overlay g,
               const uint8_t* state, bool contract, uint32_t settle, uint32_t blocks,
               uint32_t* slots, uint32_t* sflag, uint32_t* sc, uint32_t* ovf, uint32_t* ovf_n,
               uint32_t* err, hipStream_t s) {
    auto k = k_witness_wave<H, P, T>;
    hipLaunchKernelGGL(k, dim3(std::min(np, blocks)), dim3(64), sizeof(WaveLds<H, P, T>), s,
                       reinterpret_cast<const uint4*>(pairs), plist, np, g, state,
                       contract ? 1u : 0u, settle, reinterpret_cast<uint4*>(slots), sflag, sc, ovf,
                       ovf_n, err);
}

void launch_witness_wave(const uint32_t* pairs, const uint32_t* plist, uint32_t np, Overlay g,
                         const uint8_t* state, bool contract, uint32_t settle, uint32_t blocks,
                         int size, uint32_t* slots, uint32_t* sflag, uint32_t* sc, uint32_t* ovf,
                         uint32_t* ovf_n, uint32_t* err, hipStream_t s) {
    if (!np) return;
    if (size == 0)
        launch_ww<512, 384, 32>(pairs, plist, np, g, state, contract, settle, blocks, slots,
                                sflag, sc, ovf, ovf_n, err, s);
    else if (size == 1)
        launch_ww<1024, 768, 64>(pairs, plist, np, g, state, contract, settle, blocks, slots,
                                 sflag, sc, ovf, ovf_n, err, s);
    else
        launch_ww<2048, 1792, 128>(pairs, plist, np, g, state, contract, settle, blocks, slots,
                                   sflag, sc, ovf, ovf_n, err, s);
}

uint32_t witness_wave_lds_bytes(int size) {
    return size == 0 ? (uint32_t)sizeof(WaveLds<512, 384, 32>)
           : size == 1 ? (uint32_t)sizeof(WaveLds<1024, 768, 64>)
                       : (uint32_t)sizeof(WaveLds<2048, 1792, 128>);
}

void launch_record(const uint32_t* S, uint32_t nS, uint32_t rank0, Overlay g, const uint32_t* upos,
                   const uint32_t* dpos, uint64_t ubase, uint64_t dbase, uint32_t* rank,
                   uint32_t* rec_v, uint64_t* rec_uo, uint32_t* rec_un, uint64_t* rec_do,
                   uint32_t* rec_dn, uint32_t* upool, uint32_t* dpool, uint32_t* deleted,
                   uint32_t* depth, uint32_t* aff, uint8_t* state, hipStream_t s) {
    if (!nS) return;
    hipLaunchKernelGGL(k_record, grid_for(nS), dim3(256), 0, s, S, nS, rank0, g, upos, dpos, ubase,
                       dbase, rank, rec_v, rec_uo, rec_un, rec_do, rec_dn,
                       reinterpret_cast<uint2*>(upool), reinterpret_cast<uint2*>(dpool), deleted,
                       depth, aff, state);
}

void launch_compact_shortcuts(const uint32_t* slots, const uint32_t* sflag, const uint32_t* spos,
                              uint32_t nslots, uint32_t* sc, uint32_t* cnt_o, uint32_t* cnt_i,
                              uint32_t* aff, hipStream_t s) {
    if (!nslots) return;
    hipLaunchKernelGGL(k_compact_shortcuts, grid_for(nslots), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(slots), sflag, spos, nslots,
                       reinterpret_cast<uint4*>(sc), cnt_o, cnt_i, aff);
}

void launch_aff_counts(const uint32_t* A, uint32_t nA, Overlay g, const uint32_t* cnt_o,
                       const uint32_t* cnt_i, uint32_t* c0, uint32_t* c1, uint32_t* c2,
                       uint32_t* c3, hipStream_t s) {
    hipLaunchKernelGGL(k_aff_counts, grid_for(nA + 1ull), dim3(256), 0, s, A, nA, g, cnt_o, cnt_i,
                       c0, c1, c2, c3);
}

void launch_bucket_starts(const uint32_t* A, uint32_t nA, const uint32_t* s2, const uint32_t* s3,
                          uint32_t* bo_o, uint32_t* bo_i, hipStream_t s) {
    if (!nA) return;
    hipLaunchKernelGGL(k_bucket_starts, grid_for(nA), dim3(256), 0, s, A, nA, s2, s3, bo_o, bo_i);
}

void launch_fill_buckets(const uint32_t* sc, uint32_t nsc, const uint32_t* bo_o,
                         const uint32_t* bo_i, uint32_t* cur_o, uint32_t* cur_i,
                         uint32_t* bucket_o, uint32_t* bucket_i, hipStream_t s) {
    if (!nsc) return;
    hipLaunchKernelGGL(k_fill_buckets, grid_for(nsc), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(sc), nsc, bo_o, bo_i, cur_o, cur_i,
                       reinterpret_cast<uint2*>(bucket_o), reinterpret_cast<uint2*>(bucket_i));
}

void launch_merge(const uint32_t* A, uint32_t nA, uint32_t* ooff, uint32_t* odeg, uint32_t* ioff,
                  uint32_t* ideg, uint32_t* arcs, const uint8_t* state, const uint32_t* s0,
                  const uint32_t* s1, uint32_t obase, uint32_t ibase, const uint32_t* bo_o,
                  const uint32_t* bo_i, const uint32_t* cnt_o, const uint32_t* cnt_i,
                  uint32_t* bucket_o, uint32_t* bucket_i, uint32_t* maxdeg, hipStream_t s) {
    if (!nA) return;
    hipLaunchKernelGGL(k_merge, grid_for(2ull * nA, 128), dim3(128), 0, s, A, nA, ooff, odeg, ioff,
                       ideg, reinterpret_cast<uint2*>(arcs), state, s0, s1, obase, ibase, bo_o,
                       bo_i, cnt_o, cnt_i, reinterpret_cast<uint2*>(bucket_o),
                       reinterpret_cast<uint2*>(bucket_i), maxdeg);
}

void launch_sim_counts(const uint32_t* list, uint32_t k, Overlay g, uint32_t* c0, uint32_t* sc,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_sim_counts, grid_for(k + 1ull), dim3(256), 0, s, list, k, g, c0, sc);
}

void launch_prio(const uint32_t* list, uint32_t k, Overlay g, const uint32_t* sc,
                 const uint32_t* deleted, const uint32_t* depth, int64_t a, int64_t b, int64_t c,
                 int64_t* prio, uint32_t* aff, uint32_t* cnt_o, uint32_t* cnt_i, uint32_t* cur_o,
                 uint32_t* cur_i, hipStream_t s) {
    if (!k) return;
    hipLaunchKernelGGL(k_prio, grid_for(k), dim3(256), 0, s, list, k, g, sc, deleted, depth, a, b,
                       c, prio, aff, cnt_o, cnt_i, cur_o, cur_i);
}

void launch_compact_lists(const uint32_t* list, uint32_t k, uint32_t* ooff, const uint32_t* odeg,
                          uint32_t* ioff, const uint32_t* ideg, const uint32_t* arcs_old,
                          uint32_t* arcs_new, const uint32_t* s0, const uint32_t* s1,
                          uint32_t ibase, hipStream_t s) {
    if (!k) return;
    hipLaunchKernelGGL(k_compact_lists, grid_for(k), dim3(256), 0, s, list, k, ooff, odeg, ioff,
                       ideg, reinterpret_cast<const uint2*>(arcs_old),
                       reinterpret_cast<uint2*>(arcs_new), s0, s1, ibase);
}

void launch_gather_flag(const uint32_t* list, uint32_t k, const uint32_t* f, uint32_t* flag,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_gather_flag, grid_for(k + 1ull), dim3(256), 0, s, list, k, f, flag);
}

void launch_deg_counts(const uint32_t* list, uint32_t k, Overlay g, uint32_t* c0, uint32_t* c1,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_deg_counts, grid_for(k + 1ull), dim3(256), 0, s, list, k, g, c0, c1);
}

}  // namespace chk
}  // namespace cpd

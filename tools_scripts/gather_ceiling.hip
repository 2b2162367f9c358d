// Microbenchmark: the chip's rate for the memory pattern
// of the table-search walk, with no CPD logic.  Each lane runs a dependent
// chain of hops; a hop loads one 4-B word from a large "move table" at an
// address that depends on the previous hop, and beside it the 32-B
// "adjacency row" at an address from the same value (the walk's co-fetch),
// then derives the next address from both.  Addresses are uniformly random:
// no locality at all (the real walk has some: ~0.17 new 128-B move line per
// hop).  Reports hops/s per wave count, i.e. the latency-bound rate of
// random dependent round trips at that concurrency.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools_scripts/bin/gather_ceiling tools_scripts/gather_ceiling.hip
//   tools_scripts/bin/gather_ceiling [table_GiB=10] [hops=512]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

__global__ void fill(uint32_t* t, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
        t[i] = (uint32_t)(z ^ (z >> 29));
    }
}

// mode 0: move word + 32-B adjacency per hop (the walk); 1: move word only
template <int MODE>
__global__ __launch_bounds__(256) void chain(const uint32_t* __restrict__ tab, uint64_t words,
                                             const uint4* __restrict__ adj, uint32_t adj_rows,
                                             uint32_t hops, uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;
    uint64_t x = (uint64_t)g * 0x9E3779B97F4A7C15ull;
    uint32_t acc = 0;
    for (uint32_t h = 0; h < hops; ++h) {
        const uint64_t wi = (x >> 11) % words;
        const uint32_t w = tab[wi];
        uint32_t a = 0;
        if (MODE == 0) {
            const uint4* p = adj + 2u * (uint32_t)((x >> 7) % adj_rows);
            const uint4 p0 = p[0], p1 = p[1];
            a = (w & 2u) ? p1.x ^ p1.z : p0.x ^ p0.z;
        }
        acc += w;
        x = (x ^ ((uint64_t)w << 17) ^ a) * 0xBF58476D1CE4E5B9ull + h;
    }
    out[g] = acc;
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 10.0;
    const uint32_t hops = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 512;
    const uint64_t words = (uint64_t)(gib * (1ull << 30) / 4);
    const uint32_t adj_rows = 1u << 20;  // 1M nodes x 32 B = 32 MiB, as at 1M nodes
    uint32_t *tab, *adj, *out;
    CK(hipMalloc(&tab, words * 4));
    CK(hipMalloc(&adj, (size_t)adj_rows * 32));
    CK(hipMalloc(&out, 8192u * 64u * 4u));
    fill<<<4096, 256>>>(tab, words, 1);
    fill<<<4096, 256>>>(adj, (size_t)adj_rows * 8, 2);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::printf("{\"table_GiB\": %.1f, \"hops_per_lane\": %u, \"results\": [", gib, hops);
    bool first = true;
    for (int mode = 0; mode < 2; ++mode)
        for (uint32_t waves : {256u, 512u, 1024u, 2048u, 4096u, 8192u}) {
            const dim3 grid(waves / 4u), blk(256);
            for (int rep = 0; rep < 2; ++rep) {  // first launch warms
                CK(hipEventRecord(a));
                if (mode == 0) chain<0><<<grid, blk>>>(tab, words, (const uint4*)adj, adj_rows, hops, out);
                else chain<1><<<grid, blk>>>(tab, words, (const uint4*)adj, adj_rows, hops, out);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
            }
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double h = (double)waves * 64.0 * hops;
            std::printf("%s{\"mode\": \"%s\", \"waves\": %u, \"ms\": %.3f, \"Ghops_per_s\": %.2f, "
                        "\"round_trip_ns\": %.0f}",
                        first ? "" : ", ", mode == 0 ? "move+adj" : "move", waves, ms,
                        h / (ms * 1e-3) / 1e9, ms * 1e6 / hops);
            first = false;
        }
    std::printf("]}\n");
    return 0;
}

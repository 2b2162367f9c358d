// HBM commit / release cost probe (round 4): how long do
// hipMalloc, the first write of the memory, hipFree, a pooled re-allocation
// and the virtual-memory API take for the tens-of-GB buffers a CPD worker
// allocates?  Build: hipcc -O2 --offload-arch=gfx950 alloc_probe.hip -o alloc_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

static double now() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

__global__ void fill(uint4* p, size_t n16) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += stride) p[i] = make_uint4(1u, 2u, 3u, (uint32_t)i);
}

static double touch(void* p, size_t bytes) {
    const double t0 = now();
    fill<<<8192, 256>>>(static_cast<uint4*>(p), bytes / 16);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    return now() - t0;
}

int main(int argc, char** argv) {
    const double gb = 1e9;
    size_t fr = 0, tot = 0;
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    CK(hipMemGetInfo(&fr, &tot));
    std::printf("free %.1f GB of %.1f GB\n", fr / gb, tot / gb);
    // 1. plain hipMalloc at several sizes: alloc, first touch, second touch, free
    for (size_t g : {1ull, 8ull, 32ull, 64ull, 128ull}) {
        const size_t bytes = g << 30;
        void* p = nullptr;
        double t0 = now();
        CK(hipMalloc(&p, bytes));
        const double ta = now() - t0;
        const double t1 = touch(p, bytes), t2 = touch(p, bytes);
        t0 = now();
        CK(hipFree(p));
        const double tf = now() - t0;
        std::printf("hipMalloc %4zu GiB: alloc %.3fs (%.0f GB/s) touch1 %.3fs touch2 %.3fs free %.3fs (%.0f GB/s)\n",
                    g, ta, bytes / ta / gb, t1, t2, tf, bytes / tf / gb);
        std::fflush(stdout);
    }
    // 2. many 8-GiB buffers (what a batch workspace looks like), freed together
    {
        std::vector<void*> v;
        double t0 = now();
        for (int i = 0; i < 16; ++i) {
            void* p = nullptr;
            CK(hipMalloc(&p, 8ull << 30));
            v.push_back(p);
        }
        const double ta = now() - t0;
        t0 = now();
        for (void* p : v) CK(hipFree(p));
        std::printf("16 x 8 GiB hipMalloc: alloc %.3fs free %.3fs\n", ta, now() - t0);
        std::fflush(stdout);
    }
    // 3. stream-ordered pool, release threshold = max: the second allocation of
    //    the same size is served from the pool
    {
        hipMemPool_t pool;
        CK(hipDeviceGetDefaultMemPool(&pool, 0));
        uint64_t thr = ~0ull;
        CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
        hipStream_t s;
        CK(hipStreamCreate(&s));
        for (int rep = 0; rep < 2; ++rep) {
            void* p = nullptr;
            const size_t bytes = 64ull << 30;
            double t0 = now();
            CK(hipMallocAsync(&p, bytes, s));
            CK(hipStreamSynchronize(s));
            const double ta = now() - t0;
            const double t1 = touch(p, bytes);
            t0 = now();
            CK(hipFreeAsync(p, s));
            CK(hipStreamSynchronize(s));
            std::printf("pool 64 GiB rep %d: alloc %.3fs touch %.3fs free %.3fs\n", rep, ta, t1,
                        now() - t0);
            std::fflush(stdout);
        }
        CK(hipMemPoolTrimTo(pool, 0));
        CK(hipStreamDestroy(s));
    }
    // 4. virtual memory API: reserve, create physical, map, set access
    {
        const size_t bytes = 64ull << 30;
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        size_t gran = 0;
        CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
        void* va = nullptr;
        double t0 = now();
        CK(hipMemAddressReserve(&va, bytes, 0, nullptr, 0));
        const double tr = now() - t0;
        hipMemGenericAllocationHandle_t h;
        t0 = now();
        CK(hipMemCreate(&h, bytes, &prop, 0));
        const double tc = now() - t0;
        t0 = now();
        CK(hipMemMap(va, bytes, 0, h, 0));
        const double tm = now() - t0;
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        t0 = now();
        CK(hipMemSetAccess(va, bytes, &acc, 1));
        const double ts = now() - t0;
        const double t1 = touch(va, bytes);
        t0 = now();
        CK(hipMemUnmap(va, bytes));
        CK(hipMemRelease(h));
        CK(hipMemAddressFree(va, bytes));
        std::printf("vmm 64 GiB (gran %zu): reserve %.3fs create %.3fs map %.3fs access %.3fs touch %.3fs release %.3fs\n",
                    gran, tr, tc, tm, ts, t1, now() - t0);
        std::fflush(stdout);
    }
    // 5. pinned host memory (make_cpd_auto's export buffers)
    for (size_t g : {1ull, 8ull}) {
        void* p = nullptr;
        double t0 = now();
        CK(hipHostMalloc(&p, g << 30, hipHostMallocDefault));
        const double ta = now() - t0;
        t0 = now();
        CK(hipHostFree(p));
        std::printf("hipHostMalloc %zu GiB: alloc %.3fs free %.3fs\n", g, ta, now() - t0);
        std::fflush(stdout);
    }
    // 6. hipMalloc of 200 GiB total as a single block vs touch (worker-sized)
    {
        void* p = nullptr;
        const size_t bytes = 200ull << 30;
        double t0 = now();
        hipError_t e = hipMalloc(&p, bytes);
        const double ta = now() - t0;
        if (e == hipSuccess) {
            const double t1 = touch(p, bytes);
            t0 = now();
            CK(hipFree(p));
            std::printf("hipMalloc 200 GiB: alloc %.3fs touch %.3fs free %.3fs\n", ta, t1, now() - t0);
        } else {
            std::printf("hipMalloc 200 GiB failed: %s\n", hipGetErrorString(e));
        }
    }
    return 0;
}

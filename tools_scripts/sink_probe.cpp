// Host sink probe for the end-to-end worker's bucket files: one 16-GiB file
// written by T threads in 64-MiB pieces at their final offsets, four ways —
//   pwrite          what make_cpd_auto does (writes to one file serialise on
//                   its inode)
//   mmap            ftruncate + a shared mapping, pieces memcpy'd in
//   mmap+populate   the same, each piece's pages populated first with
//                   MADV_POPULATE_WRITE (one call instead of a fault per page)
//   files           one file per thread (the ceiling: no shared inode)
// Prints GB/s per method.   g++ -O2 -pthread sink_probe.cpp -o sink_probe
//   ./sink_probe DIR [threads] [GiB]
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: sink_probe DIR [threads] [GiB]\n");
        return 2;
    }
    const std::string dir = argv[1];
    const int T = argc > 2 ? std::atoi(argv[2]) : 16;
    const size_t total = (argc > 3 ? std::atoll(argv[3]) : 16) << 30;
    const size_t piece = 64u << 20, npieces = total / piece;
    std::vector<std::vector<char>> src(T, std::vector<char>(piece));
    for (int t = 0; t < T; ++t)
        for (size_t i = 0; i < piece; i += 4096) src[t][i] = (char)(t + i);
    auto run = [&](const char* name, auto body) {
        std::atomic<size_t> next{0};
        const double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (size_t p; (p = next++) < npieces;) body(t, p);
            });
        for (auto& x : th) x.join();
        const double dt = now() - t0;
        std::printf("%-14s %2d threads %5.1f GiB  %6.3f s  %6.2f GB/s\n", name, T,
                    (double)total / (1 << 30), dt, (double)total / dt / 1e9);
        std::fflush(stdout);
    };
    const std::string f1 = dir + "/probe_one.bin";
    {
        int fd = ::open(f1.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        run("pwrite", [&](int t, size_t p) {
            if (::pwrite(fd, src[t].data(), piece, (off_t)(p * piece)) != (ssize_t)piece) std::abort();
        });
        ::close(fd);
        ::unlink(f1.c_str());
    }
    for (int populate = 0; populate < 2; ++populate) {
        int fd = ::open(f1.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
        if (::ftruncate(fd, (off_t)total) != 0) std::abort();
        char* m = static_cast<char*>(::mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
        if (m == MAP_FAILED) std::abort();
        run(populate ? "mmap+populate" : "mmap", [&](int t, size_t p) {
            char* d = m + p * piece;
            if (populate && ::madvise(d, piece, MADV_POPULATE_WRITE) != 0) std::abort();
            std::memcpy(d, src[t].data(), piece);
        });
        ::munmap(m, total);
        ::close(fd);
        ::unlink(f1.c_str());
    }
    {
        std::vector<int> fds(T);
        for (int t = 0; t < T; ++t)
            fds[t] = ::open((dir + "/probe_" + std::to_string(t) + ".bin").c_str(),
                            O_WRONLY | O_CREAT | O_TRUNC, 0644);
        std::vector<size_t> off(T, 0);
        run("files", [&](int t, size_t) {
            if (::pwrite(fds[t], src[t].data(), piece, (off_t)off[t]) != (ssize_t)piece) std::abort();
            off[t] += piece;
        });
        for (int t = 0; t < T; ++t) {
            ::close(fds[t]);
            ::unlink((dir + "/probe_" + std::to_string(t) + ".bin").c_str());
        }
    }
    return 0;
}

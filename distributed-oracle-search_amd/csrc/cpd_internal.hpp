// Internal declarations shared by the host C++ and the HIP translation unit.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>
#include <stdexcept>

#include "cpd_api.h"

namespace cpd {

// Error channel: every C entry point catches cpd::Error and maps it to a code.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& msg) : std::runtime_error(msg), code(c) {}
};

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define CPD_REQUIRE(cond, code, msg)                                         \
    do {                                                                     \
        if (!(cond)) throw ::cpd::Error((code), (msg));                      \
    } while (0)

// Run `body` and translate exceptions into CPD_E_* codes.
template <class F>
int guarded(F&& body) {
    try {
        body();
        return CPD_OK;
    } catch (const Error& e) {
        return fail(e.code, e.what());
    } catch (const std::bad_alloc&) {
        return fail(CPD_E_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(CPD_E_ARG, e.what());
    }
}

// Validate a CSR graph as the .xy loader would produce it.
void check_csr(uint32_t n, uint32_t m, const uint32_t* row_ptr,
               const uint32_t* dst, const uint32_t* w);

void dfs_preorder(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                  uint32_t* order);

// Contraction hierarchy, node space.  rank[v] = contraction position.
struct Hierarchy {
    std::vector<uint32_t> rank;
    std::vector<uint64_t> up_off, dn_off;      // CSR by tail node
    std::vector<uint32_t> up_dst, up_w;        // v -> x, rank x > rank v
    std::vector<uint32_t> dn_dst, dn_w;        // u -> v, rank v < rank u
    std::vector<uint32_t> level_up, level_dn;  // sweep levels
    uint32_t nlev_up = 0, nlev_dn = 0;
};

Hierarchy build_hierarchy(uint32_t n, const uint32_t* row_ptr,
                          const uint32_t* dst, const uint32_t* w,
                          int threads, uint32_t settle_limit, int verbose);

// The same hierarchy contracted on GPU `device` (ch_gpu.cpp, ch_kernels.hip):
// identical rank, arcs and levels to build_hierarchy's.
Hierarchy build_hierarchy_gpu(uint32_t n, const uint32_t* row_ptr,
                              const uint32_t* dst, const uint32_t* w,
                              int device, uint32_t settle_limit, int verbose);

// Sweep levels (level_up / level_dn / nlev_*) of a hierarchy whose rank and
// arc CSRs are set.
void hierarchy_levels(Hierarchy& H, uint32_t n);

// Upper bound on any finite shortest-path distance (u64, exact arithmetic).
uint64_t distance_bound(uint32_t n, const uint32_t* row_ptr,
                        const uint32_t* dst, const uint32_t* w);

double now_seconds();

}  // namespace cpd

struct cpd_plan {
    uint32_t n = 0, m = 0;
    std::vector<uint32_t> row_ptr, dst, w;  // node space, file edge order
    std::vector<uint32_t> order, inv;       // node -> column, column -> node
    cpd::Hierarchy ch;
    uint64_t dist_bound = 0;
    double ch_seconds = 0.0;
};

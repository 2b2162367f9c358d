// Test harness (tests/test_query_file.py): reads a query file with
// cpd::io::read_query_file on T threads and prints "n\n" + "s t" lines, or
// "ERR <message>" — compiled from the library's own cpd_io.cpp on the host.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "cpd_internal.hpp"
#include "cpd_io.hpp"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    std::vector<uint32_t> s, t;
    try {
        cpd::io::read_query_file(argv[1], std::atoi(argv[2]), s, t);
    } catch (const std::exception& e) {
        std::printf("ERR %s\n", e.what());
        return 0;
    }
    std::printf("%zu\n", s.size());
    for (size_t i = 0; i < s.size(); ++i) std::printf("%u %u\n", s[i], t[i]);
    return 0;
}

// bin/gen_distribute_conf — drop-in for warthog's gen_distribute_conf
// (install.sh:5), called by process_query.make_parts (process_query.py:46-53):
//
//   gen_distribute_conf --nodenum N --maxworker W --partmethod {div|mod} --partkey K
//
// stdout: exactly one header line, then N lines "node,wid,bid,bidx".  The
// caller uses getstatusoutput, which merges stderr into stdout, so nothing may
// be written to stderr on success.
#include <cstdio>
#include <vector>

#include "cli.hpp"

int main(int argc, char** argv) {
    cli::Args a(argc, argv);
    long long n = a.num("nodenum", -1), w = a.num("maxworker", -1),
              k = a.num("partkey", -1);
    std::string m = a.str_any({"partmethod", "partition"});
    if (n <= 0 || w <= 0 || k <= 0 || m.empty()) {
        std::fprintf(stderr,
                     "usage: gen_distribute_conf --nodenum N --maxworker W "
                     "--partmethod {div|mod} --partkey K\n");
        return 2;
    }
    int method = cli::method_code(m);
    std::vector<char> buf(1 << 20);
    std::setvbuf(stdout, buf.data(), _IOFBF, buf.size());
    std::fputs("node,wid,bid,bidx\n", stdout);
    for (long long v = 0; v < n; ++v) {
        uint32_t wid, bid, bidx;
        cli::check(cpd_partition((uint32_t)n, (uint32_t)w, method, (uint32_t)k, (uint32_t)v, &wid,
                                 &bid, &bidx),
                   "partition");
        // getstatusoutput strips the final newline, so split('\n') sees no
        // empty trailing line
        std::printf("%lld,%u,%u,%u\n", v, wid, bid, bidx);
    }
    std::fflush(stdout);
    return 0;
}

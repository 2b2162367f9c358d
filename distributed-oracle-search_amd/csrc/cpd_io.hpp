// File formats on the drop-in boundary (host C++; used by bin/* tools).
//
//   .xy    graph: 3 comment lines, "nodes N edges M" on line 4 (read by
//          process_query.get_node_num, process_query.py:126-130), then
//          "v id x y" and "e from to cost" lines.  Out-edge k of a node is its
//          k-th "e" line (file order) [U: warthog xy_graph].
//   .diff  congested weights: "e from to cost" (or "from to cost") lines, each
//          replacing the weight of the first from->to edge [U].
//   .scen  scenario: "q s t" lines (process_query.read_p2p, :22-32).
//   query  "{n}\n" then n lines "s t" (process_query.send_queries, :93-96).
//   .cpd   one file per partition bucket (README.md:86-93 "one or more CPDs"),
//          our own layout == the HBM layout, so a load is one read + one copy.
//          DOSCPD02: the rows in their compact form, a move per column
//          (cpd_rows_export_moves) in `bits` = 1, 2 or 4 bits by the
//          graph's max out-degree (header word 7), n*bits/8 bytes per row;
//          DOSCPD03 (default): the same rows striped over part files; DOSCPD01
//          (make_cpd_auto --format rle): RLE run words, 4 B per run.
//   .order the DFS column order shared by every bucket of a graph.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace cpd {
namespace io {

struct XYGraph {
    uint32_t n = 0, m = 0;
    std::vector<uint32_t> row_ptr, dst, w;
    std::vector<int32_t> x, y;
};

XYGraph read_xy(const std::string& path);
void write_xy(const std::string& path, uint32_t n, const uint32_t* row_ptr,
              const uint32_t* dst, const uint32_t* w, const int32_t* x, const int32_t* y);

// Weights after applying a .diff to `g` ("-" or "" = free-flow copy).
std::vector<uint32_t> read_diff(const std::string& path, const XYGraph& g);
void write_diff(const std::string& path, const XYGraph& g, const std::vector<uint32_t>& w_cong);

using Pairs = std::vector<std::pair<uint32_t, uint32_t>>;
Pairs read_scen(const std::string& path);
void write_scen(const std::string& path, const Pairs& q);
Pairs read_query_file(const std::string& path);
// The same file as two arrays (sources, targets), its lines parsed by up to
// `threads` threads (pieces of >= 1 MB).
void read_query_file(const std::string& path, int threads, std::vector<uint32_t>& s,
                     std::vector<uint32_t>& t);

uint64_t graph_fingerprint(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                           const uint32_t* w);

struct CpdBucket {
    uint32_t n = 0, bid = 0, method = 0, key = 0, maxworker = 0;
    uint64_t fingerprint = 0;
    std::vector<uint32_t> targets;
    std::vector<uint64_t> offsets;
    std::vector<uint32_t> runs;
};

std::string xy_stem(const std::string& xy_path);
std::string bucket_path(const std::string& outdir, const std::string& xy_path,
                        const std::string& method, uint32_t key, uint32_t bid);
std::string order_path(const std::string& outdir, const std::string& xy_path);

void write_bucket(const std::string& path, const CpdBucket& b);

// A bucket file written in pieces, from several threads and in any order:
// header fields and targets at open, offsets and runs by positional writes
// into the layout write_bucket produces, the total at close (then the .tmp is
// renamed).  The finished file is byte-identical to write_bucket's.
class BucketFile {
public:
    // `b` supplies the header fields and targets (its offsets/runs are unused)
    BucketFile(const std::string& path, const CpdBucket& b);
    ~BucketFile();  // without close(): the .tmp is removed
    BucketFile(const BucketFile&) = delete;
    BucketFile& operator=(const BucketFile&) = delete;
    uint32_t nrows() const { return nrows_; }
    // offsets of rows [first_row, first_row + count), bucket-relative
    void write_offsets(uint32_t first_row, const uint64_t* off, uint32_t count);
    // runs [first_run, first_run + count) of the bucket
    void write_runs(uint64_t first_run, const uint32_t* runs, uint64_t count);
    void close(uint64_t total);

private:
    void pwrite_all(const void* p, size_t bytes, uint64_t pos);
    std::string path_, tmp_;
    int fd_ = -1;
    uint32_t nrows_ = 0;
};
CpdBucket read_bucket(const std::string& path);
// Header, targets and offsets only (runs left empty; total = offsets.back()),
// the file size checked against the header; then runs [first, first+count)
// read by position, so a bucket of any size streams through a small buffer.
CpdBucket read_bucket_head(const std::string& path);
void read_bucket_runs(const std::string& path, const CpdBucket& head, uint64_t first,
                      uint64_t count, uint32_t* out);
// Which layout a bucket file has: 1 (DOSCPD01, run words) or 2 (DOSCPD02,
// move tables); throws CPD_E_IO for anything else.
int bucket_format(const std::string& path);

// DOSCPD02 — compact bucket: the rows as move tables, `bits` (1, 2 or 4)
// per column (bijective with the greedy RLE rows; cpd_api.h
// cpd_rows_export_moves):
//   magic "DOSCPD02" | n nrows bid method key maxworker words bits (8 x u32) |
//   total_runs u64 | fingerprint u64 | targets u32[nrows] |
//   runs u32[nrows] (run count of each row) | zero pad to a 4-KiB boundary |
//   rows u32[nrows][words], words = ceil(n * bits / 32)
struct MoveBucket {
    uint32_t n = 0, bid = 0, method = 0, key = 0, maxworker = 0, words = 0, bits = 4;
    uint64_t fingerprint = 0, total_runs = 0;
    // striped (DOSCPD03): the rows in `stripes` (<= 4096) part files
    // {path}.{fingerprint as 16 hex digits}.p{j}, in units of stripe_rows
    // rows dealt round robin (unit u in part u % stripes)
    uint32_t stripes = 1, stripe_rows = 0;
    std::vector<uint32_t> targets, counts;
    uint64_t rows_offset() const;  // DOSCPD02: where the rows start
    uint64_t head_bytes() const;   // DOSCPD03: the main file's size
    uint64_t part_rows(uint32_t j) const;
};
std::string move_part_path(const std::string& path, uint64_t fingerprint, uint32_t j);
// Written in pieces from several threads, in any order (positional writes);
// close() writes the run total and renames the .tmp files into place (the
// parts first, the main file last).  stripes > 1: DOSCPD03, the rows in
// part files — writes to one file serialise on its inode (~10 GB/s of
// page-cache copies on the GPU box, 117 GB/s over 16 files).
class MoveBucketFile {
public:
    // `b` supplies the header fields and targets (counts / total unused)
    MoveBucketFile(const std::string& path, const MoveBucket& b, uint32_t stripes = 1,
                   uint32_t stripe_rows = 64);
    ~MoveBucketFile();  // without close(): the .tmp files are removed
    MoveBucketFile(const MoveBucketFile&) = delete;
    MoveBucketFile& operator=(const MoveBucketFile&) = delete;
    void write_counts(uint32_t first_row, const uint32_t* counts, uint32_t count);
    void write_rows(uint32_t first_row, const uint32_t* rows, uint32_t count);
    void close(uint64_t total_runs);

private:
    void pwrite_all(int fd, const void* p, size_t bytes, uint64_t pos);
    void discard();  // close and remove every .tmp still open
    std::string path_, tmp_;
    int fd_ = -1;
    uint32_t nrows_ = 0, words_ = 0, stripes_ = 1, stripe_rows_ = 0;
    uint64_t rows_off_ = 0, fp_ = 0;
    std::vector<int> part_fd_;
};
// Header, targets and counts (the file size checked against the header, and
// with check_parts the part files' sizes); rows [first, first + count) then
// read by position.
MoveBucket read_move_bucket_head(const std::string& path, bool check_parts = true);
void read_move_bucket_rows(const std::string& path, const MoveBucket& head, uint32_t first,
                           uint32_t count, uint32_t* out, int threads = 1);

void write_order(const std::string& path, uint64_t fingerprint, const std::vector<uint32_t>& order);
std::vector<uint32_t> read_order(const std::string& path, uint64_t fingerprint);
uint32_t read_order_n(const std::string& path);  // its node count (header only)

}  // namespace io
}  // namespace cpd

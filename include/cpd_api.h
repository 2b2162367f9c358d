/*
 * cpd_api.h — C ABI of the MI355X-native CPD engine (libcpd.so).
 *
 * The reference (eggeek/distributed-oracle-search) has no in-process FFI: its
 * hot path lives in the warthog executables `make_cpd_auto` and
 * `fifo_auto --alg table-search` (un-vendored submodule `pathfinding/`,
 * README.md:6-7, install.sh:3-7), driven over a process boundary by
 * make_cpds.py:20, make_fifos.py:21 and process_query.py:46,86-89.  This
 * header is the boundary our replacement executables (bin/make_cpd_auto,
 * bin/fifo_auto, bin/gen_distribute_conf) call, and the one a maintainer would
 * bind from Python (ctypes) or any other FFI.  Every
 * signature is plain C: pointers, sizes, status codes.  No torch types.
 *
 * Each entry point names the reference interface it replaces.  [U] marks
 * upstream-warthog behaviour that cannot be verified here (source absent,
 * SURVEY.md §0, §8c).
 *
 * Conventions
 *   - Node ids are the 0-based ids of the .xy file.  A "column" is a node's
 *     position in the DFS-preorder column order (warthog
 *     cpd::compute_dfs_preorder [U]); CPD runs store column indices.
 *   - Out-edge k of node n is the k-th `e n ...` line of the .xy file (file
 *     order); first moves are these k (0..14; 15 is reserved).
 *   - A run is `(start_column << 4) | move` (warthog rle_run32 [U]).
 *   - Every function returns CPD_OK (0) or a negative CPD_E_* code and sets a
 *     thread-local message readable with cpd_last_error().
 *   - Functions marked [host] never touch a GPU and work without one.
 *     Functions marked [gpu] fail loudly (CPD_E_HIP) when no gfx950 device is
 *     present; there is no CPU fallback in this library.
 */
#ifndef CPD_API_H
#define CPD_API_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPD_OK          0
#define CPD_E_ARG      -1   /* bad argument / malformed input            */
#define CPD_E_HIP      -2   /* HIP runtime error or no usable device     */
#define CPD_E_OOM      -3   /* host or device allocation failed          */
#define CPD_E_NOROW    -4   /* a query's target has no row in the index  */
#define CPD_E_RANGE    -5   /* value out of supported range (degree>15,
                               distances >= 2^32-1, N >= 2^28)            */
#define CPD_E_IO       -6   /* file open/read/write/format error         */

#define CPD_PART_DIV    0
#define CPD_PART_MOD    1

#define CPD_MAX_DEGREE 15u          /* 4-bit move field, 0xF reserved [U] */
#define CPD_INF        0xFFFFFFFFu  /* unreachable distance              */
#define CPD_FM_ALL     0xFFFFu      /* wildcard first-move set           */

typedef struct cpd_plan  cpd_plan;   /* host-side preprocessing of one graph     */
typedef struct cpd_graph cpd_graph;  /* a plan resident on one GPU               */
typedef struct cpd_rows  cpd_rows;   /* a batch of built CPD rows (device)       */
typedef struct cpd_index cpd_index;  /* CPD rows loaded for table-search (device) */

/* Thread-local description of the last error. Never NULL. */
const char* cpd_last_error(void);
/* Library version string, e.g. "cpd-mi355x 0.1 gfx950". */
const char* cpd_version(void);

/* ------------------------------------------------------------------------ */
/* [host] Partitioner — replaces warthog util/distribution_controller.h,
 * exposed by ./bin/gen_distribute_conf (README.md:31-34,75-80;
 * process_query.py:46-53).  node -> (worker id, bucket id, index in bucket).
 *   mod: bid = node % key, bidx = node / key
 *   div: chunk = ceil(nodenum / key), bid = node / chunk, bidx = node % chunk
 *   both: wid = bid % maxworker                                   [U]        */
int cpd_partition(uint32_t nodenum, uint32_t maxworker, int method,
                  uint32_t key, uint32_t node,
                  uint32_t* wid, uint32_t* bid, uint32_t* bidx);
/* Number of buckets a (nodenum, method, key) partition has. */
int cpd_partition_nbuckets(uint32_t nodenum, int method, uint32_t key,
                           uint32_t* nbuckets);

/* [host] Disk preflight of a make_cpd_auto worker (make_cpds.py:58-60 starts
 * every worker at once, each writing its buckets into one --outdir; VERDICT
 * r05 item 2).  cpd_bucket_bytes: bytes of nrows compact rows at `bits` per
 * column (DOSCPD02/03) in nbuckets bucket files of `stripes` parts, headers
 * included.  cpd_space_check: CPD_E_IO (the numbers in cpd_last_error) when
 * the file system holding `dir` has fewer than `bytes` bytes available to
 * this user; *avail (may be NULL) = what it has.                             */
int cpd_bucket_bytes(uint32_t n, uint32_t bits, uint64_t nrows, uint32_t nbuckets,
                     uint32_t stripes, uint64_t* bytes);
int cpd_space_check(const char* dir, uint64_t bytes, uint64_t* avail);

/* [host] DFS-preorder column order — replaces warthog
 * cpd::compute_dfs_preorder [U]: iterative DFS from node 0 (then from every
 * still-unvisited node in id order), out-edges pushed in file order, so the
 * last out-edge is explored first.  order[node] = column.                    */
int cpd_dfs_preorder(uint32_t n, const uint32_t* row_ptr, const uint32_t* dst,
                     uint32_t* order);

/* [host] Synthetic grid-perturbed road graph.  W x H lattice,
 * jittered coordinates, random spanning tree kept bidirectional (strongly
 * connected), extra lattice edges (a share of them one-way) up to a mean
 * out-degree `mean_outdeg`; weights ceil(euclid * speed * asym / 10) in
 * [1, 65535]; node ids randomly permuted; out-edge order shuffled.
 * Call once with row_ptr == NULL to get *n and *m, then again with buffers
 * row_ptr[n+1], dst[m], w[m], x[n], y[n] (x / y may be NULL).               */
int cpd_synth_road_graph(uint32_t width, uint32_t height, double mean_outdeg,
                         uint64_t seed, uint32_t* n, uint32_t* m,
                         uint32_t* row_ptr, uint32_t* dst, uint32_t* w,
                         int32_t* x, int32_t* y);
/* The same generator with its departures from SURVEY.md §8(d) switchable:
 * flags = 0 is the §8(d) recipe as written (node id = row-major lattice cell,
 * every edge bidirectional, out-edges ordered east, north, west, south);
 * CPD_SYNTH_SHUFFLED (= what cpd_synth_road_graph builds) permutes node ids,
 * makes a fifth of the extra edges one-way and shuffles each out-edge list.
 * The shuffled edge order makes a reverse-CPD column's move (the column's own
 * out-edge index) uncorrelated with its neighbours', so rows compress
 * poorly; the direction order lets neighbouring columns share moves.        */
#define CPD_SYNTH_SHUFFLE_IDS   1u
#define CPD_SYNTH_SHUFFLE_EDGES 2u
#define CPD_SYNTH_ONE_WAY       4u
#define CPD_SYNTH_SHUFFLED      7u
int cpd_synth_road_graph_ex(uint32_t width, uint32_t height, double mean_outdeg,
                            uint64_t seed, uint32_t flags, uint32_t* n, uint32_t* m,
                            uint32_t* row_ptr, uint32_t* dst, uint32_t* w,
                            int32_t* x, int32_t* y);
/* [host] Congested weights (the `.diff` stand-in): a share
 * `frac` of the edges get w * U[lo, hi] rounded up; others unchanged.        */
int cpd_synth_congestion(uint32_t m, const uint32_t* w, double frac, double lo,
                         double hi, uint64_t seed, uint32_t* w_out);

/* ------------------------------------------------------------------------ */
/* [host] Preprocessing plan — the part of warthog's make_cpd_auto that runs
 * once per graph (graph load, column order) [U], plus what the GPU build needs
 * instead of a per-row Dijkstra: a contraction hierarchy (CH) with its
 * up/down sweep levels (GPHAST-style one-to-all sweeps).                     */
typedef struct cpd_plan_opts {
    int      threads;          /* OpenMP threads for the CH build (0 = all)  */
    uint32_t witness_settle;   /* witness-search settle limit (0 = default)  */
    int      verbose;          /* print CH progress to stderr                */
    int      no_hierarchy;     /* skip the CH: the plan can serve queries
                                  (fifo_auto) but cannot build rows         */
    int      ch_gpu;           /* 1: contract the CH on GPU ch_device (the
                                  host build's hierarchy, arc for arc;
                                  CPD_E_HIP without a GPU); 0: host threads */
    int      ch_device;
} cpd_plan_opts;

typedef struct cpd_plan_info {
    uint32_t n, m;
    uint64_t ch_up_arcs;       /* arcs v->x with rank(x) > rank(v)           */
    uint64_t ch_dn_arcs;       /* arcs u->v with rank(v) < rank(u)           */
    uint32_t levels_up;        /* launches of the upward sweep               */
    uint32_t levels_dn;        /* launches of the downward sweep             */
    uint64_t dist_bound;       /* proven upper bound on any finite distance  */
    double   ch_seconds;       /* wall time of the CH build                  */
} cpd_plan_info;

int  cpd_plan_create(const uint32_t* row_ptr, const uint32_t* dst,
                     const uint32_t* w, uint32_t n, uint32_t m,
                     const cpd_plan_opts* opts, cpd_plan** out);
int  cpd_plan_info_get(const cpd_plan* p, cpd_plan_info* info);
int  cpd_plan_order(const cpd_plan* p, uint32_t* order /* n */);
/* Export the hierarchy in NODE space (for CPU-side checks):
 * rank[n]; up CSR (up_off[n+1], up_dst, up_w); down CSR (dn_off[n+1],
 * dn_dst, dn_w); level_up[n], level_dn[n].  Any pointer may be NULL.        */
int  cpd_plan_export_ch(const cpd_plan* p, uint32_t* rank,
                        uint64_t* up_off, uint32_t* up_dst, uint32_t* up_w,
                        uint64_t* dn_off, uint32_t* dn_dst, uint32_t* dn_w,
                        uint32_t* level_up, uint32_t* level_dn);
/* save writes `path`.tmp.<pid>.<n> and renames it into place (atomic for
 * concurrent readers; concurrent savers of the same plan do not collide).
 * load checks the file's consistency: the column order is a permutation and
 * the hierarchy's arrays agree in size and range.                           */
int  cpd_plan_save(const cpd_plan* p, const char* path);
int  cpd_plan_load(const char* path, cpd_plan** out);
/* Load the plan cached at `path` if it was built from this very graph, else
 * build it and save it there.  make_cpds.py:58-60 starts every worker at once
 * (tmux -d) on one --outdir, so several processes may reach a cold cache
 * together: an exclusive flock(2) on `path`.lock lets one of them build while
 * the others wait and then load what it saved.  *status = 0 loaded, 1 built
 * and saved, 2 built but the cache could not be written (the plan is still
 * returned: a cache failure never fails the build).                         */
int  cpd_plan_cache(const char* path, const uint32_t* row_ptr, const uint32_t* dst,
                    const uint32_t* w, uint32_t n, uint32_t m, const cpd_plan_opts* opts,
                    cpd_plan** out, int* status);
void cpd_plan_free(cpd_plan* p);

/* ------------------------------------------------------------------------ */
/* [gpu] Devices and graphs. */
int  cpd_device_count(int* count);
/* Free and total HBM bytes of `device` (hipMemGetInfo there): what a caller
 * sizes cpd_graph_set_hbm_reserve against.                                 */
int  cpd_device_mem_info(int device, uint64_t* free_bytes, uint64_t* total_bytes);
/* HBM arena: commit `bytes` on `device` up front (touch != 0: also write
 * them once, paying first-touch costs now), for the library's device buffers
 * on that device to be carved from — so that a caller can overlap the
 * commit of a build's batch buffers (~200 GB: seconds) with other work, as
 * make_cpd_auto does with the plan.  Buffers carved from it are never
 * returned to it; cpd_device_arena_release frees the block, once the graphs,
 * rows and indexes using it are freed.  What does not fit is allocated
 * separately.  cpd_batch_bytes [host]: the HBM a build at `batch` rows needs
 * on a graph of n nodes and that max out-degree (an upper bound; graph
 * arrays excluded).                                                        */
int  cpd_device_arena(int device, uint64_t bytes, int touch);
int  cpd_device_arena_release(int device);
int  cpd_batch_bytes(uint32_t n, uint32_t max_degree, uint32_t batch, uint64_t* bytes);
/* Upload a plan to `device` (column-space CSR, CH arcs, levels). */
int  cpd_graph_create(const cpd_plan* p, int device, cpd_graph** out);
/* Batch width (rows built per sweep, multiple of 1024; 0 = auto from HBM). */
int  cpd_graph_set_batch(cpd_graph* g, uint32_t batch);
int  cpd_graph_get_batch(const cpd_graph* g, uint32_t* batch);
/* Bits per move of the graph's packed compact rows (cpd_rows_move_bits of
 * every cpd_rows it builds): 1, 2 or 4 for max out-degree <= 2, <= 4, else. */
int  cpd_graph_move_bits(const cpd_graph* g, uint32_t* bits);
/* HBM bytes the auto batch (batch 0) leaves free for what follows on this
 * GPU: an index built from the rows on the same handle, or a fifo_auto
 * serving beside a make_cpd_auto.  The auto batch takes 85% of the free HBM
 * above the reserve (default 0), both emit buffer sets included.  Takes
 * effect at the next cpd_graph_set_batch(g, 0), or at the first build when
 * the batch was never set.  With a reserve set, that call fails with
 * CPD_E_OOM when what is left cannot hold a 1024-row batch.  Explicit batch
 * widths ignore the reserve.                                               */
int  cpd_graph_set_hbm_reserve(cpd_graph* g, uint64_t bytes);
/* Optional node coordinates (x[n], y[n], node-id space, e.g. the .xy file's
 * `v id x y`; NULL clears them).  A batch's targets are then laid out over
 * the lanes along a Hilbert curve of their coordinates instead of by column,
 * so every 256-target lane group is spatially compact and its final
 * distances fit the narrow rows' 16-bit offsets.  Results are identical
 * either way; only the speed changes.                                      */
int  cpd_graph_set_coords(cpd_graph* g, const int32_t* x, const int32_t* y);
void cpd_graph_free(cpd_graph* g);

/* ------------------------------------------------------------------------ */
/* [gpu] CPD row build — replaces the per-source loop of warthog
 * make_cpd_auto (README.md:82-95; make_cpds.py:20): for each target t, the
 * distances d(n,t) for all n (reverse search: rows are keyed by target
 * because queries are routed to the worker owning t, process_query.py:56-57),
 * the first-move sets FM_t(n) = {k : w(n->v_k) + d(v_k,t) = d(n,t)}
 * (t itself and unreachable nodes: wildcard), and the greedy run-length row
 * over the DFS column order with the lowest-set-bit tie-break
 * (warthog graph_oracle::add_row [U]).  Rows stay in HBM in their compact
 * form — the RLE row expanded into a move per column (1, 2 or 4 bits by the
 * graph's max out-degree: cpd_graph_move_bits), which under the
 * greedy rule is a bijection (consecutive runs always carry different moves,
 * so the runs are column 0 and every column whose move differs from its left
 * neighbour's) — and are exported either as run words or in that form.
 * `reuse` (may be NULL) recycles a previous result's buffers.               */
int  cpd_build_rows(cpd_graph* g, const uint32_t* targets, uint32_t ntargets,
                    cpd_rows* reuse, cpd_rows** out);
/* The targets the NEXT cpd_build_rows call on g will start with (its first
 * batch; copied).  The current call's last batch then starts that batch's
 * up-sweep early, beside its own first moves and RLE count (a call with
 * several batches does this between its own batches without a hint).  A
 * next call with other targets discards the early work; results never
 * depend on the hint.  Cleared by every cpd_build_rows.                     */
int  cpd_graph_hint_next(cpd_graph* g, const uint32_t* targets, uint32_t ntargets);
int  cpd_rows_count(const cpd_rows* r, uint32_t* nrows, uint64_t* total_runs);
/* Run words (start_column << 4 | move), decoded on the GPU from the compact
 * rows: the rows of warthog's rle_run32 form [U], byte for byte.            */
int  cpd_rows_export(const cpd_rows* r, uint64_t* offsets /* nrows+1 */,
                     uint32_t* runs /* total_runs */);
/* Rows [first, first + count) of r: offsets relative to row `first`
 * (count + 1 values, offsets[0] = 0) and their runs.  Copies on a stream of
 * the calling thread's own, so exports from several host threads, and a
 * cpd_build_rows into ANOTHER cpd_rows on the same device, run concurrently
 * (the overlapped writer of bin/make_cpd_auto).  Either output may be NULL. */
int  cpd_rows_export_range(const cpd_rows* r, uint32_t first, uint32_t count,
                           uint64_t* offsets /* count+1 */, uint32_t* runs);
/* The compact form (DOSCPD02 bucket files, cpd_index_append_moves): a move
 * per column in *bits = 1, 2 or 4 bits — the fewest that hold every move of
 * the graph (a move indexes its column's out-list: out-degrees <= 2, <= 4,
 * else) — column c at bits bits*c .. bits*c + bits-1 of the row, a row being
 * *words = ceil(n * bits / 32) u32; the fields past column n-1 repeat the
 * last run's move.  Rows [first, first + count) back to back, on the calling
 * thread's stream (packed on the GPU when bits < 4).                        */
int  cpd_rows_move_words(const cpd_rows* r, uint32_t* words);
int  cpd_rows_move_bits(const cpd_rows* r, uint32_t* bits);
int  cpd_rows_export_moves(const cpd_rows* r, uint32_t first, uint32_t count,
                           uint32_t* moves /* count * words */);
int  cpd_rows_targets(const cpd_rows* r, uint32_t* targets /* nrows */);
/* The batch lane each row was built in (lane = position in its sweep batch,
 * 0..batch-1; rows are lane-sorted by Hilbert key with coordinates, else by
 * column).  Results never depend on it; tests use it to cover every slab.   */
int  cpd_rows_lanes(const cpd_rows* r, uint32_t* lanes /* nrows */);
/* [gpu] Page-locked host memory for export destinations: a D2H copy into it
 * runs at PCIe rate (a pageable destination is staged through a bounce
 * buffer at a fraction of it).  Free with cpd_host_free.                    */
int  cpd_host_alloc(size_t bytes, void** out);
void cpd_host_free(void* p);
/* Wait for the device work behind r: a build returns once its rows' run
 * counts are known, while the last batch's run emit may still be running
 * (it overlaps the next build's sweeps); every accessor above waits for it,
 * this call only waits.  The bench calls it inside its timed region. */
int  cpd_rows_wait(const cpd_rows* r);
void cpd_rows_free(cpd_rows* r);

/* [gpu] Inspection (tests): distances d(n,t) in NODE order, n-major
 * (dist[node * ntargets + i]), and first-move sets fm[i * n + node].
 * ntargets <= batch.  Either output may be NULL.                            */
int  cpd_debug_rows(cpd_graph* g, const uint32_t* targets, uint32_t ntargets,
                    uint32_t* dist, uint16_t* fm);

/* ------------------------------------------------------------------------ */
/* [gpu] Table-search index — replaces fifo_auto's CPD load + `--alg
 * table-search` extraction (make_fifos.py:20-21; README.md:110).            */
int  cpd_index_create(cpd_graph* g, const uint32_t* row_targets, uint32_t nrows,
                      const uint64_t* offsets, const uint32_t* runs,
                      cpd_index** out);
/* Same, straight from device-resident rows (no host round trip). */
int  cpd_index_from_rows(cpd_graph* g, const cpd_rows* r, cpd_index** out);

/* Streamed index — the load of fifo_auto (make_fifos.py:21 loads every CPD
 * the worker owns; README.md:110).  Declare the rows (row i = target
 * row_targets[i]) and their total run count, then append the rows in order,
 * in chunks, from host arrays (a bucket file read piece by piece) or from a
 * device-built cpd_rows; queries need every row appended.  The mode is fixed
 * at creation: DENSE (or AUTO resolving to it: 4 * total_runs > n/2 * nrows)
 * expands each chunk into the 4-bit move tables as it arrives and keeps no
 * runs, so HBM holds nrows * n/2 bytes however large the runs are; RLE keeps
 * the runs (total_runs of capacity).  Dense tables hold a move per column
 * at the graph's packed width (cpd_graph_move_bits: 1, 2 or 4 bits; nrows *
 * npad * bits / 8 bytes).  Appended host rows are format-checked on the GPU
 * (first run at column 0, columns increasing and < n; for tables narrower
 * than 4 bits also every move < 2^bits), CPD_E_ARG otherwise.                */
int  cpd_index_create_empty(cpd_graph* g, const uint32_t* row_targets, uint32_t nrows,
                            int mode, uint64_t total_runs, cpd_index** out);
/* offsets: count + 1 values relative to the chunk (offsets[0] = 0). */
int  cpd_index_append_rows(cpd_index* ix, uint32_t count, const uint64_t* offsets,
                           const uint32_t* runs);
int  cpd_index_append_built_rows(cpd_index* ix, const cpd_rows* r);
/* Rows in the compact form (cpd_rows_export_moves layout: count rows of
 * ceil(n * bits / 32) words, bits = 1, 2 or 4): copied into a DENSE index's
 * tables when bits is the graph's packed width, else repacked on the GPU
 * (wider rows must carry moves that fit: CPD_E_ARG otherwise), or decoded
 * into run words for an RLE index (total_runs of the create call must cover
 * them).  No other check is needed: a move naming no out-edge of its column
 * stops a walk there, unfinished, as the oracle's walk does.               */
int  cpd_index_append_moves(cpd_index* ix, uint32_t count, uint32_t bits, const uint32_t* moves);
/* Rows declared / appended, runs resident in HBM, bytes of dense tables.     */
int  cpd_index_info(const cpd_index* ix, uint32_t* nrows, uint32_t* added,
                    uint64_t* runs_resident, uint64_t* dense_bytes);

/* In-HBM representation the extraction walks.  RLE: binary search in the run
 * rows (galloping from the previous move's run).  DENSE: the rows expanded on
 * the GPU into 4-bit move tables (n/2 bytes per row, one load per move) —
 * the same move for every column, so identical results.  AUTO (default)
 * picks the smaller of the two (reverse-CPD rows on road graphs often hold
 * more than n/8 runs, where the dense table is smaller AND faster).
 * get_mode reports the representation AUTO resolves to.                     */
#define CPD_INDEX_AUTO  0
#define CPD_INDEX_RLE   1
#define CPD_INDEX_DENSE 2
int  cpd_index_set_mode(cpd_index* ix, int mode);
int  cpd_index_get_mode(const cpd_index* ix, int* mode);
/* Edge weights used for path cost (m entries, original edge order):
 * NULL restores the free-flow weights; otherwise e.g. the .diff weights
 * (process_query.py:89,178 sends the diff name with every batch).           */
int  cpd_index_set_weights(cpd_index* ix, const uint32_t* w);

typedef struct cpd_query_stats {
    uint64_t queries;
    uint64_t finished;      /* queries whose walk reached t                  */
    uint64_t hops;          /* sum of moves taken (n_expanded / plen)        */
    uint64_t cost;          /* sum of path costs                             */
    double   kernel_ms;     /* device time of the extraction kernel          */
} cpd_query_stats;

/* Walk each query s -> t by repeated get_move(t, cur) (binary search in
 * row(t) at column(cur), warthog graph_oracle::get_move [U]) and sum the
 * selected weights.  k_moves < 0: walk to t (process_query.py:153 sends -1);
 * otherwise stop after k moves.  cost/hops/finished may be NULL.
 * Returns CPD_E_NOROW if some t has no row in this index.                    */
int  cpd_query_batch(cpd_index* ix, const uint32_t* s, const uint32_t* t,
                     uint32_t nq, int32_t k_moves, uint64_t* cost,
                     uint32_t* hops, uint8_t* finished, cpd_query_stats* st);
/* The same in three steps, so that a caller can keep the queries resident in
 * HBM and time the extraction alone: prepare uploads (s, t) as columns,
 * run launches the kernel (stats only), fetch copies per-query results.     */
int  cpd_query_prepare(cpd_index* ix, const uint32_t* s, const uint32_t* t,
                       uint32_t nq);
int  cpd_query_run(cpd_index* ix, int32_t k_moves, cpd_query_stats* st);
int  cpd_query_fetch(cpd_index* ix, uint64_t* cost, uint32_t* hops,
                     uint8_t* finished);
void cpd_index_free(cpd_index* ix);

/* [gpu] CPD-heuristic search — fifo_auto's other algorithm family
 * (args.py:29-57 --h-scale / --f-scale / -k / time
 * limits, worker JSON keys hscale, fscale, time, itrs, k_moves,
 * process_query.py:149-160).  warthog's cpd_search is absent: the semantics
 * are restated in oracle/cpd_oracle.c (ora_cpd_search) [U].  A* from s under
 * the index's current weights (cpd_index_set_weights), heuristic hscale x the
 * free-flow cost of the CPD path to t, incumbent from the CPD path's cost
 * under the current weights (only paths of <= k_moves moves when k_moves >=
 * 0); stops when f_min x (1 + fscale) >= incumbent, after itrs expansions,
 * or once time_ns have elapsed.  Runs on the queries of the last
 * cpd_query_prepare; per query results (cost, plen as hops, finished) via
 * cpd_query_fetch.  The CPD path values (heuristic, incumbent) come from
 * per-row tables — 20 B per column per index row, built once per index and
 * per weights by pointer jumping — when those fit in half of the free HBM
 * (tables = CPD_SEARCH_AUTO) or when asked for (_TABLES, CPD_E_OOM if they do
 * not fit); else (_WALKS, or AUTO on a large index) from CPD walks memoised
 * in each search's workspace, so an index of any size can be searched.  The
 * results and counters are the same either way.  A search's workspace holds
 * `capacity` columns (searched ones; with walks also the walked ones; 72 /
 * 120 B each).  Before each pop a search checks that the expansion fits;
 * when it might not, it stops there with its state whole and (when a
 * larger pass can follow) copies it into a spill pool; the next pass, at
 * 4x the capacity, resumes it from there — same pops, counters and results
 * as one uninterrupted search (a search whose record finds the pool full
 * restarts from scratch instead; `wasted_expanded` counts that work).  What
 * still overflows at capacity_max (or when no larger workspace fits in
 * HBM) stops unfinished, with finished = 2 in cpd_query_fetch, and is
 * counted in `overflow`.  capacity = 0 selects the library's workspace
 * policy (what fifo_auto runs): the first pass at 2^13 columns when fscale
 * > 0 with tables (2^14 with walks) and 2^14 at fscale 0, lowered (to 2^10
 * at most) until every query of
 * the request gets a lane; capacity_max 0 = 4 n rounded up to a power of 2
 * (<= 2^24); workspace_frac 0 = 0.85 of the free HBM.  An explicit capacity
 * keeps capacity_max 0 = no larger pass and workspace_frac 0 = 0.25.  The
 * time limit is wall clock (as fifo_auto runs it);
 * virtual_tick_ns > 0 replaces it by a deterministic clock that advances
 * virtual_tick_ns per expansion and per edge touched (the oracle's
 * restatement, for tests).                                                   */
#define CPD_SEARCH_AUTO   0
#define CPD_SEARCH_TABLES 1
#define CPD_SEARCH_WALKS  2
typedef struct cpd_search_opts {
    double   hscale;       /* 1.0 */
    double   fscale;       /* 0.0 */
    int32_t  k_moves;      /* -1: whole CPD paths */
    int64_t  itrs;         /* -1: no expansion limit */
    uint64_t time_ns;      /* 0: no time limit (per query) */
    uint32_t capacity;     /* columns per search, power of 2 (0 = automatic) */
    uint64_t virtual_tick_ns; /* 0: wall-clock time limit; else virtual clock */
    int32_t  tables;       /* CPD_SEARCH_AUTO / _TABLES / _WALKS             */
    double   workspace_frac; /* share of the free HBM the lanes' workspaces and
                                spill pools may take (0 = automatic / 0.25);
                                more lanes search at once                    */
    uint32_t capacity_max; /* 0: automatic / none; else searches that overflow
                              `capacity` continue in later passes at 4x the
                              capacity (fewer lanes) up to capacity_max: many
                              lanes for the common short searches, the big
                              workspace only for the long ones              */
} cpd_search_opts;

typedef struct cpd_search_stats {
    uint64_t queries, finished, expanded, inserted, touched, updated, surplus, plen, overflow;
    double   kernel_ms;    /* device time of the search kernel              */
    uint64_t lanes;        /* concurrent searches (workspace slots)         */
    double   tables_ms;    /* device time spent (re)building the tables     */
    int32_t  tables;       /* the form used: CPD_SEARCH_TABLES or _WALKS    */
    uint64_t reruns;       /* searches run again at a larger capacity       */
    uint64_t resumed;      /* ... of them continued from a spilled state    */
    uint64_t restarted;    /* ... of them started over (spill pool full)    */
    uint64_t wasted_expanded; /* expansions the restarted ones threw away  */
    uint32_t passes;       /* search kernel launches (1 + escalations)      */
    uint32_t capacity;     /* columns per lane of the first pass            */
    uint32_t capacity_last;/* ... of the last pass                          */
} cpd_search_stats;

int  cpd_query_search(cpd_index* ix, const cpd_search_opts* opts, cpd_search_stats* st);
/* Per-query counters of the last search: counters[5 q + k] = expanded,
 * inserted, touched, updated, surplus of query q (caller order).            */
int  cpd_query_search_counters(cpd_index* ix, uint32_t* counters);

/* ------------------------------------------------------------------------ */
/* [gpu] Per-kernel device timing (HIP events on the library's stream).      */
typedef struct cpd_kernel_time {
    char     name[32];
    uint64_t launches;
    double   ms;            /* summed device time                            */
    double   bytes;         /* summed algorithmic bytes      */
} cpd_kernel_time;

int  cpd_timing_enable(cpd_graph* g, int enable);
int  cpd_timing_reset(cpd_graph* g);
/* Fills up to `max` entries, returns the number in *count. */
int  cpd_timing_get(const cpd_graph* g, cpd_kernel_time* out, int max,
                    int* count);

#ifdef __cplusplus
}
#endif
#endif /* CPD_API_H */

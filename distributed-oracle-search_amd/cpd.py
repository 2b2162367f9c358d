"""Python mirror of the libcpd C ABI (include/cpd_api.h) over ctypes.

Host-side glue for tests, bench.py and __graft_entry__: numpy arrays in, numpy
arrays out, CPD_E_* codes raised as CpdError.  The compute path is libcpd.so
(HIP kernels for gfx950); there is no Python or CPU fallback here — if the
shared library is missing, importing this module raises.

Reference interfaces mirrored (the reference has no FFI; these are the
executables' contracts):
  partition()          <- distribution_controller / gen_distribute_conf
                          (process_query.py:46-53)
  Graph.build_rows()   <- make_cpd_auto's per-node row loop (README.md:82-95)
  Index.query()        <- fifo_auto --alg table-search (make_fifos.py:20-21)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CPD_LIB: another build of the library (A/B runs of two builds in one job)
LIB_PATH = os.environ.get("CPD_LIB") or os.path.join(_HERE, "libcpd.so")

CPD_OK = 0
CPD_E_ARG = -1
CPD_E_HIP = -2
CPD_E_OOM = -3
CPD_E_NOROW = -4
CPD_E_RANGE = -5
CPD_E_IO = -6
PART_DIV = 0
PART_MOD = 1
INF = 0xFFFFFFFF
FM_ALL = 0xFFFF

EXPORTED = [
    "cpd_last_error", "cpd_version", "cpd_partition", "cpd_partition_nbuckets",
    "cpd_dfs_preorder", "cpd_synth_road_graph", "cpd_synth_congestion",
    "cpd_plan_create", "cpd_plan_info_get", "cpd_plan_order", "cpd_plan_export_ch",
    "cpd_plan_save", "cpd_plan_load", "cpd_plan_free", "cpd_device_count",
    "cpd_graph_create", "cpd_graph_set_batch", "cpd_graph_get_batch", "cpd_graph_free",
    "cpd_build_rows", "cpd_rows_count", "cpd_rows_export", "cpd_rows_export_range",
    "cpd_rows_targets", "cpd_rows_wait", "cpd_rows_free",
    "cpd_debug_rows", "cpd_index_create", "cpd_index_from_rows", "cpd_index_set_weights",
    "cpd_query_batch", "cpd_query_prepare", "cpd_query_run", "cpd_query_fetch",
    "cpd_index_free", "cpd_timing_enable", "cpd_timing_reset", "cpd_timing_get",
    "cpd_index_set_mode", "cpd_index_get_mode", "cpd_plan_cache", "cpd_index_create_empty",
    "cpd_index_append_rows", "cpd_index_append_built_rows", "cpd_index_info",
    "cpd_synth_road_graph_ex", "cpd_query_search", "cpd_query_search_counters",
    "cpd_graph_set_coords", "cpd_host_alloc", "cpd_host_free",
    "cpd_rows_lanes", "cpd_graph_hint_next", "cpd_graph_set_hbm_reserve",
    "cpd_device_mem_info", "cpd_rows_move_words", "cpd_rows_export_moves",
    "cpd_index_append_moves", "cpd_device_arena", "cpd_device_arena_release", "cpd_batch_bytes",
    "cpd_rows_move_bits", "cpd_graph_move_bits", "cpd_bucket_bytes", "cpd_space_check",
]
# generator styles (cpd_synth_road_graph_ex flags): "shuffled" is round 1's
# graph (ids permuted, one-way streets, out-edge order shuffled); "spec" is
# SURVEY.md §8(d) as written (row-major ids, bidirectional, E/N/W/S order)
SYNTH_STYLES = {"shuffled": 7, "spec": 0}
INDEX_MODES = {"auto": 0, "rle": 1, "dense": 2}
SEARCH_FORMS = {"auto": 0, "tables": 1, "walks": 2}


class CpdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libcpd error {code}: {msg}")
        self.code = code


class PlanOpts(C.Structure):
    _fields_ = [("threads", C.c_int), ("witness_settle", C.c_uint32), ("verbose", C.c_int),
                ("no_hierarchy", C.c_int), ("ch_gpu", C.c_int), ("ch_device", C.c_int)]


class PlanInfo(C.Structure):
    _fields_ = [("n", C.c_uint32), ("m", C.c_uint32), ("ch_up_arcs", C.c_uint64),
                ("ch_dn_arcs", C.c_uint64), ("levels_up", C.c_uint32),
                ("levels_dn", C.c_uint32), ("dist_bound", C.c_uint64),
                ("ch_seconds", C.c_double)]


class QueryStats(C.Structure):
    _fields_ = [("queries", C.c_uint64), ("finished", C.c_uint64), ("hops", C.c_uint64),
                ("cost", C.c_uint64), ("kernel_ms", C.c_double)]


class SearchOpts(C.Structure):
    _fields_ = [("hscale", C.c_double), ("fscale", C.c_double), ("k_moves", C.c_int32),
                ("itrs", C.c_int64), ("time_ns", C.c_uint64), ("capacity", C.c_uint32),
                ("virtual_tick_ns", C.c_uint64), ("tables", C.c_int32),
                ("workspace_frac", C.c_double), ("capacity_max", C.c_uint32)]


class SearchStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("queries", "finished", "expanded", "inserted",
                                          "touched", "updated", "surplus", "plen", "overflow")] + \
               [("kernel_ms", C.c_double), ("lanes", C.c_uint64), ("tables_ms", C.c_double),
                ("tables", C.c_int32), ("reruns", C.c_uint64), ("resumed", C.c_uint64),
                ("restarted", C.c_uint64), ("wasted_expanded", C.c_uint64),
                ("passes", C.c_uint32), ("capacity", C.c_uint32), ("capacity_last", C.c_uint32)]


class KernelTime(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_uint64), ("ms", C.c_double),
                ("bytes", C.c_double)]


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it first (make lib, or "
                          "__graft_entry__.build()); there is no fallback")
    lib = C.CDLL(LIB_PATH)
    lib.cpd_last_error.restype = C.c_char_p
    lib.cpd_version.restype = C.c_char_p
    for name in EXPORTED:
        if name not in ("cpd_last_error", "cpd_version"):
            fn = getattr(lib, name)
            if not name.endswith("_free"):
                fn.restype = C.c_int
            else:
                fn.restype = None
    return lib


lib = _load()

u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
u16p = C.POINTER(C.c_uint16)
u8p = C.POINTER(C.c_uint8)
i32p = C.POINTER(C.c_int32)


def _check(rc: int) -> None:
    if rc != CPD_OK:
        raise CpdError(rc, lib.cpd_last_error().decode())


def _ptr(a, ctype):
    if a is None:
        return None
    return a.ctypes.data_as(ctype)


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


def version() -> str:
    return lib.cpd_version().decode()


def lib_src_sha() -> str:
    """The source hash libcpd.so was built from (embedded by the Makefile)."""
    v = version()
    return v.split("src:", 1)[1] if "src:" in v else ""


def src_sha(root: str | None = None) -> str:
    """sha256 (16 hex) of the library and tool sources in the tree at `root`,
    computed exactly as the Makefile's PROV_SRCS / SRC_SHA: the files sorted by
    repo-relative path, contents concatenated."""
    import glob
    import hashlib
    root = root or os.path.dirname(_HERE)
    pats = ["include/*.h", "distributed-oracle-search_amd/csrc/*.cpp",
            "distributed-oracle-search_amd/csrc/*.hpp", "distributed-oracle-search_amd/csrc/*.hip",
            "distributed-oracle-search_amd/tools/*.cpp", "distributed-oracle-search_amd/tools/*.hpp"]
    files = sorted({os.path.relpath(f, root) for p in pats for f in glob.glob(os.path.join(root, p))})
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(root, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


# --------------------------------------------------------------------------
# host utilities

def partition(nodenum: int, maxworker: int, method: str, key: int, node: int):
    """(wid, bid, bidx) of `node` — distribution_controller semantics [U]."""
    wid, bid, bidx = C.c_uint32(), C.c_uint32(), C.c_uint32()
    m = PART_MOD if method == "mod" else PART_DIV if method == "div" else -1
    _check(lib.cpd_partition(C.c_uint32(nodenum), C.c_uint32(maxworker), C.c_int(m),
                             C.c_uint32(key), C.c_uint32(node), C.byref(wid), C.byref(bid),
                             C.byref(bidx)))
    return wid.value, bid.value, bidx.value


def owned_nodes(nodenum: int, maxworker: int, method: str, key: int, wid: int) -> np.ndarray:
    """All nodes assigned to worker `wid` (vectorised restatement of partition())."""
    nodes = np.arange(nodenum, dtype=np.int64)
    if method == "mod":
        bid = nodes % key
    elif method == "div":
        chunk = -(-nodenum // key)
        bid = nodes // chunk
    else:
        raise ValueError("partmethod must be div or mod")
    return nodes[(bid % maxworker) == wid].astype(np.uint32)


def bucket_bytes(n: int, bits: int, nrows: int, nbuckets: int = 1, stripes: int = 16) -> int:
    """Bytes of a worker's compact bucket files (cpd_bucket_bytes)."""
    out = C.c_uint64()
    _check(lib.cpd_bucket_bytes(C.c_uint32(n), C.c_uint32(bits), C.c_uint64(nrows),
                                C.c_uint32(nbuckets), C.c_uint32(stripes), C.byref(out)))
    return out.value


def space_check(directory: str, nbytes: int) -> int:
    """Free bytes of the file system holding `directory`; CpdError (CPD_E_IO)
    when fewer than `nbytes` (cpd_space_check: make_cpd_auto's preflight)."""
    avail = C.c_uint64()
    _check(lib.cpd_space_check(directory.encode(), C.c_uint64(nbytes), C.byref(avail)))
    return avail.value


def dfs_preorder(row_ptr, dst) -> np.ndarray:
    row_ptr, dst = _u32(row_ptr), _u32(dst)
    n = len(row_ptr) - 1
    order = np.empty(n, dtype=np.uint32)
    _check(lib.cpd_dfs_preorder(C.c_uint32(n), _ptr(row_ptr, u32p), _ptr(dst, u32p),
                                _ptr(order, u32p)))
    return order


class RoadGraph:
    """CSR graph (node space, file edge order) + coordinates."""

    def __init__(self, row_ptr, dst, w, x=None, y=None):
        self.row_ptr, self.dst, self.w = _u32(row_ptr), _u32(dst), _u32(w)
        self.x, self.y = x, y

    @property
    def n(self) -> int:
        return len(self.row_ptr) - 1

    @property
    def m(self) -> int:
        return len(self.dst)


def synth_road_graph(width: int, height: int, seed: int, mean_outdeg: float = 2.5,
                     style: str = "shuffled") -> RoadGraph:
    flags = SYNTH_STYLES[style]
    n, m = C.c_uint32(), C.c_uint32()
    _check(lib.cpd_synth_road_graph_ex(width, height, C.c_double(mean_outdeg), C.c_uint64(seed),
                                       C.c_uint32(flags), C.byref(n), C.byref(m), None, None,
                                       None, None, None))
    rp = np.empty(n.value + 1, np.uint32)
    dst = np.empty(m.value, np.uint32)
    w = np.empty(m.value, np.uint32)
    x = np.empty(n.value, np.int32)
    y = np.empty(n.value, np.int32)
    _check(lib.cpd_synth_road_graph_ex(width, height, C.c_double(mean_outdeg), C.c_uint64(seed),
                                       C.c_uint32(flags), C.byref(n), C.byref(m), _ptr(rp, u32p),
                                       _ptr(dst, u32p), _ptr(w, u32p), _ptr(x, i32p),
                                       _ptr(y, i32p)))
    return RoadGraph(rp, dst, w, x, y)


def synth_congestion(w, frac=0.1, lo=1.0, hi=3.0, seed=3) -> np.ndarray:
    w = _u32(w)
    out = np.empty_like(w)
    _check(lib.cpd_synth_congestion(C.c_uint32(len(w)), _ptr(w, u32p), C.c_double(frac),
                                    C.c_double(lo), C.c_double(hi), C.c_uint64(seed),
                                    _ptr(out, u32p)))
    return out


# --------------------------------------------------------------------------
# plan (host preprocessing)

class Plan:
    def __init__(self, g: RoadGraph | None = None, threads: int = 0, settle: int = 0,
                 verbose: bool = False, hierarchy: bool = True, gpu: int | None = None,
                 _handle=None):
        """gpu: contract the hierarchy on this device (None: host threads)."""
        self._h = C.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            opts = PlanOpts(threads, settle, int(verbose), int(not hierarchy),
                            int(gpu is not None), int(gpu or 0))
            _check(lib.cpd_plan_create(_ptr(g.row_ptr, u32p), _ptr(g.dst, u32p),
                                       _ptr(g.w, u32p), C.c_uint32(g.n), C.c_uint32(g.m),
                                       C.byref(opts), C.byref(self._h)))

    @classmethod
    def load(cls, path: str) -> "Plan":
        h = C.c_void_p()
        _check(lib.cpd_plan_load(path.encode(), C.byref(h)))
        return cls(_handle=h)

    @classmethod
    def cache(cls, path: str, g: RoadGraph, threads: int = 0, hierarchy: bool = True,
              gpu: int | None = None):
        """(plan, status): the plan cached at `path` for this graph, built and
        saved under an flock if absent (status 0 loaded, 1 built and saved,
        2 built but not saved) — cpd_plan_cache."""
        h = C.c_void_p()
        st = C.c_int()
        opts = PlanOpts(threads, 0, 0, int(not hierarchy), int(gpu is not None), int(gpu or 0))
        _check(lib.cpd_plan_cache(path.encode(), _ptr(g.row_ptr, u32p), _ptr(g.dst, u32p),
                                  _ptr(g.w, u32p), C.c_uint32(g.n), C.c_uint32(g.m),
                                  C.byref(opts), C.byref(h), C.byref(st)))
        return cls(_handle=h), st.value

    def save(self, path: str) -> None:
        _check(lib.cpd_plan_save(self._h, path.encode()))

    def info(self) -> dict:
        i = PlanInfo()
        _check(lib.cpd_plan_info_get(self._h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in PlanInfo._fields_}

    def order(self) -> np.ndarray:
        o = np.empty(self.info()["n"], np.uint32)
        _check(lib.cpd_plan_order(self._h, _ptr(o, u32p)))
        return o

    def export_ch(self) -> dict:
        inf = self.info()
        n, up, dn = inf["n"], inf["ch_up_arcs"], inf["ch_dn_arcs"]
        out = {
            "rank": np.empty(n, np.uint32),
            "up_off": np.empty(n + 1, np.uint64), "up_dst": np.empty(up, np.uint32),
            "up_w": np.empty(up, np.uint32),
            "dn_off": np.empty(n + 1, np.uint64), "dn_dst": np.empty(dn, np.uint32),
            "dn_w": np.empty(dn, np.uint32),
            "level_up": np.empty(n, np.uint32), "level_dn": np.empty(n, np.uint32),
        }
        _check(lib.cpd_plan_export_ch(
            self._h, _ptr(out["rank"], u32p), _ptr(out["up_off"], u64p),
            _ptr(out["up_dst"], u32p), _ptr(out["up_w"], u32p), _ptr(out["dn_off"], u64p),
            _ptr(out["dn_dst"], u32p), _ptr(out["dn_w"], u32p), _ptr(out["level_up"], u32p),
            _ptr(out["level_dn"], u32p)))
        return out

    def __del__(self):
        if getattr(self, "_h", None):
            lib.cpd_plan_free(self._h)
            self._h = None


# --------------------------------------------------------------------------
# GPU

def device_count() -> int:
    c = C.c_int()
    _check(lib.cpd_device_count(C.byref(c)))
    return c.value


def device_mem_info(device: int = 0):
    """(free, total) HBM bytes of `device` (cpd_device_mem_info)."""
    f, t = C.c_uint64(), C.c_uint64()
    _check(lib.cpd_device_mem_info(C.c_int(device), C.byref(f), C.byref(t)))
    return f.value, t.value


class Rows:
    def __init__(self, h):
        self._h = h

    def wait(self) -> None:
        """Finish the (possibly deferred) device work behind these rows."""
        _check(lib.cpd_rows_wait(self._h))

    def count(self):
        nr, tot = C.c_uint32(), C.c_uint64()
        _check(lib.cpd_rows_count(self._h, C.byref(nr), C.byref(tot)))
        return nr.value, tot.value

    def export(self):
        nr, tot = self.count()
        off = np.empty(nr + 1, np.uint64)
        runs = np.empty(tot, np.uint32)
        _check(lib.cpd_rows_export(self._h, _ptr(off, u64p), _ptr(runs, u32p)))
        return off, runs

    def export_range(self, first: int, count: int):
        """Rows [first, first+count): offsets relative to row `first`, runs."""
        off = np.empty(count + 1, np.uint64)
        _check(lib.cpd_rows_export_range(self._h, C.c_uint32(first), C.c_uint32(count),
                                         _ptr(off, u64p), None))
        runs = np.empty(int(off[-1]), np.uint32)
        _check(lib.cpd_rows_export_range(self._h, C.c_uint32(first), C.c_uint32(count),
                                         None, _ptr(runs, u32p)))
        return off, runs

    def offsets(self, first: int = 0, count: int | None = None) -> np.ndarray:
        """Run offsets of rows [first, first+count) relative to row `first`
        (count + 1 values), without the runs."""
        if count is None:
            count = self.count()[0] - first
        off = np.empty(count + 1, np.uint64)
        _check(lib.cpd_rows_export_range(self._h, C.c_uint32(first), C.c_uint32(count),
                                         _ptr(off, u64p), None))
        return off

    def move_words(self) -> int:
        """Words per row of the compact form (ceil(n * bits / 32))."""
        w = C.c_uint32()
        _check(lib.cpd_rows_move_words(self._h, C.byref(w)))
        return w.value

    def move_bits(self) -> int:
        """Bits per move of the compact form (1, 2 or 4)."""
        b = C.c_uint32()
        _check(lib.cpd_rows_move_bits(self._h, C.byref(b)))
        return b.value

    def export_moves(self, first: int = 0, count: int | None = None) -> np.ndarray:
        """Rows [first, first+count) in the compact form: (count, words) u32,
        column c's move in bits [b*c, b*c + b) of the row, b = move_bits()
        (cpd_rows_export_moves)."""
        if count is None:
            count = self.count()[0] - first
        out = np.empty((count, self.move_words()), np.uint32)
        _check(lib.cpd_rows_export_moves(self._h, C.c_uint32(first), C.c_uint32(count),
                                         _ptr(out, u32p)))
        return out

    def targets(self):
        nr, _ = self.count()
        t = np.empty(nr, np.uint32)
        _check(lib.cpd_rows_targets(self._h, _ptr(t, u32p)))
        return t

    def lanes(self):
        """The batch lane each row was built in (cpd_rows_lanes)."""
        nr, _ = self.count()
        a = np.empty(nr, np.uint32)
        _check(lib.cpd_rows_lanes(self._h, _ptr(a, u32p)))
        return a

    def __del__(self):
        if getattr(self, "_h", None):
            lib.cpd_rows_free(self._h)
            self._h = None


class Graph:
    """A plan resident on one GPU."""

    def __init__(self, plan: Plan, device: int = 0, batch: int = 0, hbm_reserve: int = 0):
        self._h = C.c_void_p()
        self.plan = plan
        _check(lib.cpd_graph_create(plan._h, C.c_int(device), C.byref(self._h)))
        if hbm_reserve:
            self.set_hbm_reserve(hbm_reserve)
        # 0 = the largest batch that fits in free HBM above the reserve (<= 24576)
        _check(lib.cpd_graph_set_batch(self._h, C.c_uint32(batch)))

    @property
    def batch(self) -> int:
        b = C.c_uint32()
        _check(lib.cpd_graph_get_batch(self._h, C.byref(b)))
        return b.value

    def set_batch(self, batch: int) -> None:
        """Rows per sweep (multiple of 1024; 0 = what fits in free HBM)."""
        _check(lib.cpd_graph_set_batch(self._h, C.c_uint32(batch)))

    def set_hbm_reserve(self, nbytes: int) -> None:
        """HBM the auto batch leaves free for what follows on this GPU
        (cpd_graph_set_hbm_reserve); applies at the next set_batch(0)."""
        _check(lib.cpd_graph_set_hbm_reserve(self._h, C.c_uint64(nbytes)))

    def move_bits(self) -> int:
        """Bits per move of the compact rows this graph builds."""
        b = C.c_uint32()
        _check(lib.cpd_graph_move_bits(self._h, C.byref(b)))
        return b.value

    def set_coords(self, x, y) -> None:
        """Node coordinates (node-id space; None clears them): a batch's
        targets are laid out over the lanes along a Hilbert curve of them
        (compact 256-target groups; identical results, fewer wide rows)."""
        if x is None or y is None:
            _check(lib.cpd_graph_set_coords(self._h, None, None))
            return
        xs = np.ascontiguousarray(x, dtype=np.int32)
        ys = np.ascontiguousarray(y, dtype=np.int32)
        if len(xs) != self.plan.info()["n"] or len(ys) != len(xs):
            raise ValueError("coordinates must have one entry per node")
        _check(lib.cpd_graph_set_coords(self._h, _ptr(xs, i32p), _ptr(ys, i32p)))

    def build_rows(self, targets, reuse: Rows | None = None) -> Rows:
        t = _u32(targets)
        h = C.c_void_p()
        _check(lib.cpd_build_rows(self._h, _ptr(t, u32p), C.c_uint32(len(t)),
                                  reuse._h if reuse else None, C.byref(h)))
        if reuse is not None:
            return reuse
        return Rows(h)

    def hint_next(self, targets) -> None:
        """The targets the next build_rows() call starts with: its first
        batch's up-sweep may start during the current call (cpd_graph_hint_next)."""
        t = _u32(targets)
        _check(lib.cpd_graph_hint_next(self._h, _ptr(t, u32p), C.c_uint32(len(t))))

    def debug_rows(self, targets, want_dist=True, want_fm=True):
        t = _u32(targets)
        n = self.plan.info()["n"]
        dist = np.empty((n, len(t)), np.uint32) if want_dist else None
        fm = np.empty((len(t), n), np.uint16) if want_fm else None
        _check(lib.cpd_debug_rows(self._h, _ptr(t, u32p), C.c_uint32(len(t)),
                                  _ptr(dist, u32p), _ptr(fm, u16p)))
        return dist, fm

    def timing(self, enable: bool = True) -> None:
        _check(lib.cpd_timing_enable(self._h, C.c_int(int(enable))))

    def timing_reset(self) -> None:
        _check(lib.cpd_timing_reset(self._h))

    def timing_get(self) -> dict:
        arr = (KernelTime * 32)()
        cnt = C.c_int()
        _check(lib.cpd_timing_get(self._h, arr, 32, C.byref(cnt)))
        return {arr[i].name.decode(): {"launches": arr[i].launches, "ms": arr[i].ms,
                                       "bytes": arr[i].bytes} for i in range(cnt.value)}

    def __del__(self):
        if getattr(self, "_h", None):
            lib.cpd_graph_free(self._h)
            self._h = None


class Index:
    def __init__(self, graph: Graph, rows: Rows | None = None, row_targets=None,
                 offsets=None, runs=None, _handle=None):
        self.graph = graph
        self._h = C.c_void_p()
        if _handle is not None:
            self._h = _handle
        elif rows is not None:
            _check(lib.cpd_index_from_rows(graph._h, rows._h, C.byref(self._h)))
        else:
            rt, off = _u32(row_targets), np.ascontiguousarray(offsets, np.uint64)
            rn = _u32(runs)
            _check(lib.cpd_index_create(graph._h, _ptr(rt, u32p), C.c_uint32(len(rt)),
                                        _ptr(off, u64p), _ptr(rn, u32p), C.byref(self._h)))

    @classmethod
    def streamed(cls, graph: Graph, row_targets, total_runs: int, mode: str = "auto") -> "Index":
        """Empty index of len(row_targets) rows filled by append()/append_rows()
        in order (cpd_index_create_empty)."""
        rt = _u32(row_targets)
        h = C.c_void_p()
        _check(lib.cpd_index_create_empty(graph._h, _ptr(rt, u32p), C.c_uint32(len(rt)),
                                          C.c_int(INDEX_MODES[mode]), C.c_uint64(total_runs),
                                          C.byref(h)))
        return cls(graph, _handle=h)

    def append(self, offsets, runs) -> None:
        """Host rows: offsets relative to the chunk (count + 1 values)."""
        off = np.ascontiguousarray(offsets, np.uint64)
        rn = _u32(runs)
        _check(lib.cpd_index_append_rows(self._h, C.c_uint32(len(off) - 1), _ptr(off, u64p),
                                         _ptr(rn, u32p)))

    def append_moves(self, moves, bits: int = 4) -> None:
        """Host rows in the compact form: (count, ceil(n * bits / 32)) u32
        (cpd_index_append_moves)."""
        mv = np.ascontiguousarray(moves, np.uint32)
        if mv.ndim != 2:
            raise ValueError("moves must be (rows, words)")
        _check(lib.cpd_index_append_moves(self._h, C.c_uint32(mv.shape[0]), C.c_uint32(bits),
                                          _ptr(mv, u32p)))

    def append_rows(self, rows: Rows) -> None:
        _check(lib.cpd_index_append_built_rows(self._h, rows._h))

    def info(self) -> dict:
        nr, ad, rr, db = C.c_uint32(), C.c_uint32(), C.c_uint64(), C.c_uint64()
        _check(lib.cpd_index_info(self._h, C.byref(nr), C.byref(ad), C.byref(rr), C.byref(db)))
        return {"nrows": nr.value, "added": ad.value, "runs_resident": rr.value,
                "dense_bytes": db.value}

    def set_mode(self, mode: str) -> None:
        """'auto' (default), 'rle' or 'dense' — see cpd_index_set_mode."""
        _check(lib.cpd_index_set_mode(self._h, C.c_int(INDEX_MODES[mode])))

    @property
    def mode(self) -> str:
        m = C.c_int()
        _check(lib.cpd_index_get_mode(self._h, C.byref(m)))
        return {v: k for k, v in INDEX_MODES.items()}[m.value]

    def set_weights(self, w=None) -> None:
        if w is None:
            _check(lib.cpd_index_set_weights(self._h, None))
        else:
            w = _u32(w)
            _check(lib.cpd_index_set_weights(self._h, _ptr(w, u32p)))

    def query(self, s, t, k_moves: int = -1):
        s, t = _u32(s), _u32(t)
        nq = len(s)
        cost = np.empty(nq, np.uint64)
        hops = np.empty(nq, np.uint32)
        fin = np.empty(nq, np.uint8)
        st = QueryStats()
        _check(lib.cpd_query_batch(self._h, _ptr(s, u32p), _ptr(t, u32p), C.c_uint32(nq),
                                   C.c_int32(k_moves), _ptr(cost, u64p), _ptr(hops, u32p),
                                   _ptr(fin, u8p), C.byref(st)))
        return cost, hops, fin, {k: getattr(st, k) for k, _ in QueryStats._fields_}

    def prepare(self, s, t) -> None:
        s, t = _u32(s), _u32(t)
        _check(lib.cpd_query_prepare(self._h, _ptr(s, u32p), _ptr(t, u32p), C.c_uint32(len(s))))

    def run(self, k_moves: int = -1) -> dict:
        st = QueryStats()
        _check(lib.cpd_query_run(self._h, C.c_int32(k_moves), C.byref(st)))
        return {k: getattr(st, k) for k, _ in QueryStats._fields_}

    def search(self, s, t, hscale=1.0, fscale=0.0, k_moves=-1, itrs=-1, time_ns=0,
               capacity=0, virtual_tick_ns=0, tables="auto", workspace_frac=0.0,
               capacity_max=0):
        """CPD-heuristic search (cpd_query_search) for queries (s, t):
        (cost, plen, finished, counters[nq, 5], stats); finished = 2: the
        search outgrew its workspace (after the capacity_max reruns)."""
        self.prepare(s, t)
        o = SearchOpts(float(hscale), float(fscale), int(k_moves), int(itrs), int(time_ns),
                       int(capacity), int(virtual_tick_ns), SEARCH_FORMS[tables],
                       float(workspace_frac), int(capacity_max))
        st = SearchStats()
        _check(lib.cpd_query_search(self._h, C.byref(o), C.byref(st)))
        nq = len(s)
        cost = np.empty(nq, np.uint64)
        plen = np.empty(nq, np.uint32)
        fin = np.empty(nq, np.uint8)
        _check(lib.cpd_query_fetch(self._h, _ptr(cost, u64p), _ptr(plen, u32p), _ptr(fin, u8p)))
        cnt = np.empty((nq, 5), np.uint32)
        if nq:
            _check(lib.cpd_query_search_counters(self._h, _ptr(cnt, u32p)))
        return cost, plen, fin, cnt, {k: getattr(st, k) for k, _ in SearchStats._fields_}

    def __del__(self):
        if getattr(self, "_h", None):
            lib.cpd_index_free(self._h)
            self._h = None

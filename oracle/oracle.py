"""ctypes wrapper of oracle/libcpd_oracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference CPD algorithm (see cpd_oracle.c for the
citations and the parity status: distances pinned by scipy, driver I/O pinned
by fixtures from the reference Python, tie-break outputs "parity unpinned"
against the absent warthog source).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcpd_oracle.so")
INF = 0xFFFFFFFF

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make oracle`")
        L = C.CDLL(LIB_PATH)
        L.ora_rle_row.restype = C.c_uint32
        L.ora_get_move.restype = C.c_uint32
        L.ora_build_rows.restype = C.c_void_p
        L.ora_build_rows.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_uint32, C.c_int]
        L.ora_rows_total.restype = C.c_uint64
        L.ora_rows_total.argtypes = [C.c_void_p]
        L.ora_rows_export.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.ora_rows_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def partition(nodenum, maxworker, method, key, node):
    wid, bid, bidx = C.c_uint32(), C.c_uint32(), C.c_uint32()
    m = 1 if method == "mod" else 0 if method == "div" else -1
    rc = lib().ora_partition(C.c_uint32(nodenum), C.c_uint32(maxworker), C.c_int(m),
                             C.c_uint32(key), C.c_uint32(node), C.byref(wid), C.byref(bid),
                             C.byref(bidx))
    if rc:
        raise ValueError("bad partition arguments")
    return wid.value, bid.value, bidx.value


def dfs_preorder(row_ptr, dst):
    row_ptr, dst = _u32(row_ptr), _u32(dst)
    order = np.empty(len(row_ptr) - 1, np.uint32)
    lib().ora_dfs_preorder(C.c_uint32(len(order)), _p(row_ptr), _p(dst), _p(order))
    return order


def reverse_dijkstra(row_ptr, dst, w, t):
    row_ptr, dst, w = _u32(row_ptr), _u32(dst), _u32(w)
    out = np.empty(len(row_ptr) - 1, np.uint32)
    rc = lib().ora_reverse_dijkstra(C.c_uint32(len(out)), _p(row_ptr), _p(dst), _p(w),
                                    C.c_uint32(t), _p(out))
    if rc:
        raise OverflowError("distance does not fit u32")
    return out


def first_moves(row_ptr, dst, w, t):
    row_ptr, dst, w = _u32(row_ptr), _u32(dst), _u32(w)
    fm = np.empty(len(row_ptr) - 1, np.uint16)
    lib().ora_first_moves(C.c_uint32(len(fm)), _p(row_ptr), _p(dst), _p(w), C.c_uint32(t),
                          _p(fm))
    return fm


def rle_row(fm, order):
    fm = np.ascontiguousarray(fm, np.uint16)
    order = _u32(order)
    inv = np.empty_like(order)
    inv[order] = np.arange(len(order), dtype=np.uint32)
    runs = np.empty(len(fm) + 1, np.uint32)
    k = lib().ora_rle_row(C.c_uint32(len(fm)), _p(fm), _p(inv), _p(runs))
    return runs[:k].copy()


def get_move(runs, col):
    runs = _u32(runs)
    return lib().ora_get_move(_p(runs), C.c_uint32(len(runs)), C.c_uint32(col))


def build_rows(row_ptr, dst, w, order, targets, threads=0):
    """All rows for `targets`: (offsets u64[nrows+1], runs u32[])."""
    row_ptr, dst, w, order, targets = map(_u32, (row_ptr, dst, w, order, targets))
    L = lib()
    h = L.ora_build_rows(len(order), _p(row_ptr), _p(dst), _p(w), _p(order), _p(targets),
                         len(targets), threads)
    try:
        tot = L.ora_rows_total(h)
        off = np.empty(len(targets) + 1, np.uint64)
        runs = np.empty(tot, np.uint32)
        L.ora_rows_export(h, _p(off), _p(runs))
    finally:
        L.ora_rows_free(h)
    return off, runs


def moves_from_runs(offsets, runs, n, bits=4):
    """The compact form of RLE rows (the checker of cpd_rows_export_moves /
    DOSCPD02): (nrows, ceil(n*bits/32)) u32, column c's move — that of the
    last run starting at or before c (get_move) — in bits [bits*c, bits*c +
    bits) of the row; the fields past column n-1 repeat the last run's move."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    runs = _u32(runs)
    nrows, per = len(offsets) - 1, 32 // bits
    w = (n * bits + 31) // 32
    out = np.zeros((nrows, w), np.uint32)
    cols = np.arange(per * w, dtype=np.int64)
    shifts = (bits * np.arange(per, dtype=np.uint64)).astype(np.uint64)
    for r in range(nrows):
        rr = runs[int(offsets[r]):int(offsets[r + 1])]
        starts = (rr >> 4).astype(np.int64)
        idx = np.searchsorted(starts, cols, side="right") - 1  # last run starting <= c
        mv = (rr[idx] & 0xF).astype(np.uint64).reshape(w, per)
        out[r] = (mv << shifts).sum(axis=1, dtype=np.uint64).astype(np.uint32)
    return out


def runs_from_moves(moves, n, bits=4):
    """Inverse of moves_from_runs under the greedy rule: a run starts at
    column 0 and wherever the move differs from the left neighbour's."""
    moves = _u32(moves)
    nrows, per = moves.shape[0], 32 // bits
    mask = (1 << bits) - 1
    off = np.zeros(nrows + 1, np.uint64)
    out = []
    for r in range(nrows):
        mv = ((moves[r][:, None] >> (bits * np.arange(per, dtype=np.uint32))) & mask).ravel()[:n]
        starts = np.flatnonzero(np.concatenate(([True], mv[1:] != mv[:-1])))
        out.append(((starts.astype(np.uint32) << 4) | mv[starts]).astype(np.uint32))
        off[r + 1] = off[r] + len(starts)
    return off, (np.concatenate(out) if out else np.empty(0, np.uint32))


def table_search(row_ptr, dst, w_sel, order, row_targets, offsets, runs, s, t, k_moves=-1,
                 threads=0):
    row_ptr, dst, w_sel, order = map(_u32, (row_ptr, dst, w_sel, order))
    n = len(order)
    row_of_target = np.full(n, INF, np.uint32)
    row_of_target[_u32(row_targets)] = np.arange(len(row_targets), dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    runs, s, t = _u32(runs), _u32(s), _u32(t)
    nq = len(s)
    cost = np.empty(nq, np.uint64)
    hops = np.empty(nq, np.uint32)
    fin = np.empty(nq, np.uint8)
    rc = lib().ora_table_search(C.c_uint32(n), _p(row_ptr), _p(dst), _p(w_sel), _p(order),
                                _p(row_of_target), _p(offsets), _p(runs), _p(s), _p(t),
                                C.c_uint32(nq), C.c_int32(k_moves), _p(cost), _p(hops), _p(fin),
                                C.c_int(threads))
    if rc == -4:
        raise KeyError("a query target has no row")
    return cost, hops, fin


def cpd_search(row_ptr, dst, w_free, w_sel, order, row_targets, offsets, runs, s, t,
               hscale=1.0, fscale=0.0, k_moves=-1, itrs=-1, time_ns=0, tick_ns=0, threads=0,
               columns=False):
    """CPD-heuristic search (cpd_oracle.c ora_cpd_search): per query cost,
    plen, finished and stats[q] = (expanded, inserted, touched, updated,
    surplus); with columns=True also the distinct nodes each query met (a 6th
    stats column).  time_ns with tick_ns > 0: the deterministic time limit."""
    row_ptr, dst, w_free, w_sel, order = map(_u32, (row_ptr, dst, w_free, w_sel, order))
    n = len(order)
    row_of_target = np.full(n, INF, np.uint32)
    row_of_target[_u32(row_targets)] = np.arange(len(row_targets), dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    runs, s, t = _u32(runs), _u32(s), _u32(t)
    nq = len(s)
    cost = np.empty(nq, np.uint64)
    plen = np.empty(nq, np.uint32)
    fin = np.empty(nq, np.uint8)
    stats = np.empty((nq, 6), np.uint64)
    L = lib()
    L.ora_cpd_search.argtypes = [C.c_uint32] + [C.c_void_p] * 10 + [
        C.c_uint32, C.c_double, C.c_double, C.c_int32, C.c_int64, C.c_uint64, C.c_uint64] + \
        [C.c_void_p] * 4 + [C.c_int]
    rc = L.ora_cpd_search(n, _p(row_ptr), _p(dst), _p(w_free), _p(w_sel), _p(order),
                          _p(row_of_target), _p(offsets), _p(runs), _p(s), _p(t), nq,
                          float(hscale), float(fscale), int(k_moves), int(itrs), int(time_ns),
                          int(tick_ns), _p(cost), _p(plen), _p(fin), _p(stats), int(threads))
    if rc == -4:
        raise KeyError("a query target has no row")
    return cost, plen, fin, (stats if columns else stats[:, :5].copy())

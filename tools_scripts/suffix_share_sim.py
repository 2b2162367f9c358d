"""Offline estimate: how many walk hops would suffix sharing between walks to
the same target save on the bench's query mix (46 random sources per target)?"""
import sys, time
import numpy as np
sys.path.insert(0, "/root/repo/distributed-oracle-search_amd"); sys.path.insert(0, "/root/repo/oracle")
import cpd, oracle
W = int(sys.argv[1]) if len(sys.argv) > 1 else 300
T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
Q = int(sys.argv[3]) if len(sys.argv) > 3 else 46
g = cpd.synth_road_graph(W, W, seed=1)
order = oracle.dfs_preorder(g.row_ptr, g.dst)
rng = np.random.default_rng(0)
targets = rng.choice(g.n, T, replace=False).astype(np.uint32)
t0 = time.time()
off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets, threads=8)
print("rows", time.time() - t0, file=sys.stderr)
inv = np.empty(g.n, np.int64); inv[order] = np.arange(g.n)
rp = g.row_ptr.astype(np.int64); dst = g.dst.astype(np.int64)
tot = 0; uni = 0
for i, t in enumerate(targets):
    rr = runs[off[i]:off[i + 1]]
    starts = (rr >> 4).astype(np.int64)
    mv_of_col = (rr & 0xF)[np.searchsorted(starts, np.arange(g.n), side="right") - 1]
    seen = set()
    for s in rng.integers(0, g.n, Q):
        cur = int(s); L = 0
        while cur != t:
            if cur in seen:
                break
            seen.add(cur)
            k = int(mv_of_col[order[cur]])
            cur = int(dst[rp[cur] + k]); L += 1
        # full length for the total (walk to t regardless)
        tot_len = 0; c = int(s)
        while c != t:
            c = int(dst[rp[c] + int(mv_of_col[order[c]])]); tot_len += 1
        tot += tot_len; uni += L
print(f"W={W} T={T} Q={Q}: total hops {tot}, hops with suffix sharing {uni}, saved {1 - uni / tot:.3f}, mean len {tot / (T * Q):.1f}")

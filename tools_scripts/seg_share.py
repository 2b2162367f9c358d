# Offline: neighbour rows first_moves gathers per 32-column segment (and per
# group of segments) against the distinct rows, on the bench graph and its
# host-built plan (DESIGN §5 "first_moves' re-reads").  CPU only, ~1 min.
import sys, time, numpy as np
sys.path.insert(0, '/root/repo/distributed-oracle-search_amd'); sys.path.insert(0, '/root/repo')
import cpd
t=time.time()
g = cpd.synth_road_graph(1000, 1000, 1, style="shuffled")
plan = cpd.Plan(g, threads=8)
print("plan", time.time()-t, flush=True)
order = plan.order()            # node -> column
ch = plan.export_ch()
n = g.n
dn_deg = np.diff(ch["dn_off"].astype(np.int64))
leaf = dn_deg == 0               # no down-arcs
print("leaf frac", leaf.mean())
rp = g.row_ptr.astype(np.int64); dst = g.dst
src = np.repeat(np.arange(n), np.diff(rp))
# gathers: for non-leaf column c, neighbour rows col(dst)
m = ~leaf[src]
gc = order[src[m]].astype(np.int64); gr = order[dst[m]].astype(np.int64)
seg = gc // 32
print("gathers", len(gc), "unique rows", len(np.unique(gr)))
# distinct (segment, row) pairs
key = np.unique(seg * (1<<21) + gr)
s_of = key >> 21; r_of = key & ((1<<21)-1)
print("sum |U_s|", len(key), "ratio to unique rows", len(key)/len(np.unique(gr)))
# how far apart (in segment index) are the segments sharing a row
# for each row: sorted segments; consecutive distance
o = np.lexsort((s_of, r_of)); rr = r_of[o]; ss = s_of[o]
same = rr[1:] == rr[:-1]
d = (ss[1:] - ss[:-1])[same]
print("re-reads", same.sum())
for lim in [1,2,4,8,16,64,256,1024]:
    print(" seg distance <=", lim, (d<=lim).mean())
for spw in [1,8,32,128,512]:
    k2 = np.unique((seg//spw) * (1<<21) + gr)
    print("spw", spw, "sum|U|", len(k2), len(k2)/len(np.unique(gr)))

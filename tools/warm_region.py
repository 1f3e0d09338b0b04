"""Timed region of the warm leg from a rocprofv3 kernel trace (csv) of the default bench at W warm-up + K timed steps:
every kernel of the K timed table calls from the first timed gather (t = 0), then the SIMD-equivalent occupancy per
0.5 ms (one-lane and lane-group G2 waves hold a whole SIMD, a gather wave half of one; all waves of a running grid are
counted, so values above 1,024 mean queued waves).
  python tools/warm_region.py run_kernel_trace.csv [W] [K] > profiles/rNN_warm_timeline_20steps.txt"""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
g = [r for r in rows if r["Kernel_Name"] == "mbls_k_g1_aggregate_idx"]
# split gathers into runs separated by > 3 ms gaps
runs, cur = [], [g[0]]
for a, b in zip(g, g[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 3_000_000:
        runs.append(cur); cur = []
    cur.append(b)
runs.append(cur)
print("gather runs:", [len(r) for r in runs])
W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
timed = g[W:W + K]
t0 = int(timed[0]["Start_Timestamp"])
# end: the last verdict that starts after t0 and before the next run
nxt = g[W + K] if len(g) > W + K else None
tend_lim = int(nxt["Start_Timestamp"]) if nxt else 1 << 62
win = [r for r in rows if t0 - 1 <= int(r["Start_Timestamp"]) < tend_lim]
t1 = max(int(r["End_Timestamp"]) for r in win)
print("region ms %.3f" % ((t1 - t0) / 1e6))
simd = {"mbls_k_g1_aggregate_idx": 0.5}
ev = []
for r in win:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6; e = (int(r["End_Timestamp"]) - t0) / 1e6
    w = int(r["Grid_Size_X"]) // 64
    ev.append((s, e, r["Kernel_Name"], w, r["Queue_Id"]))
for s, e, k, w, q in ev:
    print(f"{k[7:]:22s} q{q:>2} {w:6d} {s:8.2f} {e:8.2f} {e-s:6.2f}")
# occupancy in SIMD-equivalents per 0.5 ms bin
T = (t1 - t0) / 1e6
nb = int(T / 0.5) + 1
occ = [0.0] * nb
for s, e, k, w, q in ev:
    f = simd.get(k, 1.0)
    for b in range(nb):
        lo, hi = b * 0.5, (b + 1) * 0.5
        ov = max(0.0, min(hi, e) - max(lo, s))
        if ov > 0 and e > s:
            # waves resident: assume all waves of the grid resident (upper bound)
            occ[b] += min(w * f, 1024) * ov / 0.5
print("occupancy per 0.5 ms (SIMD-equivalents, all grid waves resident, capped per kernel at 1024):")
print(" ".join("%d" % min(o, 9999) for o in occ))

"""Summarise a rocprofv3 kernel trace (csv) of the warm (table) epoch leg: the per-call chain
(table gather + per-set sums, lane-group G2 prep, verdict), how many calls overlap, and the
resident lane-group waves over time against the 1,024 SIMDs (one lane-group wave holds a SIMD).
  python tools/warm_timeline.py gpurun_out/.../run_kernel_trace.csv > profiles/rNN_warm_timeline.txt"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gath = [r for r in rows if r["Kernel_Name"] == "mbls_k_g1_aggregate_idx"]
if gath:  # the epoch's gathers: the most common grid (2,048 sets at 64 / L sets per wave)
    g = max({r["Grid_Size_X"] for r in gath}, key=lambda x: sum(r["Grid_Size_X"] == x for r in gath))
    gath = [r for r in gath if r["Grid_Size_X"] == g]
if not gath:
    sys.exit("no warm-leg gathers in the trace")
# the timed warm run is the longest uninterrupted series of gathers; take its last 12 calls
t0 = int(gath[-12]["Start_Timestamp"])
t1 = int(gath[-1]["End_Timestamp"])
ms = lambda r: ((int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6)
win = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1 + 20_000_000]
print("# kernel, queue, grid waves, start ms, end ms, duration ms (warm epoch, 2,048 x 512-key indexed FAV per call)")
for r in win:
    s, e = ms(r)
    waves = int(r["Grid_Size_X"]) // 64
    print(f"{r['Kernel_Name']:28s} q{r['Queue_Id']:>2} {waves:6d} {s:9.3f} {e:9.3f} {e - s:7.3f}")
print("# summary")
starts = [ms(r)[0] for r in gath[-12:]]
print(f"call period (gather starts): median {statistics.median([b - a for a, b in zip(starts, starts[1:])]):.3f} ms")
names = sorted({r["Kernel_Name"] for r in win})
for k in names:
    v = [ms(r)[1] - ms(r)[0] for r in win if r["Kernel_Name"] == k]
    print(f"{k}: median {statistics.median(v):.3f} ms, min {min(v):.3f}, max {max(v):.3f}, launches {len(v)}")
# resident-wave estimate: every launched wave of a running kernel counted (upper bound)
ev = []
for r in win:
    s, e = ms(r)
    w = int(r["Grid_Size_X"]) // 64
    ev += [(s, w), (e, -w)]
ev.sort()
cur, last, acc, span = 0, None, 0.0, 0.0
for t, d in ev:
    if last is not None and 0 <= last and t <= (t1 - t0) / 1e6:
        acc += cur * (t - last)
        span += t - last
    cur += d
    last = t
print(f"mean launched waves in flight over the window: {acc / max(span, 1e-9):.0f} (1,024 SIMDs)")

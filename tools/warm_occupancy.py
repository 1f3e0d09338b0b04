"""SIMD occupancy of the timed warm epoch in a rocprofv3 kernel trace: the 20 (or --calls)
timed calls are the indexed gathers after the warm-up ones; prints the timed region's span,
the SIMD-ms each kernel family holds (waves x duration; a lane-group / one-lane wave holds a
whole SIMD, a gather wave half of one), and occupancy over time in 1 ms buckets.
  python tools/warm_occupancy.py trace.csv [--warmup 5] [--calls 20]"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--calls", type=int, default=20)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
gath = [r for r in rows if r["Kernel_Name"] == "mbls_k_g1_aggregate_idx"]
timed = gath[a.warmup:a.warmup + a.calls]
t0 = int(timed[0]["Start_Timestamp"])
# the region ends with the last verdict launched before the next gather (roofline calls) begins
nxt = int(gath[a.warmup + a.calls]["Start_Timestamp"]) if len(gath) > a.warmup + a.calls else 1 << 62
win = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < nxt and not r["Kernel_Name"].startswith("__amd")]
t1 = max(int(r["End_Timestamp"]) for r in win)
simd = {"mbls_k_g1_aggregate_idx": 0.5}
tot = defaultdict(float)
buckets = defaultdict(float)
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    waves = int(r["Grid_Size_X"]) // 64
    share = simd.get(r["Kernel_Name"], 1.0)
    tot[r["Kernel_Name"]] += waves * share * (e - s) / 1e6
    for b in range(int((s - t0) // 1e6), int((e - t0) // 1e6) + 1):
        lo, hi = max(s, t0 + b * 1e6), min(e, t0 + (b + 1) * 1e6)
        if hi > lo:
            buckets[b] += waves * share * (hi - lo) / 1e6
span = (t1 - t0) / 1e6
print(f"timed region {span:.2f} ms for {a.calls} calls; SIMD-ms by kernel (per call):")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {k:28s} {v:9.1f}  ({v / a.calls:7.1f} per call)")
w = sum(tot.values())
print(f"total {w:.0f} SIMD-ms = {w / 1024:.2f} ms of a fully packed 1,024-SIMD chip ({100 * w / 1024 / span:.0f}% packing)")
print("occupied SIMDs per 1 ms bucket:", " ".join(f"{buckets[b]:.0f}" for b in range(int(span) + 1)))

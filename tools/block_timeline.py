"""Kernel timeline of the LAST synchronous mainnet block of a rocprofv3 kernel trace of
`bench.py --workload mainnet_block` (its latency loop runs one block + synchronize at a time):
every kernel of that block with queue, start / end relative to the block's first kernel.
  python tools/block_timeline.py gpurun_out/blk/run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if r["Kernel_Name"].startswith("mbls_k_")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# blocks are separated by idle gaps (the synchronize): split at gaps > 0.3 ms
blocks, cur, last_end = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if last_end is not None and s - last_end > 300_000:
        blocks.append(cur)
        cur = []
    cur.append(r)
    last_end = e if last_end is None else max(last_end, e)
blocks.append(cur)
blk = blocks[-1]
t0 = int(blk[0]["Start_Timestamp"])
print("# kernel, queue, grid, start ms, end ms, duration ms (last synchronous block)")
for r in blk:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"{r['Kernel_Name']:28s} q{r['Queue_Id']:>2} {r['Grid_Size_X']:>8} {s:8.3f} {e:8.3f} {e - s:7.3f}")
print(f"# block span {(max(int(r['End_Timestamp']) for r in blk) - t0) / 1e6:.3f} ms over {len(blocks)} gap-separated groups")

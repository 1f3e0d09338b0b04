"""Summarise a rocprofv3 kernel trace of the cold epoch leg (tools/prof_cold.sh): per call the
key grid, the per-set sums and the one-lane G2 chain, plus steady-state step period.
  python tools/timeline.py gpurun_out/cold/run_kernel_trace.csv > profiles/rNN_cold_timeline.txt"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
keys = [r for r in rows if r["Kernel_Name"] == "mbls_k_g1_decode_validate" and r["Grid_Size_X"] == "1048576"]
t0 = int(keys[0]["Start_Timestamp"])
ms = lambda r: ((int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6)
print("# kernel, queue, start ms, end ms, duration ms (cold epoch leg, 2,048 x 512-key FAV per call)")
last = ms(keys[-1])[1] + 80
for r in rows:
    s, e = ms(r)
    if 0 <= s <= last and r["Grid_Size_X"] in ("1048576", "2048", "16384", "131072"):
        print(f"{r['Kernel_Name']:28s} q{r['Queue_Id']:>2} {s:9.2f} {e:9.2f} {e - s:7.2f}")
per = lambda name: [ms(r)[1] - ms(r)[0] for r in rows if r["Kernel_Name"] == name and ms(r)[0] >= 0]
starts = [ms(r)[0] for r in keys]
print("# summary")
print(f"key grid: median {statistics.median(per('mbls_k_g1_decode_validate')):.2f} ms over {len(keys)} calls")
print(f"step period (key grid starts): median {statistics.median([b - a for a, b in zip(starts, starts[1:])]):.2f} ms")
for k in ("mbls_k_g2_sig_decode", "mbls_k_hash_to_g2", "mbls_k_sig_miller", "mbls_k_fav_verdict", "mbls_k_fav_verdict_lg"):
    v = per(k)
    if v:
        print(f"{k}: median {statistics.median(v):.2f} ms, min {min(v):.2f} ms, launches {len(v)}")

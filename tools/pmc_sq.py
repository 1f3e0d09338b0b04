#!/usr/bin/env python3
"""Per-kernel issue / occupancy / LDS figures from one rocprofv3 `--pmc` pass of
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE (tools/pmc_passes.sh, pass sq).

Units per /opt/skills/guides/MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* /
SQ_WAIT_* count quad-cycles; GRBM_GUI_ACTIVE counts cycles summed over the 8 XCDs, so one
XCD's busy cycles = GRBM_GUI_ACTIVE / 8 (checked: sk_to_pk's value / its duration = 8 x the
2.4 GHz clock).  ROCm 7.2 has no gfx950 derived-counter formulas, so they are computed here:
  valu_busy     = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * cycles)
  waves_per_simd= 4 * SQ_WAVE_CYCLES      / (1024 SIMDs * cycles)   (mean resident waves)
  issue_stall   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES                  (share of wave time)
  lds_conflict  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
and, from the "stall" pass (SQ_WAIT_ANY, SQ_IFETCH, SQC_ICACHE_REQ / _MISSES):
  wait_any      = SQ_WAIT_ANY / SQ_WAVE_CYCLES                       (waiting on s_waitcnt)
  icache_miss   = SQC_ICACHE_MISSES / SQC_ICACHE_REQ
Under --pmc the dispatches are serialised, so `ms` is the kernel's isolated duration.

usage: pmc_sq.py PMC_DIR OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024


def main(d, out):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = defaultdict(dict)
    meta = {}
    for fn in files:
        with open(fn) as fh:
            for row in csv.DictReader(fh):
                key = (row["Kernel_Name"].split("(")[0], row["Dispatch_Id"])
                disp[key][row["Counter_Name"]] = float(row["Counter_Value"])
                meta[key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"]), int(row["VGPR_Count"]),
                             int(row["Accum_VGPR_Count"]), int(row["Scratch_Size"]), int(row["Grid_Size"]))
    agg = defaultdict(lambda: defaultdict(float))
    for key, c in disp.items():
        k = key[0]
        a = agg[k]
        a["n"] += 1
        a["ns"] += meta[key][0]
        for name, v in c.items():
            a[name] += v
        a["vgpr"], a["agpr"], a["scratch"], a["grid"] = meta[key][1:]
    res = {}
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        cyc = a.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc <= 0:
            continue
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        res[k] = {
            "dispatches": int(a["n"]),
            "ms": round(a["ns"] / a["n"] / 1e6, 4),
            "vgpr": int(a["vgpr"]), "agpr": int(a["agpr"]), "scratch_bytes_per_lane": int(a["scratch"]),
            "grid": int(a["grid"]),
            "waves": int(a.get("SQ_WAVES", 0) / a["n"]),
            "valu_busy": round(4 * a.get("SQ_ACTIVE_INST_VALU", 0) / (SIMDS * cyc), 4),
            "waves_per_simd": round(4 * wc / (SIMDS * cyc), 3),
            "issue_stall": round(a.get("SQ_WAIT_INST_ANY", 0) / wc, 4) if wc else None,
            "lds_conflict": (round(a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"], 4)
                             if a.get("SQ_LDS_IDX_ACTIVE") else None),
            "valu_insts_per_wave": round(a.get("SQ_INSTS_VALU", 0) / max(a.get("SQ_WAVES", 1), 1)),
        }
        # the "stall" pass (tools/pmc_passes.sh): waiting on dependencies / memory (s_waitcnt) and
        # instruction-cache behaviour
        if "SQ_WAIT_ANY" in a and wc:
            res[k]["wait_any"] = round(a["SQ_WAIT_ANY"] / wc, 4)
        if a.get("SQC_ICACHE_REQ"):
            res[k]["icache_miss"] = round(a.get("SQC_ICACHE_MISSES", 0) / a["SQC_ICACHE_REQ"], 4)
            res[k]["icache_req_per_wave"] = round(a["SQC_ICACHE_REQ"] / max(a.get("SQ_WAVES", 1), 1))
        if "SQ_IFETCH" in a:
            res[k]["ifetch_per_wave"] = round(a["SQ_IFETCH"] / max(a.get("SQ_WAVES", 1), 1))
        if not a.get("SQ_ACTIVE_INST_VALU"):
            res[k].pop("valu_busy")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    cols = ["ms", "vgpr", "agpr", "scratch_bytes_per_lane", "waves", "valu_busy", "waves_per_simd", "issue_stall",
            "lds_conflict", "wait_any", "icache_miss", "ifetch_per_wave"]
    print(f"{'kernel':34s} " + " ".join(f"{c[:12]:>12s}" for c in cols))
    for k, r in res.items():
        print(f"{k[:34]:34s} " + " ".join(f"{str(r.get(c)):>12s}" for c in cols))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

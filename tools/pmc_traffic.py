#!/usr/bin/env python3
"""Fold two rocprofv3 `--pmc` passes (FETCH_SIZE, WRITE_SIZE; one counter per pass, they do not
fit one TCC pass on gfx950) into per-launch HBM bytes for each kernel.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the
bytes of a coalesced read on gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: [0.0, 0])
    for fn in files:
        with open(fn) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = row.get("Kernel_Name", "?").split("(")[0]
                acc[k][0] += float(row["Counter_Value"])
                acc[k][1] += 1
    return {k: (v[0] / v[1]) for k, v in acc.items() if v[1]}


def lib_digest(path=None):
    """First 16 hex digits of the SHA-256 of the in-tree libmbls.so (the build a pass measured)."""
    import hashlib

    path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lambda_ethereum_consensus_amd",
                                "lib", "libmbls.so")
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch = _per_kernel(fdir, "FETCH_SIZE")
    write = _per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * 1024.0 * fetch.get(k, 0.0)  # KiB -> B, gfx950 half-count correction
        wb = 1024.0 * write.get(k, 0.0)
        kernels[k] = {"fetch_bytes": fb, "write_bytes": wb, "bytes_per_launch": fb + wb}
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, --kernel-trace only",
           "correction": "FETCH_SIZE x2 (gfx950), KiB->B", "kernels": kernels,
           # provenance: the library build and the engine knobs the passes ran with
           "libmbls_sha256_16": lib_digest(), "env": {k: v for k, v in os.environ.items() if k.startswith("MBLS_")}}
    dv = [v for k, v in kernels.items() if k == "mbls_k_g1_decode_validate"]
    if dv:
        res["g1_decode_validate_bytes_per_launch"] = dv[0]["bytes_per_launch"]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps({k: round(v["bytes_per_launch"]) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()

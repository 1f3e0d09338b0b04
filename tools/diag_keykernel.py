#!/usr/bin/env python3
"""Diagnostic (GPU): the key-validation kernel alone on the epoch's 2^20 keys, timed with the
engine's HIP-event hooks -- the standalone reference point for the in-pipeline duration that
bench.py's roofline reports.  Usage: python tools/diag_keykernel.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from lambda_ethereum_consensus_amd import device as D  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    D.init(0)
    d_pks, d_off, d_msgs, d_sigs, msgs, perm = bench.make_inputs(D, 2048, 512, 3, 0)
    st = D.Buffer(4 * 2048 * 512)
    D.validate_pubkeys(d_pks, st)
    D.synchronize()
    D.prof_enable(True)
    D.prof_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        D.validate_pubkeys(d_pks, st)
    D.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ms, n = D.prof_read("g1_decode_validate")
    print(json.dumps({"keys": 2048 * 512, "reps": reps, "kernel_avg_ms": round(ms / max(n, 1), 4),
                      "wall_ms_per_rep": round(wall * 1e3, 4), "cu_mask_g2": os.environ.get("MBLS_G2_CUS")}))


if __name__ == "__main__":
    main()

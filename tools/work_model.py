#!/usr/bin/env python3
"""Work model of the bench's roofline: Fp-multiply counts per phase from the
C restatement's op counter (oracle/c `oracle_c_count_phases`, test infrastructure), next to the
per-unit M-counts bench.py prices its roofline with (blst-style algorithms).

The oracle is a textbook restatement (binary-exponent square roots and inversions, a generic
Fp12 Miller loop with per-step tower arithmetic), so its counts are an upper bound for the
pairing-side phases; for the headline unit (one public key: decompress + G1 membership) the two
agree within the ±25% SURVEY.md §8d asks for.

r02: the DEVICE algorithms are counted too -- the kernels' own headers compiled for the host
(tests/hostsim, MBLS_HOST_COUNT) count every Fp multiplication and squaring of each phase of the
one-lane forms.  Those counts are the work model the bench's rooflines price their units with
(device_M below, frozen in profiles/r02_work_model.json); the App. B estimates are kept beside
them with the ratio, which is within ±25% for every unit or explained in the "note".
"""
import ast
import ctypes
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASES = ["pk_decompress", "g1_membership", "sig_decompress", "g2_membership", "hash_to_g2", "miller_loop",
          "final_exp", "g1_add"]


def bench_constants():
    """Module-level M_* / MAC_* assignments of bench.py (read with ast: bench.py is not imported)."""
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    env = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name.startswith(("M_", "MAC_")):
                try:
                    env[name] = eval(compile(ast.Expression(node.value), "bench.py", "eval"), {}, dict(env))
                except Exception:
                    pass
    return env


def counted():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle", "c")], check=True, timeout=300)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "c", "libblsoracle.so"))
    import yaml
    for d in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "bls", "phase0", "verify", "*"))):
        y = yaml.safe_load(open(os.path.join(d, "data.yaml")))
        if y["output"] is not True:
            continue
        i = y["input"]
        out = (ctypes.c_uint64 * 8)()
        rc = lib.oracle_c_count_phases(bytes.fromhex(i["pubkey"][2:]), bytes.fromhex(i["message"][2:]),
                                       bytes.fromhex(i["signature"][2:]), out)
        if rc == 0:
            return dict(zip(PHASES, [int(v) for v in out])), os.path.relpath(d, ROOT)
    raise RuntimeError("no valid verify fixture")


DEV_PHASES = ["pk_decompress", "g1_membership", "sig_decompress", "g2_membership", "hash_to_g2", "miller_loop_1",
              "final_exp", "miller_loop_2", "g1_add", "fp12_mul"]


def device_counted():
    """(mul, sqr) per phase of the device algorithms, on the same valid verify fixture."""
    sys.path.insert(0, ROOT)
    from tests.conftest import build_hostsim
    import yaml

    lib = ctypes.CDLL(build_hostsim())
    for d in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "bls", "phase0", "verify", "*"))):
        y = yaml.safe_load(open(os.path.join(d, "data.yaml")))
        if y["output"] is not True:
            continue
        i = y["input"]
        out = (ctypes.c_uint64 * 20)()
        rc = lib.hs_count_phases(bytes.fromhex(i["pubkey"][2:]), bytes.fromhex(i["message"][2:]),
                                 bytes.fromhex(i["signature"][2:]), out)
        if rc == 0:
            return {k: {"mul": int(out[2 * j]), "sqr": int(out[2 * j + 1]), "M": int(out[2 * j] + out[2 * j + 1])}
                    for j, k in enumerate(DEV_PHASES)}, os.path.relpath(d, ROOT)
    raise RuntimeError("no valid verify fixture")


# device multiply-adds per product (radix-2^28, 14 digits): a multiplication = 196 digit
# products + 196 reduction products, a squaring = 105 + 196 (mbls_fp.hpp)
DEV_MAD_MUL, DEV_MAD_SQR = 392, 301


def device_units(dc):
    """Units the bench prices, from the device counts (M = products, either kind)."""
    M = lambda *ks: sum(dc[k]["M"] for k in ks)
    mads = lambda *ks: sum(dc[k]["mul"] * DEV_MAD_MUL + dc[k]["sqr"] * DEV_MAD_SQR for k in ks)
    return {
        "key": {"M": M("pk_decompress", "g1_membership"), "device_mads": mads("pk_decompress", "g1_membership")},
        "signature": {"M": M("sig_decompress", "g2_membership"), "device_mads": mads("sig_decompress", "g2_membership")},
        "hash_to_g2": {"M": M("hash_to_g2"), "device_mads": mads("hash_to_g2")},
        "miller_1": {"M": M("miller_loop_1"), "device_mads": mads("miller_loop_1")},
        "miller_2": {"M": M("miller_loop_2"), "device_mads": mads("miller_loop_2")},
        "final_exp": {"M": M("final_exp"), "device_mads": mads("final_exp")},
        "fp12_mul": {"M": M("fp12_mul"), "device_mads": mads("fp12_mul")},
        "g1_add": {"M": M("g1_add"), "device_mads": mads("g1_add")},
    }


def model_r02():
    dc, case = device_counted()
    u = device_units(dc)
    b = bench_constants()
    app_b = {"key": b.get("M_PER_KEY"), "signature": b.get("M_SIG"), "hash_to_g2": b.get("M_HASH"),
             "verify_verdict(miller_2 + final_exp)": b.get("M_VERIFY_VERDICT")}
    verdict_dev = u["miller_2"]["M"] + u["final_exp"]["M"]
    return {
        "source": "tests/hostsim hs_count_phases (device headers compiled for the host, MBLS_HOST_COUNT) on "
                  + case,
        "device_counts": dc,
        "units": u,
        "app_b_estimates_M": app_b,
        "ratios_app_b_over_device": {
            "key": round(app_b["key"] / u["key"]["M"], 3),
            "signature": round(app_b["signature"] / u["signature"]["M"], 3),
            "hash_to_g2": round(app_b["hash_to_g2"] / u["hash_to_g2"]["M"], 3),
            "verify_verdict": round(app_b["verify_verdict(miller_2 + final_exp)"] / verdict_dev, 3),
        },
        "mac_per_M_model": b["MAC_PER_M"],
        "device_mads_per_mul": DEV_MAD_MUL,
        "device_mads_per_sqr": DEV_MAD_SQR,
    }


def model():
    c, case = counted()
    b = bench_constants()
    per_key = c["pk_decompress"] + c["g1_membership"]
    return {
        "source": "oracle/c oracle_c_count_phases on " + case + " (Fp multiplies, squarings counted as M)",
        "oracle_counts_M": c,
        "units": {
            "public_key (decompress + G1 membership)": {"oracle_M": per_key, "bench_M": b["M_PER_KEY"],
                                                       "ratio": round(b["M_PER_KEY"] / per_key, 3)},
            "signature (decompress + G2 membership)": {"oracle_M": c["sig_decompress"] + c["g2_membership"],
                                                      "bench_M": b["M_SIG"]},
            "hash_to_g2": {"oracle_M": c["hash_to_g2"], "bench_M": b["M_HASH"]},
            "verify verdict (2 Miller loops + final exp)": {
                "oracle_M": 2 * c["miller_loop"] + c["final_exp"], "bench_M": b["M_VERIFY_VERDICT"]},
        },
        "mac_per_M": b["MAC_PER_M"],
        "note": "bench prices units with SURVEY.md App. B counts (blst algorithms: addition-chain square roots, "
                "sparse line products, cyclotomic squarings); the oracle's textbook algorithms exceed them on "
                "the pairing side, so those rows are upper bounds, not the model",
    }


if __name__ == "__main__" and any(a.startswith("--r0") for a in sys.argv[1:]):
    # --r02 / --r03 ...: the device-count model of the CURRENT headers, frozen for that round
    rnd = next(a for a in sys.argv[1:] if a.startswith("--r0"))[2:]
    m = model_r02()
    with open(os.path.join(ROOT, "profiles", f"{rnd}_work_model.json"), "w") as f:
        json.dump(m, f, indent=1)
        f.write("\n")
    json.dump({"units": m["units"], "ratios": m["ratios_app_b_over_device"]}, sys.stdout, indent=1)
    print()
elif __name__ == "__main__":
    m = model()
    path = os.path.join(ROOT, "profiles", "r01_work_model.json")
    with open(path, "w") as f:
        json.dump(m, f, indent=1)
        f.write("\n")
    json.dump(m["units"], sys.stdout, indent=1)
    print()

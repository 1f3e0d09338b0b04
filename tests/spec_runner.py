"""Python restatement of the reference's BLS spec-test harness.

* Directory layout: <root>/<config>/<fork>/bls/<handler>/<suite>/<case>/data.yaml as in
  lib/spec/testcase.ex:39-49 (our committed fixtures use <root>/<fork>/<handler>/<case>).
* YAML sanitising: hex strings -> binaries, with the reference's quirk that "0x" becomes a
  single zero byte (lib/spec/utils.ex:35).
* Pass criteria: lib/spec/runners/bls.ex:36-138 — byte equality for sign / aggregate /
  eth_aggregate_pubkeys, `:error` when output is null, and for the verify family `{:ok, b}`
  must equal the output while `{:error, _}` is accepted only when the output is false.

`run_case(bls_module, handler, data)` returns (passed, detail).  `bls_module` is either
`lambda_ethereum_consensus_amd.bls` (GPU engine) or `oracle.bls12_381` (checker).
"""
from __future__ import annotations

import glob
import os

import yaml

HANDLERS = (
    "sign",
    "verify",
    "aggregate",
    "fast_aggregate_verify",
    "aggregate_verify",
    "eth_aggregate_pubkeys",
    "eth_fast_aggregate_verify",
)


_LOWER_HEX = frozenset("0123456789abcdef")


def decode16_lower(h):
    """`Base.decode16!(h, case: :lower)` (lib/spec/utils.ex:36): lowercase digits only, even
    length; anything else raises (ArgumentError there, ValueError here)."""
    if len(h) % 2 or not set(h) <= _LOWER_HEX:
        raise ValueError(f"non-alphabet or odd-length digit in lowercase hex: {h[:16]!r}")
    return bytes.fromhex(h)


def sanitize(v):
    if isinstance(v, dict):
        return {k: sanitize(x) for k, x in v.items()}
    if isinstance(v, list):
        return [sanitize(x) for x in v]
    if isinstance(v, str) and v.startswith("0x"):
        return b"\x00" if v == "0x" else decode16_lower(v[2:])
    return v


def discover(root):
    """Yield (handler, case_dir) for every data.yaml below root."""
    for path in sorted(glob.glob(os.path.join(root, "**", "data.yaml"), recursive=True)):
        parts = path.split(os.sep)
        handler = next((p for p in reversed(parts[:-1]) if p in HANDLERS), None)
        if handler:
            yield handler, os.path.dirname(path)


def load_case(case_dir):
    with open(os.path.join(case_dir, "data.yaml")) as f:
        d = yaml.safe_load(f)
    return sanitize(d["input"]), sanitize(d["output"])


def _bytes_case(res, output):
    tag, v = res
    if output is None:
        return tag == "error", res
    return tag == "ok" and v == output, res


def _bool_case(res, output):
    tag, v = res
    if tag == "ok":
        return bool(v) == bool(output), res
    return not output, res


def run_case(bls, handler, inp, output):
    if handler == "sign":
        return _bytes_case(bls.sign(inp["privkey"], inp["message"]), output)
    if handler == "aggregate":
        return _bytes_case(bls.aggregate(inp), output)
    if handler == "eth_aggregate_pubkeys":
        return _bytes_case(bls.eth_aggregate_pubkeys(inp), output)
    if handler == "verify":
        return _bool_case(bls.verify(inp["pubkey"], inp["message"], inp["signature"]), output)
    if handler == "fast_aggregate_verify":
        return _bool_case(bls.fast_aggregate_verify(inp["pubkeys"], inp["message"], inp["signature"]), output)
    if handler == "eth_fast_aggregate_verify":
        return _bool_case(bls.eth_fast_aggregate_verify(inp["pubkeys"], inp["message"], inp["signature"]), output)
    if handler == "aggregate_verify":
        return _bool_case(bls.aggregate_verify(inp["pubkeys"], inp["messages"], inp["signature"]), output)
    raise ValueError(handler)


def run_dir(bls, root):
    """Run every case below root; returns list of (handler, case_dir, passed, detail)."""
    out = []
    for handler, case_dir in discover(root):
        inp, output = load_case(case_dir)
        ok, detail = run_case(bls, handler, inp, output)
        out.append((handler, case_dir, ok, detail))
    return out


if __name__ == "__main__":  # `make spec-test-bls`
    import argparse
    import sys

    ap = argparse.ArgumentParser()
    ap.add_argument("roots", nargs="*", default=[os.path.join(os.path.dirname(__file__), "golden", "bls")])
    ap.add_argument("--oracle", action="store_true", help="run the CPU oracle instead of the GPU engine")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if a.oracle:
        from oracle import bls12_381 as impl
    else:
        from lambda_ethereum_consensus_amd import bls as impl
    fails = 0
    total = 0
    for r in a.roots:
        for handler, case_dir, ok, detail in run_dir(impl, r):
            total += 1
            if not ok:
                fails += 1
                print("FAIL", handler, case_dir, detail)
    print(f"{total - fails}/{total} BLS spec cases passed")
    sys.exit(1 if fails else 0)

"""Generates tests/golden/ssz.yaml: signing-root fixtures from the SSZ oracle (oracle/ssz.py,
pinned by the reference's own hash_tree_root(Fork) vector, test/unit/ssz_test.exs:30-41).
Inputs are seeded; run `python tests/golden/gen_ssz.py` from the repo root to regenerate."""
import os
import random
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ssz  # noqa: E402


def attestation_data(rng, slot, index, src_epoch, tgt_epoch):
    rb = lambda: bytes(rng.randrange(256) for _ in range(32))
    return (slot.to_bytes(8, "little") + index.to_bytes(8, "little") + rb() + src_epoch.to_bytes(8, "little") + rb()
            + tgt_epoch.to_bytes(8, "little") + rb())


def main():
    rng = random.Random(2024)
    out = {"fork": [{"epoch": 5125, "previous_version": "01050406", "current_version": "02050600",
                     "root": ssz.fork_root(5125, bytes([1, 5, 4, 6]), bytes([2, 5, 6, 0])).hex()}]}
    att = []
    edge = [(0, 0, 0, 0), (2**64 - 1, 2**64 - 1, 2**64 - 1, 2**64 - 1), (6_000_000, 63, 187_499, 187_500)]
    for slot, index, se, te in edge + [(rng.randrange(2**40), rng.randrange(64), rng.randrange(2**35),
                                        rng.randrange(2**35)) for _ in range(5)]:
        d = attestation_data(rng, slot, index, se, te)
        dom = bytes(rng.randrange(256) for _ in range(32))
        att.append({"data": d.hex(), "domain": dom.hex(), "data_root": ssz.attestation_data_root(d).hex(),
                    "signing_root": ssz.attestation_data_signing_root(d, dom).hex()})
    out["attestation_data"] = att
    chunks = []
    for leaves in (1, 2, 3, 5, 8, 11, 16):
        leaf = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(leaves)]
        chunks.append({"leaves": [x.hex() for x in leaf], "root": ssz.merkleize(leaf).hex()})
    out["containers"] = chunks
    with open(os.path.join(ROOT, "tests", "golden", "ssz.yaml"), "w") as f:
        yaml.safe_dump(out, f, sort_keys=False, width=200)


if __name__ == "__main__":
    main()

"""TEST INFRASTRUCTURE ONLY (checker, never the product path): CPU restatement of the SSZ
merkleization behind the reference's signing roots.

Follows the consensus-specs SSZ `hash_tree_root` for fixed-size containers as the reference
calls it: `Misc.compute_signing_root/2` (lib/lambda_ethereum_consensus/state_transition/
misc.ex:243-260) -> `Ssz.hash_tree_root/1` (lib/ssz.ex:51-55, the ssz_nif Rust crate, which
is not buildable here).  Pinned by the reference's own known answer, test/unit/ssz_test.exs:30-41
(hash_tree_root(Fork{epoch 5125, <<1,5,4,6>>, <<2,5,6,0>>}) = 0x0270...6d14), checked in
tests/test_oracle_golden.py.
"""
import hashlib

ZERO_CHUNK = b"\x00" * 32


def h(a: bytes, b: bytes) -> bytes:
    return hashlib.sha256(a + b).digest()


def merkleize(chunks):
    """SSZ merkleize: pad to the next power of two with zero chunks, hash pairs to the root."""
    layer = list(chunks) or [ZERO_CHUNK]
    size = 1
    while size < len(layer):
        size *= 2
    layer += [ZERO_CHUNK] * (size - len(layer))
    while len(layer) > 1:
        layer = [h(layer[i], layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def uint64_leaf(v: int) -> bytes:
    return v.to_bytes(8, "little") + b"\x00" * 24


def bytes_leaf(b: bytes) -> bytes:
    """Bytes4 / Bytes32 as one chunk (right zero padded)."""
    assert len(b) <= 32
    return bytes(b) + b"\x00" * (32 - len(b))


def fork_root(epoch: int, previous_version: bytes, current_version: bytes) -> bytes:
    return merkleize([bytes_leaf(previous_version), bytes_leaf(current_version), uint64_leaf(epoch)])


def checkpoint_root(epoch: int, root: bytes) -> bytes:
    return merkleize([uint64_leaf(epoch), root])


def attestation_data_root(data128: bytes) -> bytes:
    """phase0 AttestationData: slot, index, beacon_block_root, source, target (SSZ 128 bytes)."""
    assert len(data128) == 128
    u = lambda o: int.from_bytes(data128[o:o + 8], "little")
    return merkleize([
        uint64_leaf(u(0)),
        uint64_leaf(u(8)),
        data128[16:48],
        checkpoint_root(u(48), data128[56:88]),
        checkpoint_root(u(88), data128[96:128]),
    ])


def signing_root(object_root: bytes, domain: bytes) -> bytes:
    """hash_tree_root(SigningData{object_root, domain})."""
    return merkleize([object_root, domain])


def attestation_data_signing_root(data128: bytes, domain: bytes) -> bytes:
    return signing_root(attestation_data_root(data128), domain)

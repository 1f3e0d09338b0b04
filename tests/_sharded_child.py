"""Child process for the RCCL sharded pubkey-table build, one process per
rank: `python -m tests._sharded_child RANK WORLD ID_FILE OUT_FILE`.  Rank 0 writes the RCCL
unique id to ID_FILE; every rank builds the table sharded over the job from the same keys,
then checks every row against a local (unsharded) build of the same keys in a second engine
pass and writes its per-key status codes to OUT_FILE.  Prints OK on success."""
import os
import random
import sys
import time

import numpy as np

from oracle import bls12_381 as o


def keys(n):
    rng = random.Random(31)
    pks = [o.sk_to_pk(rng.randrange(1, o.R)) for _ in range(n - 3)]
    return pks + [bytes(48), o.INFINITY_PUBKEY, b"\x80" + bytes(47)]


def main():
    rank, world, id_file, out_file = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    from lambda_ethereum_consensus_amd import bls
    from lambda_ethereum_consensus_amd import device as D

    D.init(int(os.environ.get("MBLS_TEST_DEVICE", "0")))
    if rank == 0:
        with open(id_file + ".tmp", "wb") as f:
            f.write(D.comm_unique_id())
        os.replace(id_file + ".tmp", id_file)
    t0 = time.time()
    while not os.path.exists(id_file):
        if time.time() - t0 > 60:
            raise SystemExit("no RCCL id")
        time.sleep(0.05)
    uid = open(id_file, "rb").read()
    D.comm_init(uid, rank, world)
    table = keys(37)  # not a multiple of world: the last shard is ragged
    n = len(table)
    d_pks = D.Buffer.from_host(b"".join(table))
    st = D.Buffer(4 * n)
    t = bls.PubkeyTable()
    t.clear()
    D.pk_table_set_sharded(d_pks, n, st)
    D.synchronize()
    sharded = st.to_numpy(np.int32).tolist()
    assert t.size == n
    # committees over every row, verified against the table: equal to the cold path
    rng = random.Random(3)
    sets, cold = [], []
    for s in range(24):
        members = [rng.randrange(n) for _ in range(rng.randrange(1, 5))]
        m = bytes(rng.randrange(256) for _ in range(32))
        sig = o.sign((rng.randrange(1, o.R)).to_bytes(32, "big"), m)[1]
        sets.append((members, m, sig))
        cold.append(([table[i] for i in members], m, sig))
    assert t.fast_aggregate_verify_batch(sets) == bls.fast_aggregate_verify_batch(cold)
    D.comm_destroy()
    local = t.set(0, table)  # the unsharded build of the same keys
    assert sharded == local, (sharded, local)
    with open(out_file, "w") as f:
        f.write(",".join(map(str, sharded)))
    print("OK")


if __name__ == "__main__":
    sys.exit(main())

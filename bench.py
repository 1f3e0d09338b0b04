#!/usr/bin/env python3
"""bench.py — `fast_aggregate_verify` sets/sec (512-key) on MI355X, BASELINE.json's metric.

Workload (N=1 default): BASELINE.json configs[3] "Epoch replay": 32 slots x 64 committees =
2,048 fast_aggregate_verify sets over disjoint 512-key committees of a 2^20-validator table,
cold (every public key decompressed + subgroup-checked each call, exactly as the reference
NIF does at native/bls_nif/src/lib.rs:92-96).  A "step" = one such batch through
`mbls_dev_fast_aggregate_verify` with inputs already resident in HBM.  Multi-GPU: one
process per GPU (torch.distributed.run launches the ranks), every rank verifies its own epoch
batch (sets are independent: no data-path collective, "scaling": "weak"); a file rendezvous
(lambda_ethereum_consensus_amd/rendezvous.py, standard library only) carries the barrier, the
max-over-ranks of the timed region and the RCCL id -- torch is never imported in a rank, so
libmbls runs on /opt/rocm's HIP runtime and RCCL at every N.

Synthetic data (deterministic): sk_j = S0 + j, committees are a seeded
permutation of the table, m_s = SHA-256("mbls-bench-msg" || seed || s), sigma_s =
(sum of the committee's sk) * H(m_s); keys and signatures are produced on the device by
the engine's own SkToPk / Sign kernels.  All-valid batches are timed; a separate mixed batch
(1/64 of the sets with a wrong message) checks verdicts before timing.

Extra JSON fields: `roofline` (dominant kernel g1_decode_validate, INT VALU multiply-add
bound, timed with HIP events on its own stream) and `cpu_baseline` (the oracle, timed on a
bounded sample on this host).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

# Work model: Fp multiplications per unit, 300 32x32
# multiply-adds each (12-limb CIOS), i.e. an implementation-independent INT multiply-add count.
# Per-unit M counts are the device algorithms' own products, counted by the host build of the
# CURRENT kernels' headers (tools/work_model.py --r05 -> profiles/r05_work_model.json; r03 after the
# r02 SSWU rewrite).  The headline key is priced at the COUNTED 1,482 (decompress 466 +
# membership 1,016, SURVEY.md §8(d): the counted figure is the frozen one);
# SURVEY.md App. B's 1,560 model is reported beside it (frac_app_b).
M_PER_KEY = 466 + 1016
M_PER_KEY_APP_B = 460 + 1100
MAC_PER_M = 300
MAC_PER_KEY = M_PER_KEY * MAC_PER_M
M_SIG = 2535             # signature decompress + G2 membership (counted; App. B 2,250)
M_HASH = 4890            # hash_to_G2 incl. cofactor clearing and the affine conversion (App. B 4,800;
                         # r05: Jacobian [|x|] ladders, 6,065 with the complete ones, r05_work_model.json)
M_MILLER1 = 6863         # one-pair Miller loop
M_MILLER2 = 11494        # two-pair Miller loop with shared squarings
M_FE = 7668              # final exponentiation (HHT hard part; re-counted r05, 8,155 in r03_work_model.json)
M_FP12_MUL = 54
# aggregate_verify Miller work per set of configs[4] (16 key pairs + the signature pair), in the
# units the r04 verdict priced mbls_k_miller_pairs in: key pairs as couples with shared
# squarings (M_MILLER2 per two pairs), the signature pair as one loop
M_AV_PAIRS_PER_SET = 8 * M_MILLER2 + M_MILLER1
M_G1_ADD = 11            # one complete mixed G1 addition (aggregation)
# Measured v_mad_u64_u32 issue peak on MI355X (tools/isa_rates.hip, profiles/r01_isa_rates.json)
PEAK_MAD_PER_S = 3.196e13
# The guide-derived ceiling (MI355X_MICROARCH.md): 256 CU x 4 SIMD x 32 lanes x 2.4 GHz =
# 7.86e13 simple-VALU lane-ops/s; a 64-bit-result mad issues at half that rate
PEAK_MAD_GUIDE = 256 * 4 * 32 * 2.4e9 / 2
PEAK_INT_OPS_PER_S = 5.928e13  # measured v_add_u32 lane rate (profiles/r01_isa_rates.json)
# FAV-512 cold set = 512 keys + verify tail; used for the whole-job MAC figure
M_PER_SET_TAIL = M_SIG + M_HASH + M_MILLER2 + M_FE
BLST_WARM_MS_APP_B = 1.2  # SURVEY.md App. B "target sanity check": blst, one warm FAV-512 set per core


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node.  Under torch.distributed.run (WORLD_SIZE set) it must equal the world "
                         "size: one rank per GPU.  Run directly with N > 1, bench.py launches the N ranks itself "
                         "(--multi ranks, the default) or drives N engines from one process (--multi engines: "
                         "mbls_init_devices, the one-BEAM-node deployment)")
    ap.add_argument("--multi", default="ranks", choices=["ranks", "engines"])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets", type=int, default=2048, help="FAV sets per step per GPU (epoch = 32x64)")
    ap.add_argument("--keys-per-set", type=int, default=512)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-warm", action="store_true", help="skip the validator-pubkey-table (warm) leg")
    ap.add_argument("--no-rlc", action="store_true", help="skip the opt-in RLC batch-check legs")
    ap.add_argument("--no-extra-legs", action="store_true", help="skip the mixed-batch and host end-to-end legs")
    ap.add_argument("--shard", action="store_true",
                    help="strong scaling as the headline: one epoch per step split over the ranks by key count "
                         "(at N > 1 the default line carries it as the `strong` leg)")
    ap.add_argument("--table-build", default="local", choices=["local", "sharded"],
                    help="warm leg's table build at N > 1: every rank validates all keys (local) or 1/N of them "
                         "plus one RCCL all-gather (sharded, SURVEY.md §8e)")
    ap.add_argument("--workload", default="epoch_replay_cold",
                    choices=["epoch_replay_cold", "gossip_verify", "mainnet_block", "deposit_av", "signing_roots"],
                    help="BASELINE.json configs[3] (default, the headline), [1], [2] or [4]")
    ap.add_argument("--traffic-file", default=None,
                    help="per-launch HBM bytes of g1_decode_validate measured by rocprofv3 --pmc (default: the "
                         "newest profiles/r*_pmc_traffic_cold*.json)")
    return ap.parse_args()


# --------------------------------------------------------------------------- inputs ------
def make_inputs(D, n_sets, kps, seed, rank):
    n_keys = n_sets * kps
    tag = seed.to_bytes(4, "big") + rank.to_bytes(4, "big")
    s0 = int.from_bytes(hashlib.sha256(b"mbls-bench-sk" + tag).digest(), "big") % (R_ORDER >> 1)
    s0 = (s0 >> 64 << 64) | (s0 & ((1 << 62) - 1))  # low 64 bits + j never carries
    rng = np.random.default_rng(seed * 1000 + rank)
    perm = rng.permutation(n_keys).astype(np.uint64)  # committee order -> table index
    # sk bytes (big-endian): constant high 24 bytes of S0, low 8 bytes = S0_lo + perm
    hi = (s0 >> 64).to_bytes(24, "big")
    lo = (np.uint64(s0 & ((1 << 64) - 1)) + perm).astype(">u8")
    sk = np.empty((n_keys, 32), dtype=np.uint8)
    sk[:, :24] = np.frombuffer(hi, dtype=np.uint8)
    sk[:, 24:] = lo.view(np.uint8).reshape(n_keys, 8)
    msgs = b"".join(hashlib.sha256(b"mbls-bench-msg" + tag + s.to_bytes(4, "big")).digest() for s in range(n_sets))
    sums = perm.reshape(n_sets, kps).sum(axis=1, dtype=np.uint64)
    agg = [((kps * s0 + int(x)) % R_ORDER).to_bytes(32, "big") for x in sums]
    d_sk = D.Buffer.from_host(sk.reshape(-1))
    d_pks = D.Buffer(n_keys * 48)
    D.sk_to_pk(d_sk, d_pks, n_keys)
    d_agg = D.Buffer.from_host(b"".join(agg))
    d_msgs = D.Buffer.from_host(msgs)
    d_sigs = D.Buffer(n_sets * 96)
    D.sign(d_agg, d_msgs, d_sigs, n_sets)
    D.synchronize()
    d_sk.free()
    d_agg.free()
    key_off = np.arange(0, n_keys + 1, kps, dtype=np.uint32)
    d_off = D.Buffer.from_host(key_off)
    return d_pks, d_off, d_msgs, d_sigs, msgs, perm.astype(np.uint32)


def check_verdicts(D, d_pks, d_off, msgs, d_sigs, n_sets):
    """All-valid batch -> all 1; mixed batch (every 64th set gets a different message) -> 0 there."""
    st = D.Buffer(4 * n_sets)
    d_msgs = D.Buffer.from_host(msgs)
    D.fast_aggregate_verify(d_pks, d_off, d_msgs, d_sigs, st, n_sets)
    D.synchronize()
    ok_all = bool((st.to_numpy(np.int32) == 1).all())
    bad = bytearray(msgs)
    for s in range(0, n_sets, 64):
        bad[32 * s] ^= 0x5A
    d_bad = D.Buffer.from_host(bytes(bad))
    D.fast_aggregate_verify(d_pks, d_off, d_bad, d_sigs, st, n_sets)
    D.synchronize()
    got = st.to_numpy(np.int32)
    exp = np.ones(n_sets, dtype=np.int32)
    exp[::64] = 0
    return ok_all and bool((got == exp).all())


def mixed_leg(D, d_pks, d_off, msgs, d_sigs, n_sets, steps, dist):
    """Throughput on the mixed batch (every 64th set verdicts false): a false
    set takes the same kernels as a true one, so this must equal the all-valid rate to noise."""
    bad = bytearray(msgs)
    for s in range(0, n_sets, 64):
        bad[32 * s] ^= 0x5A
    d_bad = D.Buffer.from_host(bytes(bad))
    ring = StatusRing(D, n_sets, steps + 1)
    el = timed(D, dist, lambda: D.fast_aggregate_verify(d_pks, d_off, d_bad, d_sigs, ring.next(), n_sets), steps, 1)
    exp = np.ones(n_sets, dtype=np.int32)
    exp[::64] = 0
    ok = ring.all_equal(exp)
    ring.free()
    if dist:
        el, ok = reduce_over_ranks(dist, el, ok)
    world = dist.get_world_size() if dist else 1
    d_bad.free()
    return {"value": round(n_sets * steps * world / el, 3), "unit": "sets/s", "steps": steps,
            "ms_per_step": round(el * 1e3 / steps, 3), "false_sets": len(exp[::64]), "verdicts_ok": ok}


def host_e2e_leg(D, d_pks, msgs, d_sigs, n_sets, kps, steps, dist, callers=(1, 3, 4), variants=4):
    """End to end from host binaries, as the NIF hands them over: one
    mbls_bls_fast_aggregate_verify_batch call per epoch = marshal the Erlang-style binary
    list into pinned staging + H2D + kernels + D2H of the verdicts.  `callers` concurrent
    host threads (concurrent dirty-scheduler NIF calls / the batching queue's workers) share
    the `steps` calls: the engine pipelines them (staging and key validation of one call under
    the G2 chain of another).  Consecutive calls carry different wrong-message sets (`variants`
    message lists) and every call's codes land in their own sentinel-filled array, so a call
    that returned stale or unfinished verdicts fails the check.  Not `value`: that
    one starts with the inputs resident in HBM."""
    import threading

    from lambda_ethereum_consensus_amd import _lib, bls

    lib = _lib.load()
    pk = d_pks.to_numpy().reshape(-1, 48)
    sg = d_sigs.to_numpy().reshape(-1, 96)
    pa, _k1 = bls._bins([bytes(r) for r in pk])
    sa, _k3 = bls._bins([bytes(r) for r in sg])
    mvar, keep, expect = [], [], []
    for v in range(variants):
        bad = bytearray(msgs)
        wrong = list(range(7 * v + 1, n_sets, 61 + v))
        for p in wrong:
            bad[32 * p] ^= 0x5A
        ma, k2 = bls._bins([bytes(bad[32 * i:32 * i + 32]) for i in range(n_sets)])
        mvar.append(ma)
        keep.append(k2)
        e = np.ones(n_sets, dtype=np.int32)
        e[wrong] = 0
        expect.append(e)
    off = (ctypes.c_uint32 * (n_sets + 1))(*range(0, n_sets * kps + 1, kps))
    world = dist.get_world_size() if dist else 1
    out = {"unit": "sets/s", "steps": steps,
           "path": "mbls_bls_fast_aggregate_verify_batch (host binaries -> pinned staging -> H2D -> kernels -> D2H)",
           "check": f"every call's codes vs its own wrong-message set ({variants} variants, sentinel-filled outputs)"}
    for t in callers:
        per = [steps // t + (1 if i < steps % t else 0) for i in range(t)]
        codes = [[(ctypes.c_int32 * n_sets)(*([StatusRing.SENTINEL] * n_sets)) for _ in range(per[i])]
                 for i in range(t)]
        gots = [(ctypes.c_size_t * n_sets)() for _ in range(t)]
        errs = []

        def call(i, j, dst):
            v = (i + j * t) % variants
            rc = lib.mbls_bls_fast_aggregate_verify_batch(pa, off, mvar[v], sa, n_sets, 0, dst, gots[i])
            if rc:
                errs.append(_lib.status_message(rc))

        def worker(i):
            for j in range(per[i]):
                call(i, j, codes[i][j])

        warm = (ctypes.c_int32 * n_sets)()
        call(0, 0, warm)  # warm: staging contexts allocated
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        th = [threading.Thread(target=worker, args=(i,)) for i in range(t)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        el = time.perf_counter() - t0
        if errs:
            raise RuntimeError(errs[0])
        ok = all(np.array_equal(np.frombuffer(codes[i][j], dtype=np.int32), expect[(i + j * t) % variants])
                 for i in range(t) for j in range(per[i]))
        if dist:
            el, ok = reduce_over_ranks(dist, el, ok)
        leg = {"value": round(n_sets * steps * world / el, 3), "ms_per_step": round(el * 1e3 / steps, 3),
               "verdicts_ok": ok}
        out[f"callers_{t}"] = leg
    best = max((v for k, v in out.items() if k.startswith("callers_")), key=lambda v: v["value"])
    out["value"] = best["value"]
    out["ms_per_step"] = best["ms_per_step"]
    out["verdicts_ok"] = all(v["verdicts_ok"] for k, v in out.items() if k.startswith("callers_"))
    return out


# --------------------------------------------------------------------------- warm leg ----
def comm_setup(D, dist, barrier=True):
    """the RCCL communicator of the sharded table build; rank 0's unique id
    travels over the gloo group, then every rank joins (one process per GPU).  A failure to make
    the id is broadcast too (every rank raises), so no rank is left waiting in the broadcast."""
    ids = [None]
    if dist.get_rank() == 0:
        try:
            ids = [D.comm_unique_id()]
        except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
            ids = [f"comm_unique_id: {e}"]
    dist.broadcast_object_list(ids, src=0)
    if not isinstance(ids[0], (bytes, bytearray)):
        raise RuntimeError(ids[0])
    D.comm_init(ids[0], dist.get_rank(), dist.get_world_size())
    if barrier:
        dist.barrier()
    return ids[0]


def warm_leg(D, d_pks, d_off, d_msgs, d_sigs, perm, n_sets, steps, warmup, dist, rlc_too=False,
             table_build="local", roofline=True):
    """Same committees through the device-resident validator pubkey table:
    the table is built once in validator order (timed separately), then each step is an
    index-addressed FAV over the epoch's committees (idx = the committee permutation)."""
    n_keys = len(perm)
    pks = d_pks.to_numpy().reshape(n_keys, 48)
    table = np.empty_like(pks)
    table[perm] = pks  # row v = validator v's key
    d_table = D.Buffer.from_host(table.reshape(-1))
    D.synchronize()
    sharded = table_build == "sharded" and dist is not None  # the communicator is set up by the caller
    t0 = time.perf_counter()
    if sharded:
        D.pk_table_set_sharded(d_table, n_keys)
    else:
        D.pk_table_set(0, d_table, n_keys)
    build_s = time.perf_counter() - t0
    d_table.free()
    d_idx = D.Buffer.from_host(perm)
    st = D.Buffer(4 * n_sets)

    world = dist.get_world_size() if dist else 1

    def run(rlc):
        ring = StatusRing(D, n_sets, steps + warmup)

        def step():
            D.fast_aggregate_verify_indexed(d_idx, d_off, d_msgs, d_sigs, ring.next(), n_sets, rlc=rlc)

        elapsed = timed(D, dist, step, steps, warmup)
        ok = ring.all_equal(np.ones(n_sets, dtype=np.int32))
        ring.free()
        if dist:
            elapsed, ok = reduce_over_ranks(dist, elapsed, ok)
        return n_sets * steps * world / elapsed, elapsed, ok

    v, elapsed, ok = run(False)
    roof = warm_roofline(D, lambda: D.fast_aggregate_verify_indexed(d_idx, d_off, d_msgs, d_sigs, st, n_sets),
                         n_sets, n_keys // n_sets) if roofline else None
    if roof is not None:
        # whole-chip fraction of the warm step (the per-kernel fractions above use launch
        # durations that overlap across the G2 streams): all multiply-adds of a set, i.e. the
        # gather's additions, signature decode + check, H(m), the 2-pair Miller loop and the
        # final exponentiation, at the step's rate, over the peak
        per_set = ((n_keys // n_sets - 1) * M_G1_ADD + M_SIG + M_HASH + M_MILLER2 + M_FE) * MAC_PER_M
        roof["chip_mad_per_set"] = per_set
        roof["chip_achieved"] = round(v / world * per_set / 1e12, 4)
        roof["chip_frac"] = round(v / world * per_set / PEAK_MAD_PER_S, 4)
    out = {
        "value": round(v, 3),
        "unit": "sets/s",
        "ms_per_step": round(elapsed * 1e3 / steps, 3),
        "table_build_ms": round(build_s * 1e3, 3),
        "table_build": "sharded (RCCL all-gather)" if sharded else "local",
        "validators_per_gpu": n_keys,
        "verdicts_ok": ok,
        "roofline": roof,
    }
    if rlc_too:
        v, elapsed, ok = run(True)
        out["rlc"] = {"value": round(v, 3), "ms_per_step": round(elapsed * 1e3 / steps, 3), "verdicts_ok": ok}
    return out


def _all_ranks_ok(dist, ok):
    """AND of a per-rank flag over the gloo group (every rank calls it: no rank waits alone in a
    later collective after another one failed)."""
    _, all_ok = reduce_over_ranks(dist, 0.0, ok)
    return all_ok


def sharded_table_leg(D, d_pks, d_off, d_msgs, d_sigs, perm, n_sets, steps, warmup, dist):
    """SURVEY.md §8e's one collective, exercised on every N > 1 line: the
    2^20-key validator table built with mbls_dev_pk_table_set_sharded (rank k decodes +
    KeyValidates 1/N of the rows, one RCCL all-gather over xGMI replicates them), then the warm
    epoch over it with every call's verdicts checked.  Never fatal and never the headline: any
    failure (RCCL refusing two ranks on one GPU in a rehearsal, a communicator that times out in
    libmbls -- MBLS_COMM_TIMEOUT_MS) is reported in `error`, and the ranks agree on each stage's
    outcome over gloo before the next, so no rank waits alone in a collective."""
    out = {"table_build": "sharded (RCCL all-gather)", "world": dist.get_world_size()}
    err = None
    try:
        comm_setup(D, dist, barrier=False)  # the agreement below replaces the barrier
    except Exception as e:  # noqa: BLE001 -- reported, never fatal
        err = f"comm_init: {e}"
    if not _all_ranks_ok(dist, err is None):
        out["error"] = err or "comm_init failed on another rank"
        return out
    try:
        w = warm_leg(D, d_pks, d_off, d_msgs, d_sigs, perm, n_sets, steps, warmup, dist, table_build="sharded",
                     roofline=False)
        out.update(value=w["value"], unit=w["unit"], ms_per_step=w["ms_per_step"],
                   table_build_sharded_ms=w["table_build_ms"], verdicts_ok=w["verdicts_ok"])
    except Exception as e:  # noqa: BLE001
        err = f"sharded build / warm epoch: {e}"
    if not _all_ranks_ok(dist, err is None):
        out["error"] = err or "failed on another rank"
    try:
        D.comm_destroy()
    except Exception:  # noqa: BLE001
        pass
    return out


def warm_roofline(D, step, n_sets, kps):
    """Roofline of the warm (table) epoch's kernels, each timed with HIP events on its own
    stream: the table gather + per-set sums (g1_aggregate_idx: 512 x 128-byte rows per set,
    HBM/L2 gather), the lane-group signature decode + H(m) (g2_prep) and the lane-group
    two-pair Miller loop + final exponentiation (fav_verdict).  The dominant one (longest
    average launch) is the line's `kernel`; INT multiply-add bound except the gather."""
    ks = kernel_avgs(D, step, ("g1_aggregate_idx", "g2_prep", "fav_verdict"))
    work = {  # multiply-adds per launch (SURVEY.md §8d model, counted M x 300)
        "g1_aggregate_idx": n_sets * (kps - 1) * M_G1_ADD * MAC_PER_M,
        "g2_prep": n_sets * (M_SIG + M_HASH) * MAC_PER_M,
        "fav_verdict": n_sets * (M_MILLER2 + M_FE) * MAC_PER_M,
    }
    per = {}
    for k, ms in ks.items():
        if ms <= 0:
            continue
        ach = work[k] / (ms / 1e3)
        per[k] = {"avg_launch_ms": round(ms, 4), "achieved_Tmad_s": round(ach / 1e12, 4),
                  "frac": round(ach / PEAK_MAD_PER_S, 4), "frac_guide": round(ach / PEAK_MAD_GUIDE, 4)}
    gather_bytes = n_sets * kps * 128 + n_sets * kps * 4
    if "g1_aggregate_idx" in per:
        g = per["g1_aggregate_idx"]
        g["gather_bytes"] = gather_bytes
        g["achieved_GB_s"] = round(gather_bytes / (g["avg_launch_ms"] / 1e3) / 1e9, 1)
    dom = max(per, key=lambda k: per[k]["avg_launch_ms"]) if per else None
    if dom is None:
        return None
    d = per[dom]
    # PMC bytes per launch of the kernel form the warm leg runs (2,048-set launches, as in the
    # traffic passes over the default bench command): the 6-lane verdict unless MBLS_LG6=0
    pmc_name = {"fav_verdict": "mbls_k_fav_verdict_lg" + ("" if os.environ.get("MBLS_LG6") == "0" else "6"),
                "g2_prep": "mbls_k_g2_prep_1l", "g1_aggregate_idx": "mbls_k_g1_aggregate_idx"}[dom]
    traffic, traffic_src = pmc_kernel_bytes(pmc_name)
    return {"bound": "valu-int", "kernel": dom, "achieved": d["achieved_Tmad_s"], "peak": round(PEAK_MAD_PER_S / 1e12, 4),
            "unit": "Tmad/s", "frac": d["frac"], "peak_guide": round(PEAK_MAD_GUIDE / 1e12, 4),
            "frac_guide": d["frac_guide"], "traffic": traffic, "traffic_kernel": pmc_name if traffic else None,
            "traffic_source": traffic_src, **(traffic_provenance(traffic_src) if traffic else {}),
            "avg_launch_ms": d["avg_launch_ms"],
            "units_per_launch": n_sets, "mad_per_unit": work[dom] // n_sets, "kernels": per}


# --------------------------------------------------------------------------- cpu leg -----
def _oracle_fav_task(args):
    """One cold FAV-512 on the CPU oracle (test infrastructure; the checker, not the product)."""
    pks, msg, sig = args
    from oracle import bls12_381 as o

    t = time.perf_counter()
    res = o.fast_aggregate_verify(pks, msg, sig)
    return res, time.perf_counter() - t


def host_info():
    """nproc, the cores this process may use, physical cores, the cgroup CPU quota and the CPU
    model."""
    model = "unknown"
    phys = set()
    cur = {}
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model == "unknown":
                model = v
            elif k in ("physical id", "core id"):
                cur[k] = v
            elif not k and cur:
                phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count() or 1, "usable_cpus": usable, "physical_cores": len(phys) or None,
            "cgroup_cpu_quota": quota, "cpu_model": model}


def _median_rate(run, n, runs):
    """Median sets/s of `runs` timed calls of run(n) after one warm-up call."""
    walls = []
    for r in range(runs + 1):
        t = time.perf_counter()
        run(n)
        if r:
            walls.append(time.perf_counter() - t)
    return n / float(np.median(walls)), min(walls), max(walls)


def cpu_baseline_c(D, d_pks, msgs, d_sigs, kps, budget_s, cores, runs=3):
    """The C restatement of the oracle (oracle/c, pthreads, one independent set per task, as
    concurrent BEAM schedulers each in a single-threaded NIF call) on bounded samples of the
    same batch, BASELINE.md §2's protocol (one warm-up run, then the median of `runs` runs),
    MEASURED at 1, 4 and `cores` threads.  Cold = every key decompressed + KeyValidated per call
    (lib.rs:92-96); warm = the sample's keys decoded once into a table (a client's validator
    pubkey cache), then per set only the aggregation and the verify tail -- the like-for-like for
    the engine's indexed FAV.

    All host cores: the pool gives one GPU's run a 16-core share of the host (and asks that
    worker pools stay within it), so the 128-physical-core run that north_star's "all-host-core"
    figure names is not run here.  `all_host_cores_estimate` is the measured per-core rate at
    `cores` threads x the host's PHYSICAL cores (SMT siblings add nothing to this integer-mul
    bound loop; r03 counted all 256 logical CPUs linearly), next to the
    measured 1 -> 4 -> `cores` thread scaling it rests on."""
    from tests import coracle  # test infrastructure: the checker / CPU baseline, never the product

    pks = d_pks.to_numpy()
    sigs = d_sigs.to_numpy()
    m = np.frombuffer(msgs, dtype=np.uint8)
    n_avail = len(msgs) // 32
    info = host_info()
    per_leg = budget_s / 2.0  # cold and warm
    threads = sorted({1, min(4, cores), cores})

    def cold_run(thr):
        def run(n):
            off = np.arange(0, n * kps + 1, kps, dtype=np.uint32)
            out = coracle.fav_batch(pks[:48 * n * kps], off, m[:32 * n], sigs[:96 * n], nthreads=thr)
            assert (out == 1).all()
        return run

    t = time.perf_counter()
    cold_run(1)(1)
    t1 = time.perf_counter() - t
    cold = {}
    for thr in threads:
        # ~per_leg / len(threads) / (runs + 1) seconds per timed run, at least one set per thread
        n = int(min(n_avail, max(thr, per_leg / len(threads) / (runs + 1) / max(t1, 1e-9) * thr)))
        rate, lo, hi = _median_rate(cold_run(thr), n, runs)
        cold[thr] = {"sets": n, "sets_per_s": round(rate, 3), "run_s": [round(lo, 2), round(hi, 2)]}
    n_warm = int(min(n_avail, cold[cores]["sets"]))
    tb = time.perf_counter()
    table = coracle.Table(pks[:48 * n_warm * kps], nthreads=cores)
    build_s = time.perf_counter() - tb
    idx = np.arange(n_warm * kps, dtype=np.uint32)
    ioff = np.arange(0, n_warm * kps + 1, kps, dtype=np.uint32)

    def warm_run(thr):
        def run(n):
            out = table.fav_batch(idx[:n * kps], ioff[:n + 1], m[:32 * n], sigs[:96 * n], nthreads=thr)
            assert (out == 1).all()
        return run

    t = time.perf_counter()
    warm_run(1)(1)
    tw1 = time.perf_counter() - t
    warm = {}
    for thr in threads:
        n = int(min(n_warm, max(thr, per_leg / len(threads) / (runs + 1) / max(tw1, 1e-9) * thr)))
        rate, lo, hi = _median_rate(warm_run(thr), n, runs)
        warm[thr] = {"sets": n, "sets_per_s": round(rate, 3), "run_s": [round(lo, 2), round(hi, 2)]}
    phys = info["physical_cores"] or cores

    def est(curve):
        per_core = curve[cores]["sets_per_s"] / cores
        return {"value": round(per_core * phys, 1), "cores": phys,
                "basis": f"measured {cores}-thread rate / {cores} x {phys} physical cores (estimate, not a run)",
                "scaling_efficiency_1_to_{}".format(cores): round(curve[cores]["sets_per_s"] /
                                                                  (cores * curve[1]["sets_per_s"]), 3)}

    # per counted Fp product (the work model the rooflines use), from the 1-thread runs: the
    # cold and warm legs of one port should cost about the same per product (VERDICT r05 weak #8:
    # before r06 the port's affine Miller loop made its warm path ~4x its cold path per product)
    m_cold = kps * M_PER_KEY + (kps - 1) * M_G1_ADD + M_PER_SET_TAIL
    m_warm = (kps - 1) * M_G1_ADD + M_PER_SET_TAIL
    ns_m = lambda curve, m: round(1e9 / (curve[1]["sets_per_s"] * m), 2)
    return {
        "value": cold[cores]["sets_per_s"],
        "unit": "sets/s",
        "cores": cores,
        "kind": "port",
        "ns_per_counted_M": ns_m(cold, m_cold),
        "counted_M_per_set": m_cold,
        "sample": f"{cold[cores]['sets']} cold FAV-{kps} sets of this batch through oracle/c/bls_oracle.c (C restatement "
                  f"of the oracle, 6x64-bit Montgomery, not blst: blst is not in the image), {cores} threads = the "
                  f"box's CPU share for one GPU; median of {runs} runs after 1 warm-up",
        "threads_measured": {str(k): v for k, v in cold.items()},
        "all_host_cores_estimate": est(cold),
        **info,
        "warm": {"value": warm[cores]["sets_per_s"], "unit": "sets/s", "cores": cores,
                 "sample": f"FAV-{kps} sets over a pre-decoded table of {n_warm * kps} keys (decode + KeyValidate once: "
                           f"{build_s:.2f} s on {cores} threads); median of {runs} runs after 1 warm-up",
                 "threads_measured": {str(k): v for k, v in warm.items()},
                 "ns_per_counted_M": ns_m(warm, m_warm), "counted_M_per_set": m_warm,
                 "all_host_cores_estimate": est(warm),
                 # not a measurement: blst is not in the image; SURVEY.md App. B's per-core figure
                 "blst_app_b_estimate": {"ms_per_set_per_core": BLST_WARM_MS_APP_B,
                                         "value": round(phys / (BLST_WARM_MS_APP_B * 1e-3), 1), "cores": phys,
                                         "basis": "SURVEY.md App. B: ~1.2 ms per warm FAV-512 set per core "
                                                  "(estimate, not a run) x the host's physical cores"}},
    }


def cpu_baseline(D, d_pks, msgs, d_sigs, kps, budget_s, cores):
    """Time the oracle on a bounded sample of the same workload (sets from the same batch)."""
    import multiprocessing as mp

    pks = D.Buffer.to_numpy(d_pks)
    sigs = D.Buffer.to_numpy(d_sigs)
    # calibrate one set, then size the sample to ~budget_s of wall time on `cores` workers
    first = ([bytes(pks[48 * j:48 * j + 48]) for j in range(kps)], msgs[:32], bytes(sigs[:96]))
    res, t1 = _oracle_fav_task(first)
    assert res == ("ok", True), res
    n = max(cores, int(budget_s / max(t1, 1e-9)) * cores)
    n = min(n, len(msgs) // 32)
    tasks = []
    for s in range(n):
        tasks.append(([bytes(pks[48 * (s * kps + j):48 * (s * kps + j) + 48]) for j in range(kps)],
                      msgs[32 * s:32 * s + 32], bytes(sigs[96 * s:96 * s + 96])))
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        out = pool.map(_oracle_fav_task, tasks, chunksize=1)
    wall = time.perf_counter() - t0
    assert all(r == ("ok", True) for r, _ in out)
    return {
        "value": round(n / wall, 4),
        "unit": "sets/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{n} cold FAV-512 sets of this batch through oracle/bls12_381.py (pure-Python restatement), "
                  f"{cores} worker processes, {wall:.1f} s",
    }


# ------------------------------------------------------------- other BASELINE configs ----
# Per-unit algorithmic work (Fp multiplications; x 300 multiply-adds each)
M_VERIFY_VERDICT = M_MILLER2 + M_FE  # 2-pair Miller loop + final exponentiation (counted)


def sks_for(n, seed, rank, tag):
    """n deterministic secret keys S0 + j (big-endian 32 bytes), as make_inputs."""
    t = tag + seed.to_bytes(4, "big") + rank.to_bytes(4, "big")
    s0 = int.from_bytes(hashlib.sha256(b"mbls-bench-sk" + t).digest(), "big") % (R_ORDER >> 1)
    s0 = (s0 >> 64 << 64) | (s0 & ((1 << 62) - 1))
    hi = (s0 >> 64).to_bytes(24, "big")
    lo = (np.uint64(s0 & ((1 << 64) - 1)) + np.arange(n, dtype=np.uint64)).astype(">u8")
    sk = np.empty((n, 32), dtype=np.uint8)
    sk[:, :24] = np.frombuffer(hi, dtype=np.uint8)
    sk[:, 24:] = lo.view(np.uint8).reshape(n, 8)
    return sk, s0


def msgs_for(n, seed, rank, tag):
    t = tag + seed.to_bytes(4, "big") + rank.to_bytes(4, "big")
    return b"".join(hashlib.sha256(b"mbls-bench-msg" + t + j.to_bytes(4, "big")).digest() for j in range(n))


def pmc_kernel_bytes(kernel, src=None):
    """HBM bytes per launch of `kernel` (its mbls_k_ name) from the latest PMC traffic summary
    of the default bench command (the cold and warm legs run in it), with the file it came
    from; (None, None) when no summary holds the kernel."""
    src = src or newest_traffic_file()
    if not src or not os.path.exists(src):
        return None, None
    try:
        k = json.load(open(src)).get("kernels", {}).get(kernel)
    except Exception:
        return None, None
    if not k or "bytes_per_launch" not in k:
        return None, None
    return k["bytes_per_launch"], os.path.relpath(src, ROOT)


def traffic_provenance(src):
    """Where a roofline's `traffic` comes from: an earlier rocprofv3 --pmc pass over
    the default bench command, never this run; `traffic_same_build` says whether that pass
    measured the library this run loaded (the summary records its SHA-256) with the same MBLS_*
    knobs."""
    if not src:
        return {}
    try:
        d = json.load(open(src if os.path.isabs(src) else os.path.join(ROOT, src)))
    except Exception:  # noqa: BLE001
        return {}
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        from pmc_traffic import lib_digest
    finally:
        sys.path.pop(0)
    lib = os.environ.get("MBLS_LIB_PATH") or os.path.join(ROOT, "lambda_ethereum_consensus_amd", "lib", "libmbls.so")
    env = {k: v for k, v in os.environ.items() if k.startswith("MBLS_") and k not in ("MBLS_HW_QUEUES",)}
    same = d.get("libmbls_sha256_16") is not None and d.get("libmbls_sha256_16") == lib_digest(lib) and \
        {k: v for k, v in (d.get("env") or {}).items() if k != "MBLS_HW_QUEUES"} == env
    return {"traffic_measured": "earlier rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (not this run)",
            "traffic_same_build": bool(same)}


def newest_traffic_file():
    """The latest round's PMC traffic summary of the cold epoch (rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes, tools/pmc_traffic.py): profiles/rNN_pmc_traffic_cold*.json."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_traffic_cold*.json")))
    return files[-1] if files else None


class StatusRing:
    """One status buffer per call (filled with a sentinel beforehand), so that every timed
    call's verdicts are checked afterwards -- not only the last call's."""

    SENTINEL = -77

    def __init__(self, D, n_sets, count):
        self.D, self.n = D, n_sets
        fill = np.full(n_sets, self.SENTINEL, dtype=np.int32).tobytes()
        self.bufs = [D.Buffer.from_host(fill) for _ in range(max(count, 1))]
        self.used = 0

    def next(self):
        b = self.bufs[self.used % len(self.bufs)]
        self.used += 1
        return b

    def all_equal(self, expect) -> bool:
        """Every buffer a call wrote holds `expect` (a buffer written twice holds the last)."""
        written = self.bufs[:min(self.used, len(self.bufs))]
        return bool(written) and all(bool((b.to_numpy(np.int32) == expect).all()) for b in written)

    def free(self):
        for b in self.bufs:
            b.free()
        self.bufs = []


def timed(D, dist, step, steps, warmup):
    for _ in range(warmup):
        step()
    D.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    D.synchronize()
    if dist:
        dist.barrier()
    return time.perf_counter() - t0


# the kernel symbol of each verdict form counter / aggregate_verify path (the PMC traffic key)
FORM_KERNELS = {"fav_verdict_lg6": "mbls_k_fav_verdict_lg6", "fav_verdict_lg8": "mbls_k_fav_verdict_lg",
                "fav_verdict_lg16": "mbls_k_fav_verdict_lg16", "fav_verdict_1l": "mbls_k_fav_verdict",
                "path_av_grouped": "mbls_k_av_pairs_lg6", "path_av_onelane": "mbls_k_miller_pairs"}


def kernel_avgs(D, step, names, reps=2, forms=None):
    """Average launch ms of the named kernels over `reps` steps (HIP events on their streams);
    with `forms`, also {counter: launches} of those form / path counters over the same steps."""
    step()  # warm: code objects loaded, buffers allocated
    D.synchronize()
    D.prof_enable(True)
    D.prof_reset()
    for _ in range(reps):
        step()
    D.synchronize()
    out = {k: D.prof_read(k) for k in names}
    seen = {k: D.prof_read(k)[1] for k in (forms or ())}
    D.prof_enable(False)
    avgs = {k: (ms / max(n, 1)) for k, (ms, n) in out.items()}
    return (avgs, seen) if forms else avgs


def ran_kernel(seen):
    """The kernel symbol of the one form that ran (the traffic of the form the
    counters saw, not whichever form a PMC file happens to hold); None if none or several ran."""
    ran = [k for k, n in seen.items() if n]
    return FORM_KERNELS[ran[0]] if len(ran) == 1 else None


def other_workload(a, D, dist, rank, world):
    """gossip_verify (configs[1]), mainnet_block (configs[2]), deposit_av (configs[4])."""
    from lambda_ethereum_consensus_amd.rendezvous import runtime_libraries

    seed = a.seed
    roof = None
    # from the warm-up on, every call writes its own sentinel-filled status
    # buffer (StatusRing), all checked after the timed loop -- not one buffer overwritten per call
    ring = [None, None]  # [per-call status ring, the block's sync-aggregate ring]

    def out(i, fallback):
        return ring[i].next() if ring[i] is not None else fallback

    if a.workload == "gossip_verify":
        n = 65_536
        sk, _ = sks_for(n, seed, rank, b"gossip")
        msgs = msgs_for(n, seed, rank, b"gossip")
        d_sk, d_pk, d_m, d_sig = D.Buffer.from_host(sk.reshape(-1)), D.Buffer(48 * n), D.Buffer.from_host(msgs), D.Buffer(96 * n)
        D.sk_to_pk(d_sk, d_pk, n)
        D.sign(d_sk, d_m, d_sig, n)
        D.synchronize()
        st = D.Buffer(4 * n)

        def step():
            D.verify(d_pk, d_m, d_sig, out(0, st), n)

        units, unit_name = n, "verify sets"
        metric = "Bls.verify sets/sec (gossip attestation stream: 65,536 single-key verify, distinct messages)"
        config = {"workload": "gossip_verify", "sets_per_gpu": n, "keys_per_set": 1, "cold": True}
        expect = np.ones(n, dtype=np.int32)
        # (the prep: the two-wave hash_to_g2 + g2_sig_decode since r05, g2_prep with MBLS_PREP_SPLIT=0)
        ks, seen = kernel_avgs(D, step, ("g1_decode_validate", "g2_prep", "hash_to_g2", "g2_sig_decode", "fav_verdict"),
                               forms=("fav_verdict_lg6", "fav_verdict_lg8", "fav_verdict_lg16", "fav_verdict_1l"))
        dom, m_unit = "fav_verdict", M_VERIFY_VERDICT
        traffic_kernel = ran_kernel(seen)
    elif a.workload == "mainnet_block":
        kps, n_att = 512, 128
        d_pks, d_off, d_msgs, d_sigs, msgs, _ = make_inputs(D, n_att + 1, kps, seed, rank)
        # attestations: sets 0..127 (FAV); the sync aggregate: set 128 (eth_fast_aggregate_verify)
        pk_all = d_pks.to_numpy()
        sig_all = d_sigs.to_numpy()
        d_pk_a = D.Buffer.from_host(pk_all[:48 * kps * n_att])
        d_off_a = D.Buffer.from_host(np.arange(0, kps * n_att + 1, kps, dtype=np.uint32))
        d_m_a, d_s_a = D.Buffer.from_host(msgs[:32 * n_att]), D.Buffer.from_host(sig_all[:96 * n_att])
        d_pk_s = D.Buffer.from_host(pk_all[48 * kps * n_att:])
        d_off_s = D.Buffer.from_host(np.array([0, kps], dtype=np.uint32))
        d_m_s, d_s_s = D.Buffer.from_host(msgs[32 * n_att:]), D.Buffer.from_host(sig_all[96 * n_att:])
        st, st_s = D.Buffer(4 * n_att), D.Buffer(4)

        def step():
            D.fast_aggregate_verify(d_pk_a, d_off_a, d_m_a, d_s_a, out(0, st), n_att)
            D.fast_aggregate_verify(d_pk_s, d_off_s, d_m_s, d_s_s, out(1, st_s), 1, eth=True)

        units, unit_name = 1, "blocks"
        metric = "mainnet block signature checks/sec (128 x 512-key FAV + 512-key sync-aggregate eth_FAV)"
        config = {"workload": "mainnet_block", "attestations": n_att, "keys_per_set": kps, "cold": True}
        expect = np.ones(n_att, dtype=np.int32)
        ks = kernel_avgs(D, step, ("g1_decode_validate", "g1_aggregate", "g2_prep", "g2_sig_decode", "hash_to_g2",
                                   "sig_miller", "fav_verdict"))
        dom, m_unit = "g1_decode_validate", M_PER_KEY
        traffic_kernel = "mbls_k_g1_decode_validate"
    elif a.workload == "signing_roots":
        # AttestationData -> compute_signing_root (predicates.ex:118-121) for a
        # full epoch's worth of attestations, one domain per attestation, resident in HBM
        n = 1 << 20
        rng = np.random.default_rng(seed + 17 * rank)
        data = rng.integers(0, 256, size=(n, 128), dtype=np.uint8)
        doms = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        d_data, d_dom, d_out = D.Buffer.from_host(data.reshape(-1)), D.Buffer.from_host(doms.reshape(-1)), D.Buffer(32 * n)

        def step():
            D.attestation_data_signing_roots(d_data, d_dom, n, d_out)

        units, unit_name = n, "signing roots"
        metric = "AttestationData signing roots/sec (compute_signing_root, 2^20 attestations, per-object domains)"
        config = {"workload": "signing_roots", "attestations_per_gpu": n}
        expect = None
        ks = kernel_avgs(D, step, ("ssz_roots",))
        dom, m_unit = "ssz_roots", None
        traffic_kernel = None
        # spot check of a sample with hashlib (the parity tests compare against oracle/ssz.py)
        D.synchronize()
        out = d_out.to_numpy().reshape(n, 32)
        h = lambda x, y: hashlib.sha256(x + y).digest()
        z = bytes(32)
        leaf = lambda b8: b8 + bytes(24)
        for i in rng.integers(0, n, size=64):
            r = data[i].tobytes()
            src, tgt = h(leaf(r[48:56]), r[56:88]), h(leaf(r[88:96]), r[96:128])
            root = h(h(h(leaf(r[0:8]), leaf(r[8:16])), h(r[16:48], src)), h(h(tgt, z), h(z, z)))
            assert out[i].tobytes() == h(root, doms[i].tobytes()), "signing root mismatch"
    else:  # deposit_av
        n_sets, per = 16_384, 16
        n_pairs = n_sets * per
        sk, _ = sks_for(n_pairs, seed, rank, b"deposit")
        msgs = msgs_for(n_pairs, seed, rank, b"deposit")
        d_sk, d_pk, d_m = D.Buffer.from_host(sk.reshape(-1)), D.Buffer(48 * n_pairs), D.Buffer.from_host(msgs)
        d_sig1 = D.Buffer(96 * n_pairs)
        D.sk_to_pk(d_sk, d_pk, n_pairs)
        D.sign(d_sk, d_m, d_sig1, n_pairs)
        d_off = D.Buffer.from_host(np.arange(0, n_pairs + 1, per, dtype=np.uint32))
        d_sig, agg_st = D.Buffer(96 * n_sets), D.Buffer(4 * n_sets)
        D.aggregate_signatures(d_sig1, d_off, d_sig, agg_st, n_sets)
        D.synchronize()
        assert (agg_st.to_numpy(np.int32) == 2).all()
        d_sk.free()
        d_sig1.free()
        st = D.Buffer(4 * n_sets)

        def step():
            D.aggregate_verify(d_pk, d_m, d_off, d_sig, out(0, st), n_sets)

        units, unit_name = n_sets, "aggregate_verify sets"
        metric = "Bls.aggregate_verify sets/sec (16,384 sets x 16 distinct (pk, msg) pairs)"
        config = {"workload": "deposit_av", "sets_per_gpu": n_sets, "pairs_per_set": per, "cold": True}
        expect = np.ones(n_sets, dtype=np.int32)
        ks, seen = kernel_avgs(D, step, ("g1_decode_validate", "g2_sig_decode", "hash_to_g2", "miller_pairs",
                                         "av_verdict"), forms=("path_av_grouped", "path_av_onelane"))
        # the roofline kernel is the pairs' Miller loops (the longest kernel in
        # isolation, 37 vs 27 ms for H(m); under this line's concurrency H(m), keys and signature
        # decode overlap and their event-timed durations stretch, so the choice is fixed, not a max)
        dom, m_unit = "miller_pairs", M_AV_PAIRS_PER_SET
        traffic_kernel = ran_kernel(seen)
    lat_calls = 20 if a.workload == "mainnet_block" else 0
    if a.workload != "signing_roots":
        ring[0] = StatusRing(D, len(expect), a.warmup + a.steps + lat_calls)
        if a.workload == "mainnet_block":
            ring[1] = StatusRing(D, 1, a.warmup + a.steps + lat_calls)
    elapsed = timed(D, dist, step, a.steps, a.warmup)
    latency_ms = None
    if a.workload == "mainnet_block":
        # one block at a time (synchronised): the import-path latency, beside the pipelined rate
        lat = []
        for _ in range(lat_calls):
            t0 = time.perf_counter()
            step()
            D.synchronize()
            lat.append(time.perf_counter() - t0)
        latency_ms = round(float(np.median(lat)) * 1e3, 3)
    ok, checked = True, None
    if a.workload == "signing_roots":
        ok = True  # checked against the oracle above
    else:  # every call since the warm-up: its own buffer, no sentinel left, every verdict true
        ok = ring[0].all_equal(expect) and (ring[1] is None or ring[1].all_equal(np.ones(1, np.int32)))
        checked = min(ring[0].used, len(ring[0].bufs))
        for r in ring:
            if r is not None:
                r.free()
    if dist:
        elapsed, ok = reduce_over_ranks(dist, elapsed, ok)
    value = units * a.steps * world / elapsed
    avg_ms = ks.get(dom, 0.0)
    if a.workload == "signing_roots" and avg_ms > 0:
        # INT VALU bound (SHA-256): 10 two-block hashes per attestation, model 1,440 simple int
        # ops per general compression + 960 for the constant padding block,
        # against the measured v_add_u32 lane rate
        ops = units * 10 * (1440 + 960)
        roof = {"bound": "valu-int", "kernel": "attestation_signing_roots", "achieved": round(ops / (avg_ms / 1e3) / 1e12, 4),
                "peak": round(PEAK_INT_OPS_PER_S / 1e12, 4), "unit": "Tops/s",
                "frac": round(ops / (avg_ms / 1e3) / PEAK_INT_OPS_PER_S, 4), "traffic": None,
                "avg_launch_ms": round(avg_ms, 4), "bytes_per_unit": 192}
    elif m_unit is not None and avg_ms > 0:
        per_launch = {"fav_verdict": 65_536, "g1_decode_validate": 129 * 512, "hash_to_g2": 16_384 * 16,
                      "miller_pairs": 16_384}[dom] \
            if a.workload != "mainnet_block" else 129 * 512 / 2  # two FAV calls per block: mean keys per launch
        ach = per_launch * m_unit * MAC_PER_M / (avg_ms / 1e3)
        roof = {"bound": "valu-int", "kernel": dom, "achieved": round(ach / 1e12, 4),
                "peak": round(PEAK_MAD_PER_S / 1e12, 4), "unit": "Tmad/s", "frac": round(ach / PEAK_MAD_PER_S, 4),
                "traffic": None, "avg_launch_ms": round(avg_ms, 4)}
        if a.workload in ("deposit_av", "gossip_verify"):
            # r05: consecutive aggregate_verify / verify calls overlap (pipelined stages), so a
            # launch's event-timed duration includes the SIMD time of the next call's keys and H(m)
            # beside it; the same work priced at the step period is the kernel's rate as the line
            # sees it
            step_s = elapsed / a.steps
            roof["step_frac"] = round(per_launch * m_unit * MAC_PER_M / step_s / PEAK_MAD_PER_S, 4)
            roof["step_frac_basis"] = f"{dom}'s counted mads per call / the step period (calls overlap)"
        # this workload's PMC passes (tools/pmc_passes.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over
        # this same command): HBM bytes per launch of the dominant kernel, like `achieved` (the
        # block: mean over its two key launches)
        import glob

        tag = {"mainnet_block": "block", "gossip_verify": "gossip", "deposit_av": "deposit"}.get(a.workload)
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc_traffic_{tag}*.json"))) if tag else []
        if files:
            try:
                t = json.load(open(files[-1]))
                if a.workload == "mainnet_block" and dom == "g1_decode_validate":
                    roof["traffic"] = t.get("g1_decode_validate_bytes_per_launch")
                else:  # the form the counters saw run (ran_kernel), never a guess from the file
                    kern = t.get("kernels", {})
                    name = traffic_kernel if traffic_kernel in kern else None
                    roof["traffic"] = (kern.get(name) or {}).get("bytes_per_launch") if name else None
                    roof["traffic_kernel"] = name
                roof["traffic_source"] = os.path.relpath(files[-1], ROOT)
                roof.update(traffic_provenance(files[-1]))
            except Exception:
                pass
    if rank == 0:
        print(json.dumps({
            "metric": metric, "value": round(value, 3), "unit": unit_name + "/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32 (SHA-256 words)" if a.workload == "signing_roots"
            else "u32 (radix-2^28 Montgomery, int64 accumulate)",
            "data": "synthetic (seeded random AttestationData and domains)" if a.workload == "signing_roots"
            else "synthetic (deterministic keys/messages; signatures made by the engine's Sign kernel)",
            "config": config, "verdicts_ok": ok,
            **({"verdicts_checked_calls": checked} if checked is not None else {}), "roofline": roof,
            "kernels_avg_ms": {k: round(v, 4) for k, v in ks.items()},
            **({"block_latency_ms": latency_ms} if latency_ms is not None else {}),
            "runtime": runtime_libraries(),
        }), file=RESULT_OUT, flush=True)


# --------------------------------------------------------- strong scaling (shards) ----
def shard_bounds(key_off, parts):
    """contiguous chunks of sets balanced by key count -- the engine's own
    partition (mbls_plan_shards, host-only), so ranks and in-process engines split alike."""
    from lambda_ethereum_consensus_amd import device as D

    return D.plan_shards(np.diff(np.asarray(key_off, dtype=np.int64)), parts)


def gather_verdicts(dist, local):
    """Every rank's chunk of verdicts, concatenated in rank order (gloo; outside timed regions)."""
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, [int(x) for x in local])
    return np.array([c for p in parts for c in p], dtype=np.int32)


def sharded_verdicts(dist, rank, world, key_off, verify):
    """One batch split over the ranks: rank r verifies sets [b[r], b[r+1]) with verify(lo, hi)
    and the full verdict vector is gathered.  Returns (bounds, verdicts)."""
    b = shard_bounds(key_off, world)
    local = verify(b[rank], b[rank + 1])
    return b, gather_verdicts(dist, local)


def shard_leg(D, dist, rank, world, pks, key_off, msgs, sigs, steps, warmup):
    """Strong scaling (BASELINE.json configs[3] "sharded across 8 GPUs"): ONE 2,048-set epoch
    per step, split over the N ranks by key count (256 sets per GPU at N = 8); each rank's chunk
    is resident on its GPU; value = epoch sets x steps / max-over-ranks time."""
    key_off = np.asarray(key_off, dtype=np.uint32)
    n_sets = len(key_off) - 1
    b = shard_bounds(key_off, world)
    lo, hi = b[rank], b[rank + 1]
    k0, k1 = int(key_off[lo]), int(key_off[hi])
    n = hi - lo
    d_pk = D.Buffer.from_host(pks[48 * k0:48 * k1])
    d_off = D.Buffer.from_host((key_off[lo:hi + 1] - k0).astype(np.uint32))
    d_m = D.Buffer.from_host(msgs[32 * lo:32 * hi])
    d_s = D.Buffer.from_host(sigs[96 * lo:96 * hi])
    st = D.Buffer(4 * max(n, 1))

    def step():
        if n:
            D.fast_aggregate_verify(d_pk, d_off, d_m, d_s, st, n)

    el = timed(D, dist, step, steps, warmup)
    local = st.to_numpy(np.int32)[:n]
    full = gather_verdicts(dist, local) if dist else local
    ok = len(full) == n_sets and bool((full == 1).all())
    if dist:
        el, ok = reduce_over_ranks(dist, el, ok)
    return {"value": round(n_sets * steps / el, 3), "unit": "sets/s", "scaling": "strong", "steps": steps,
            "ms_per_step": round(el * 1e3 / steps, 3), "sets_per_step": n_sets, "bounds": b,
            "sets_per_gpu": [b[i + 1] - b[i] for i in range(world)], "verdicts_ok": ok}


# --------------------------------------------------------------------------- ranks -------
def reduce_over_ranks(dist, elapsed, ok):
    """Max of the timed region over ranks and AND of the verdict checks (any group with
    all_gather_object: the file rendezvous of the ranks, or a torch.distributed group)."""
    vals = [None] * dist.get_world_size()
    dist.all_gather_object(vals, [float(elapsed), bool(ok)])
    return max(v[0] for v in vals), all(v[1] for v in vals)


# --------------------------------------------------------------------------- main --------
# The one JSON line goes to the original stdout; everything else the process prints there
# (gloo / RCCL / runtime chatter from C++ at init and on first collectives) is sent to stderr.
RESULT_OUT = sys.stdout


def _claim_stdout():
    global RESULT_OUT
    sys.stdout.flush()
    RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def resolve_parallelism(gpus, multi, env):
    """How `--gpus N` maps onto processes (BASELINE.json: the metric at 1/2/4/8 GPUs).
    Returns (mode, n): "ranks" = this process is one of N ranks started by
    torch.distributed.run (one GPU each); "spawn" = run directly with N > 1 ranks wanted, so
    launch them; "engines" = N engines driven from this one process (mbls_init_devices);
    "single" = one GPU."""
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: need at least one GPU")
    world = int(env.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in env and world >= 1 and ("RANK" in env or world > 1):
        if gpus not in (1, world):
            raise SystemExit(f"--gpus {gpus} but torch.distributed.run started WORLD_SIZE={world} ranks")
        return ("ranks", world) if world > 1 else ("single", 1)
    if gpus == 1:
        return "single", 1
    return ("engines", gpus) if multi == "engines" else ("spawn", gpus)


def spawn_ranks(n, argv):
    """Start N ranks of this script under torch.distributed.run (one process per GPU, as the
    driver's multi-GPU runs do) as child processes -- before this process touched the GPU --
    forward their output and exit with their status."""
    import socket
    import subprocess

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    r = subprocess.run(cmd, stdout=RESULT_OUT, env=dict(os.environ, PYTHONUNBUFFERED="1"))
    return r.returncode


def engines_leg(D, a, n_eng):
    """--gpus N --multi engines: N engines in THIS process (mbls_init_devices(0..N-1), the
    one-BEAM-node deployment of SURVEY.md §8e), one host thread per engine, each verifying its
    own resident epoch per step (weak scaling, no exchange).  The timed region starts at a
    common barrier after every engine's warm-up and ends when the slowest engine has
    synchronised; every call of every engine has its own status buffer, all checked."""
    import threading

    have = D.device_count()
    if have < n_eng:
        raise SystemExit(f"--gpus {n_eng}: only {have} GPU(s) visible")
    D.init_devices(list(range(n_eng)))
    n_sets, kps = a.sets, a.keys_per_set
    start = threading.Barrier(n_eng + 1)
    done = [None] * n_eng
    oks = [False] * n_eng
    errs = []

    def run(j):
        try:
            D.select(j)
            d_pks, d_off, d_msgs, d_sigs, _msgs, _perm = make_inputs(D, n_sets, kps, a.seed, 0)
            ring = StatusRing(D, n_sets, a.steps)
            for _ in range(a.warmup):
                D.fast_aggregate_verify(d_pks, d_off, d_msgs, d_sigs, ring.bufs[0], n_sets)
            D.synchronize()
            ring.used = 0
            start.wait()
            for _ in range(a.steps):
                D.fast_aggregate_verify(d_pks, d_off, d_msgs, d_sigs, ring.next(), n_sets)
            D.synchronize()
            done[j] = time.perf_counter()
            oks[j] = ring.all_equal(np.ones(n_sets, dtype=np.int32))
        except BaseException as e:  # surfaced below; the barrier is released so no thread hangs
            errs.append(repr(e))
            start.abort()

    th = [threading.Thread(target=run, args=(j,)) for j in range(n_eng)]
    for x in th:
        x.start()
    try:
        start.wait()
    except threading.BrokenBarrierError:
        pass
    t0 = time.perf_counter()
    for x in th:
        x.join()
    if errs:
        raise RuntimeError(errs[0])
    elapsed = max(done) - t0
    return elapsed, all(oks)


def main():
    _claim_stdout()
    a = parse()
    mode, n_par = resolve_parallelism(a.gpus, a.multi, os.environ)
    if mode == "spawn":
        sys.exit(spawn_ranks(n_par, sys.argv[1:]))
    # Hardware queues of this process (HIP reads it at its first call; libmbls sizes its G2
    # stream pool from it and never changes the environment itself): 10 is the measured best
    # (two latency key streams + seven lane-group streams; r03 A/B one mainnet
    # block pipelined 157 -> 218 blocks/s at 6.44 ms latency, cold epoch unchanged), the boxes
    # export HIP's default 4.  MBLS_HW_QUEUES overrides.
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MBLS_HW_QUEUES", "10")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1")) if mode == "ranks" else 1
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        # the ranks meet through a file rendezvous, never torch: importing torch here would map
        # PyTorch-ROCm's own libamdhip64 / librccl before libmbls loads
        from lambda_ethereum_consensus_amd import rendezvous

        dist = rendezvous.init_from_env(rank, world)

    from lambda_ethereum_consensus_amd import device as D
    from lambda_ethereum_consensus_amd.rendezvous import runtime_libraries

    if mode == "engines":
        if a.workload != "epoch_replay_cold":
            raise SystemExit("--multi engines runs the headline workload (epoch_replay_cold) only")
        elapsed, ok = engines_leg(D, a, n_par)
        value = a.sets * a.steps * n_par / elapsed
        print(json.dumps({
            "metric": "fast_aggregate_verify sets/sec (512-key) at 1/2/4/8 MI355X vs host blst",
            "value": round(value, 3), "unit": "sets/s", "n_gpus": n_par, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (radix-2^28 Montgomery, int64 accumulate)",
            "data": "synthetic (deterministic keys/messages; signatures made by the engine's Sign kernel)",
            "config": {"workload": "epoch_replay_cold", "sets_per_gpu": a.sets, "keys_per_set": a.keys_per_set,
                       "validators_per_gpu": a.sets * a.keys_per_set, "cold": True,
                       "parallelism": f"{n_par} engines in one process (mbls_init_devices), independent sets"},
            "verdicts_ok": ok, "runtime": runtime_libraries()}), file=RESULT_OUT, flush=True)
        return
    # one process per GPU: rank -> its local device (MBLS_BENCH_DEVICE pins every rank to one
    # device, for rehearsing the N > 1 path on a one-GPU box; never for a measured run)
    if mode == "ranks" and "MBLS_BENCH_DEVICE" not in os.environ and D.device_count() < world:
        raise SystemExit(f"{world} ranks but only {D.device_count()} GPU(s) visible")
    D.init(int(os.environ.get("MBLS_BENCH_DEVICE", local_rank)))
    if a.workload != "epoch_replay_cold":
        other_workload(a, D, dist, rank, world)
        if dist:
            dist.destroy_process_group()
        return
    assert "torch" not in sys.modules, "a rank must not import torch (its bundled HIP runtime)"
    n_sets, kps = a.sets, a.keys_per_set
    # every rank builds the same epoch (seed of rank 0): the weak-scaling headline has each rank
    # verify all of it (one independent batch per GPU), the strong leg splits it over the ranks,
    # and the sharded table build needs one registry on every rank anyway
    data_rank = 0
    d_pks, d_off, d_msgs, d_sigs, msgs, perm = make_inputs(D, n_sets, kps, a.seed, data_rank)
    verdicts_ok = check_verdicts(D, d_pks, d_off, msgs, d_sigs, n_sets)
    st = D.Buffer(4 * n_sets)
    # every timed call writes its own status buffer; all of them are checked after the loop
    ring = StatusRing(D, n_sets, a.steps)

    def step():
        D.fast_aggregate_verify(d_pks, d_off, d_msgs, d_sigs, st, n_sets)

    for _ in range(a.warmup):
        step()
    D.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        D.fast_aggregate_verify(d_pks, d_off, d_msgs, d_sigs, ring.next(), n_sets)
    D.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    all_valid = ring.all_equal(np.ones(n_sets, dtype=np.int32))
    ring.free()
    if dist:
        elapsed, verdicts_ok = reduce_over_ranks(dist, elapsed, verdicts_ok and all_valid)
    sets_total = n_sets * a.steps * world
    value = sets_total / elapsed

    roofline = None
    if not a.no_roofline:
        # dominant kernel timed with HIP events on the stream it runs on (engine hooks)
        D.prof_enable(True)
        D.prof_reset()
        reps = max(2, min(a.steps, 3))
        for _ in range(reps):
            step()
        D.synchronize()
        ms, launches = D.prof_read("g1_decode_validate")
        tails = {k: D.prof_read(k) for k in ("g1_aggregate", "g2_prep", "g2_sig_decode", "hash_to_g2", "fav_verdict")}
        D.prof_enable(False)
        avg_s = ms / 1e3 / max(launches, 1)
        n_keys = n_sets * kps
        achieved = n_keys * MAC_PER_KEY / avg_s
        traffic, traffic_src = None, a.traffic_file or newest_traffic_file()
        if traffic_src and os.path.exists(traffic_src):
            try:
                traffic = json.load(open(traffic_src)).get("g1_decode_validate_bytes_per_launch")
            except Exception:
                traffic = None
        roofline = {
            "bound": "valu-int",
            "kernel": "g1_decode_validate",
            "achieved": round(achieved / 1e12, 4),
            "peak": round(PEAK_MAD_PER_S / 1e12, 4),
            "unit": "Tmad/s",
            "frac": round(achieved / PEAK_MAD_PER_S, 4),
            "peak_guide": round(PEAK_MAD_GUIDE / 1e12, 4),
            "frac_guide": round(achieved / PEAK_MAD_GUIDE, 4),
            "traffic": traffic,
            "traffic_source": os.path.relpath(traffic_src, ROOT) if traffic is not None else None,
            **(traffic_provenance(traffic_src) if traffic is not None else {}),
            "avg_launch_ms": round(avg_s * 1e3, 4),
            "units_per_launch": n_keys,
            "mad_per_unit": MAC_PER_KEY,
            "mad_per_unit_basis": "counted device Fp products (profiles/r03_work_model.json units.key.M = 1,482) x 300",
            "frac_app_b": round(n_keys * M_PER_KEY_APP_B * MAC_PER_M / avg_s / PEAK_MAD_PER_S, 4),
            "other_kernels_avg_ms": {k: round(v[0] / max(v[1], 1), 4) for k, v in tails.items()},
        }

    rlc = None
    if not a.no_rlc:
        # opt-in random-linear-combination batch check: not the headline
        rring = StatusRing(D, n_sets, a.steps + a.warmup)

        def step_rlc():
            D.fast_aggregate_verify(d_pks, d_off, d_msgs, d_sigs, rring.next(), n_sets, rlc=True)

        el = timed(D, dist, step_rlc, a.steps, a.warmup)
        ok = rring.all_equal(np.ones(n_sets, dtype=np.int32))
        rring.free()
        if dist:
            el, ok = reduce_over_ranks(dist, el, ok)
        rlc = {"value": round(n_sets * a.steps * world / el, 3), "unit": "sets/s",
               "ms_per_step": round(el * 1e3 / a.steps, 3), "verdicts_ok": ok,
               "note": "opt-in MBLS_FAV_RLC: one combined pairing check per batch, exact fallback; "
                       "equals exact verdicts except with probability <= 2^-64 per batch"}

    mixed = host_e2e = None
    if not a.no_extra_legs:
        mixed = mixed_leg(D, d_pks, d_off, msgs, d_sigs, n_sets, a.steps, dist)
        host_e2e = host_e2e_leg(D, d_pks, msgs, d_sigs, n_sets, kps, max(2, min(a.steps, 20)), dist)

    warm = None
    if not a.no_warm:
        if a.table_build == "sharded" and dist is not None:
            comm_setup(D, dist)
        warm = warm_leg(D, d_pks, d_off, d_msgs, d_sigs, perm, n_sets, a.steps, a.warmup, dist, rlc_too=not a.no_rlc,
                        table_build=a.table_build)

    sharded = None
    if world > 1 and not a.no_warm and a.table_build != "sharded":
        sharded = sharded_table_leg(D, d_pks, d_off, d_msgs, d_sigs, perm, n_sets, a.steps, a.warmup, dist)

    strong = None
    if world > 1 or a.shard:
        strong = shard_leg(D, dist, rank, world, d_pks.to_numpy(), d_off.to_numpy(np.uint32), msgs,
                           d_sigs.to_numpy(), a.steps, a.warmup)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cores = min(16, os.cpu_count() or 1)
        try:
            if os.path.exists(os.path.join(ROOT, "oracle", "c", "libblsoracle.so")):
                cpu = cpu_baseline_c(D, d_pks, msgs, d_sigs, kps, a.cpu_baseline_seconds, cores)
            else:
                cpu = cpu_baseline(D, d_pks, msgs, d_sigs, kps, a.cpu_baseline_seconds, cores)
        except Exception as e:  # the baseline never hides the GPU line
            cpu = {"value": None, "unit": "sets/s", "cores": cores, "kind": "port", "sample": f"failed: {e}"}

    if rank == 0:
        line = {
            "metric": "fast_aggregate_verify sets/sec (512-key) at 1/2/4/8 MI355X vs host blst",
            "value": round(value, 3),
            "unit": "sets/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (radix-2^28 Montgomery, int64 accumulate)",
            "data": "synthetic (deterministic keys/messages; signatures made by the engine's Sign kernel)",
            "config": {
                "workload": "epoch_replay_cold",
                "sets_per_gpu": n_sets,
                "keys_per_set": kps,
                "validators_per_gpu": n_sets * kps,
                "cold": True,
                "parallelism": f"independent sets, {world} rank(s)",
            },
            "verdicts_ok": bool(verdicts_ok and all_valid),
            "roofline": roofline,
            "warm": warm,
            "warm_sharded_table": sharded,
            "strong": strong,
            "mixed": mixed,
            "host_e2e": host_e2e,
            "rlc": rlc,
            "cpu_baseline": cpu,
            "runtime": runtime_libraries(),
        }
        if cpu and cpu.get("warm") and warm and warm.get("value"):
            # the warm GPU line against the App. B blst ESTIMATE on all host cores (north_star's 20x
            # is posed against blst, which this image cannot run), beside the measured port ratio
            est = cpu["warm"]["blst_app_b_estimate"]["value"]
            cpu["warm"]["gpu_warm_vs_blst_app_b_estimate"] = round(warm["value"] / est, 2)
            cpu["warm"]["gpu_warm_vs_port_all_host_cores_estimate"] = round(
                warm["value"] / cpu["warm"]["all_host_cores_estimate"]["value"], 2)
        if a.shard and strong is not None:
            # --shard: the strong-scaling figure is the headline (one epoch per step over N GPUs)
            line.update(value=strong["value"], ms_per_step=strong["ms_per_step"], scaling="strong",
                        verdicts_ok=bool(line["verdicts_ok"] and strong["verdicts_ok"]))
            line["config"].update(sets_per_gpu=strong["sets_per_gpu"],
                                  parallelism=f"one epoch split over {world} rank(s) by key count")
        print(json.dumps(line), file=RESULT_OUT, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

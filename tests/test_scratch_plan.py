"""CPU: the engine's scratch plan against the kernels' frame sizes.

The runtime backs every hardware queue's scratch out of one pool per device and keeps a
queue's block sized for a full-device dispatch of the largest frame it ran (measured:
tools/scratch_probe.hip -> profiles/r05_scratch_probe.json).  Two r04 runs aborted with
HSA_STATUS_ERROR_OUT_OF_RESOURCES that way (profiles/r04_ab18_fill_retune.txt,
r04_ab11_defer_window.txt).  Here, without a GPU:

* the frames come from libmbls's own gfx950 code objects (the .hip_fatbin bundles of the shipped
  libmbls.so, read with the LLVM tools), and the engine's priced kernel list
  (mbls_scratch_kernel) covers every kernel that has a frame;
* with the measured pool / threshold / CU count and the ten hardware queues every stream of the
  process maps onto (GPU_MAX_HW_QUEUES), the plan
  (mbls_scratch_plan) is safe for ANY assignment of kernels to queues, and the r04 state --
  the runtime's threshold left alone -- is not;
* the r04 bench process's actual per-queue blocks left less free pool than one queue's growth
  step, the mechanism of the two aborts.
"""
import json
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from lambda_ethereum_consensus_amd import _lib
from lambda_ethereum_consensus_amd import device as D

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
PROBE = os.path.join(ROOT, "profiles", "r05_scratch_probe.json")
HW_QUEUES = 10  # what bench.py, the tests and smoke() run with (GPU_MAX_HW_QUEUES)


def code_object_frames():
    """{kernel: private segment bytes per lane} over every gfx950 code object in libmbls.so."""
    if not all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler",
                                                               "llvm-readelf")):
        pytest.skip("LLVM tools not available")
    tmp = tempfile.mkdtemp()
    try:
        sec = os.path.join(tmp, "fatbin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + sec, _lib.LIB_PATH,
                        os.path.join(tmp, "copy.so")], check=True, capture_output=True)
        data = open(sec, "rb").read()
        starts = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", data)]
        frames = {}
        for i, a in enumerate(starts):
            chunk = os.path.join(tmp, f"b{i}")
            with open(chunk, "wb") as f:
                f.write(data[a:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = chunk + ".co"
            r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                                "--input=" + chunk, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co],
                               capture_output=True)
            if r.returncode or not os.path.getsize(co):
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            for blk in notes.split("  - .agpr_count:")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)
                frames[name] = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1))
        return frames
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


@pytest.fixture(scope="module")
def frames():
    f = code_object_frames()
    assert len(f) >= 40, sorted(f)
    return f


@pytest.fixture(scope="module")
def probe():
    return json.load(open(PROBE))


def test_engine_prices_every_kernel_with_a_frame(frames):
    priced = set(D.scratch_kernels())
    with_frame = {k for k, v in frames.items() if v > 0}
    assert with_frame <= priced, sorted(with_frame - priced)
    assert priced <= set(frames), sorted(priced - set(frames))  # no stale names either


def test_probe_record_backs_the_model(probe):
    """The measured facts the plan rests on: one pool shared by all queues, a retain threshold
    below it, and a retained block = frame x 64 lanes x 32 wave slots x CUs whatever the grid."""
    a = probe["agents"][0]
    slots = 64 * 32 * probe["cus"]
    assert a["scratch_limit_max"] == 32 << 30 and a["scratch_limit_current"] == 24 << 30
    rows = {r["step"]: r for r in probe["retained"]}
    assert rows["s1 full grid (8192 waves) ~2.2 KB frame"]["free_mem_drop_bytes"] == 2256 * slots
    assert rows["s3 one wave ~4.2 KB frame"]["free_mem_drop_bytes"] == 4256 * slots     # one wave: full size
    assert rows["s2 one wave ~9.4 KB frame"]["free_mem_drop_bytes"] == 9424 * slots
    assert rows["s0 again, same frame"]["free_mem_drop_bytes"] == 0                      # kept, not re-taken
    assert rows["s1 one wave ~5.2 KB frame (grows)"]["free_mem_drop_bytes"] == (5216 - 2256) * slots
    assert probe["use_once"]["set_limit_status"] == 0 and probe["use_once"]["retained_after_one_wave"] == 0


def priced(frames):
    """(frames, gated flags) of the engine's priced kernels that have a frame."""
    gated = set(D.scratch_gated_kernels())
    ks = [k for k in D.scratch_kernels() if frames.get(k, 0) > 0]
    return [frames[k] for k in ks], [k in gated for k in ks], ks


def test_gated_kernels_are_the_use_once_ones(frames):
    """The engine gates exactly Sign, the one-lane verdicts and the two-wave H(m)."""
    assert set(D.scratch_gated_kernels()) == {"mbls_k_sign", "mbls_k_fav_verdict", "mbls_k_av_verdict",
                                              "mbls_k_hash_to_g2"}


@pytest.mark.parametrize("queues", [4, 10, 11, 12, 32])
def test_plan_with_the_gate_bounds_the_pool_for_any_queue_count(frames, probe, queues):
    """with Q queues, every queue keeps at most the threshold's block and the
    use-once gate lets all live use-once blocks -- any number of concurrent dispatches, on any
    queues -- hold at most use_once_budget = pool - Q x threshold, which holds the largest
    full-device use-once block; every ungated frame is retained (the gate never sees it).  Where
    no threshold satisfies that, the plan is unsafe and the engine refuses to initialise
    (MBLS_ERR_SCRATCH_PLAN)."""
    a = probe["agents"][0]
    pool, cur, cus = a["scratch_limit_max"], a["scratch_limit_current"], probe["cus"]
    slots = 64 * 32 * cus
    fr, gated, ks = priced(frames)
    plan = D.scratch_plan(pool, cur, queues, cus, fr, gated)
    ungated_max = max(f for f, g in zip(fr, gated) if not g)
    largest_once = max([f * slots for f in fr if f * slots > plan["retain_bytes"]], default=0)
    if queues * ungated_max * slots + max(fr) * slots <= pool:
        assert plan["safe"], plan
        assert plan["worst_retained"] == queues * plan["retain_bytes"]
        assert plan["use_once_budget"] == pool - plan["worst_retained"]
        # retained blocks + everything the gate admits <= pool, for ANY mix of dispatches
        assert plan["worst_retained"] + plan["use_once_budget"] <= pool
        if largest_once:
            assert plan["use_once_budget"] >= largest_once  # a full-device use-once always admissible
        for f, g, k in zip(fr, gated, ks):
            if not g:
                assert f <= plan["max_retained_frame"], k  # ungated kernels never run use-once
    else:
        assert not plan["safe"], plan
    if queues == 4:  # HIP's default: every frame retained, nothing use-once
        assert plan["safe"] and plan["max_retained_frame"] == max(fr)
    if queues == 10:  # the shipped configuration
        assert plan["safe"] and plan["max_retained_frame"] == frames["mbls_k_g2_prep_1l"]
    if queues == 32:  # 32 queues x the one-lane prep's block alone exceed the pool
        assert not plan["safe"]


def test_plan_is_safe_for_any_queue_assignment(frames, probe):
    a = probe["agents"][0]
    pool, cur, cus = a["scratch_limit_max"], a["scratch_limit_current"], probe["cus"]
    fr = [v for v in frames.values() if v > 0]
    plan = D.scratch_plan(pool, cur, HW_QUEUES, cus, fr)
    slots = 64 * 32 * cus
    assert plan["safe"] and plan["max_frame"] == max(fr)
    # every queue may keep up to the threshold, and one full-device use-once dispatch fits beside
    assert plan["worst_retained"] + plan["worst_use_once"] <= pool
    assert plan["retain_bytes"] == plan["max_retained_frame"] * slots <= cur
    # exhaustive over assignments: a queue keeps the largest retained frame it ran, so the worst
    # case is every queue having run the largest frame not above the threshold
    kept = max([f for f in fr if f * slots <= plan["retain_bytes"]], default=0)
    once = max([f for f in fr if f * slots > plan["retain_bytes"]], default=0)
    assert HW_QUEUES * kept * slots + once * slots <= pool
    # the preps and the pairs' Miller loops stay retained (a use-once dispatch per pipelined
    # table call cost 11% of the warm epoch, profiles/r05_scratch_ab.txt); Sign, the one-lane
    # verdicts and aggregate_verify's two-wave H(m) (one dispatch per batch) are use-once
    for k in ("mbls_k_g2_prep_1l", "mbls_k_miller_pairs", "mbls_k_g2_prep_lg6", "mbls_k_fav_verdict_lg6",
              "mbls_k_sig_miller"):
        assert frames[k] <= plan["max_retained_frame"], k
    for k in ("mbls_k_sign", "mbls_k_fav_verdict", "mbls_k_av_verdict", "mbls_k_hash_to_g2"):
        assert frames[k] > plan["max_retained_frame"], k
    # and the threshold is the largest such: the next frame up would not fit
    bigger = sorted(f for f in set(fr) if f > plan["max_retained_frame"] and f * slots <= cur)
    if bigger:
        nxt = bigger[0]
        once_n = max([f for f in fr if f > nxt], default=0)
        assert HW_QUEUES * nxt * slots + once_n * slots > pool


def test_r04_threshold_was_unsafe_and_the_aborts_follow(frames, probe):
    a = probe["agents"][0]
    pool, cur, cus = a["scratch_limit_max"], a["scratch_limit_current"], probe["cus"]
    slots = 64 * 32 * cus
    fr = [v for v in frames.values() if v > 0]
    # leaving the runtime's 24 GiB threshold: every frame is retained, ten queues x the largest
    # is far past the pool
    assert HW_QUEUES * max(fr) * slots > pool
    # the r04 bench process: three one-lane streams (one-lane verdict), five more G2 streams
    # (one-lane prep, table calls), the engine stream (Sign while making inputs) -- with the r04
    # code objects' frames (the r05 Jacobian [|x|] of hash_to_G2 shrank the prep's and Sign's;
    # the shipped ones are no larger)
    r04f = {"mbls_k_fav_verdict": 9428, "mbls_k_g2_prep_1l": 5232, "mbls_k_sign": 7104}
    assert all(frames[k] <= v for k, v in r04f.items()), {k: frames[k] for k in r04f}
    r04 = 3 * r04f["mbls_k_fav_verdict"] + 5 * r04f["mbls_k_g2_prep_1l"] + r04f["mbls_k_sign"]
    held = r04 * slots
    free = pool - held
    growth = r04f["mbls_k_g2_prep_1l"] * slots  # a queue moving from the lane-group prep's frame
    assert held < pool and free < growth, (held / 1e9, free / 1e9, growth / 1e9)
    # ... to the one-lane prep's needs a whole new block: the pool held it only if the queue's
    # own freed block happened to lie next to the free space (aborted with fill = 4, window 2)
    assert frames["mbls_k_g2_prep_lg"] < r04f["mbls_k_g2_prep_1l"]


def test_plan_edge_cases():
    slots = 64 * 32 * 256
    p = D.scratch_plan(32 << 30, 24 << 30, 11, 256, [])
    assert p["safe"] and p["retain_bytes"] == 0 and p["worst_use_once"] == 0
    p = D.scratch_plan(1 << 30, 24 << 30, 11, 256, [9428])  # one full-device frame exceeds the pool
    assert not p["safe"]
    p = D.scratch_plan(32 << 30, 1 << 30, 11, 256, [176, 5232])  # the runtime's own threshold is lower
    assert p["safe"] and p["max_retained_frame"] == 176 and p["retain_bytes"] == 176 * slots
    with pytest.raises(RuntimeError):
        D.scratch_plan(32 << 30, 24 << 30, 0, 256, [1])
    # an ungated frame must stay retained: 10 queues x 5,232 B plus the gated 9,428 B fit,
    # 12 do not -- and then no lower threshold is allowed
    p = D.scratch_plan(32 << 30, 24 << 30, 10, 256, [5232, 9428], [False, True])
    assert p["safe"] and p["max_retained_frame"] == 5232
    p = D.scratch_plan(32 << 30, 24 << 30, 12, 256, [5232, 9428], [False, True])
    assert not p["safe"]
    p = D.scratch_plan(32 << 30, 24 << 30, 12, 256, [5232, 9428])  # all gated: a lower threshold
    assert p["safe"] and p["max_retained_frame"] == 0 and p["use_once_budget"] == 32 << 30

"""Every engine knob that selects a verdict, prep or stream form has a parity test that pins
the form (a stray MBLS_* variable in a BEAM node's environment must never select
an unverified path).  Each case runs in a child process with the knob set, compares every
verdict with the oracle, and asserts through the per-form / per-path counters
(mbls_prof_read "fav_verdict_*" / "path_*") that the forced form decided EVERY call (exact
counts).

Knob -> case:
  MBLS_WARM_PREP=lg            table_epoch-warm-prep-lg        (2,048-set table calls, lane-group prep)
  MBLS_WARM_FILL=0             table_epoch-fill-0              (no lane-group prep during the pipeline fill)
  MBLS_WARM_FILL=4             table_epoch-fill-4              (the value whose run aborted in r04: scratch plan)
  MBLS_DEFER_VERDICT=0         table_epoch-fill-0-defer-0      (table verdicts launched at once)
  MBLS_MILLER=split / joint    table_epoch-miller-split, small-miller-joint
  MBLS_FAV_VERDICT=lg          small-cold-fav-verdict-lg       (non-critical cold calls on lane groups)
  MBLS_KEY_STREAMS=2 / 1       small-cold-key-streams-2, verify-key-streams-1
  MBLS_VERIFY_VERDICT=1l       verify-one-lane                 (Bls.verify verdicts one lane per set)
  MBLS_LAT_KEY_STREAMS=1       small-lat-key-streams-1
  MBLS_AV_FORM=grouped         av-grouped                      (aggregate_verify joint Miller loops on 6-lane groups)
and the defaults they replace: small-default, table_epoch-default, verify-default.  (The
lane-group verdict / prep / chain knobs MBLS_LG16, MBLS_LG16_PREP, MBLS_LAT_SPLIT, MBLS_LG6,
MBLS_LG6_CHAIN, MBLS_DEFER_VERDICT, MBLS_G2_CRITICAL_KEYS and MBLS_AGG_LANES* are pinned in
tests/test_gpu_parity.py.)
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COLD1L = {"MBLS_G2_CRITICAL_KEYS": "0", "MBLS_DEFER_VERDICT": "0"}  # small batches down the cold path

CASES = {
    # small ragged / invalid sets (tests/_onelane_child.py), two device calls (a host batch call
    # between them takes the other latency key stream, so both device calls take the second)
    "small-default": ("small", {}, "lg16", "prep_lg=2,miller_split=2,lat_kstream2=2"),
    "small-lat-key-streams-1": ("small", {"MBLS_LAT_KEY_STREAMS": "1"}, "lg16", "prep_lg=2,lat_kstream2=0"),
    "small-miller-joint": ("small", {"MBLS_MILLER": "joint"}, "lg16", "prep_lg=2,miller_joint=2,miller_split=0"),
    "small-cold-one-lane": ("small", COLD1L, "1l", "prep_1l_cold=2,key_alt=0,prep_split=0"),
    "small-cold-key-streams-2": ("small", dict(COLD1L, MBLS_KEY_STREAMS="2"), "1l", "prep_1l_cold=2,key_alt=1"),
    # the cold one-lane prep as the two-wave hash + decode kernels (MBLS_PREP_SPLIT mask 2)
    "small-cold-prep-split": ("small", dict(COLD1L, MBLS_PREP_SPLIT="2"), "1l", "prep_1l_cold=2,prep_split=2"),
    "small-cold-fav-verdict-lg": ("small", {"MBLS_G2_CRITICAL_KEYS": "0", "MBLS_FAV_VERDICT": "lg"}, "lg16",
                                  "prep_1l_cold=2,miller_split=2"),
    # 2,048-set table calls (the pipelined warm form)
    # 2,048-set table calls (the pipelined warm form).  The first call starts an empty pipeline, so
    # by default it takes the fill's lane-group prep; both G2 sides are deferred: the first
    # launched by the second call, the second by the synchronize (lane-group prep either way --
    # the latency form -- then the 6-lane verdict, counted lg6 since r05).
    "table_epoch-default": ("table_epoch", {}, "lg6",
                            "prep_lg=2,warm_fill=1,warm_defer=2,prep_1l_table=0,miller_joint=2"),
    "table_epoch-fill-2": ("table_epoch", {"MBLS_WARM_FILL": "2"}, "lg6",
                           "prep_lg=2,warm_fill=2,warm_defer=2,prep_1l_table=0,miller_joint=2"),
    # MBLS_WARM_FILL=4 ran the runtime's scratch pool out in r04 (profiles/r04_ab18_fill_retune.txt);
    # with the scratch plan (csrc/mbls_engine.cpp apply_scratch_plan) any value is safe
    "table_epoch-fill-4": ("table_epoch", {"MBLS_WARM_FILL": "4"}, "lg6",
                           "prep_lg=2,warm_fill=2,warm_defer=2,prep_1l_table=0,miller_joint=2"),
    # the padded 8-lane verdict (MBLS_LG6=0) on the same calls: its own counter
    "table_epoch-lg6-0": ("table_epoch", {"MBLS_LG6": "0"}, "lg8",
                          "prep_lg=2,warm_fill=1,warm_defer=2,prep_1l_table=0,miller_joint=2"),
    "table_epoch-fill-0": ("table_epoch", {"MBLS_WARM_FILL": "0"}, "lg6",
                           "prep_1l_table=1,prep_lg=1,warm_fill=0,warm_defer=2,miller_joint=2"),
    "table_epoch-fill-0-defer-0": ("table_epoch", {"MBLS_WARM_FILL": "0", "MBLS_DEFER_VERDICT": "0"}, "lg6",
                                   "prep_1l_table=2,warm_defer=0,miller_joint=2,prep_split=0"),
    "table_epoch-warm-prep-lg": ("table_epoch", {"MBLS_WARM_PREP": "lg"}, "lg6",
                                 "prep_lg=2,prep_1l_table=0,warm_fill=0,warm_defer=2"),
    # the table one-lane prep split (MBLS_PREP_SPLIT mask 4; slower in the warm pipeline, r05)
    "table_epoch-prep-split": ("table_epoch", {"MBLS_PREP_SPLIT": "4", "MBLS_WARM_FILL": "0", "MBLS_DEFER_VERDICT": "0"},
                               "lg6", "prep_1l_table=2,prep_split=2,warm_defer=0"),
    "table_epoch-miller-split": ("table_epoch", {"MBLS_MILLER": "split", "MBLS_WARM_FILL": "0"}, "lg6",
                                 "prep_1l_table=2,miller_split=2,miller_joint=0,warm_defer=0"),
    # Bls.verify batches: the one-lane prep split into the two-wave hash + decode kernels by
    # default (MBLS_PREP_SPLIT mask 1, r05), fused with MBLS_PREP_SPLIT=0
    "verify-default": ("verify", {}, "lg16", "verify_key_alt=1,prep_split=2"),  # (<= 1,024 sets: 16-lane groups)
    "verify-prep-fused": ("verify", {"MBLS_PREP_SPLIT": "0"}, "lg16", "verify_key_alt=1,prep_split=0"),
    "verify-one-lane": ("verify", {"MBLS_VERIFY_VERDICT": "1l"}, "1l", "verify_key_alt=1,prep_split=2"),
    "verify-key-streams-1": ("verify", {"MBLS_KEY_STREAMS": "1"}, "lg16", "verify_key_alt=0"),
    # aggregate_verify: the key pairs one lane per couple (default) and the grouped joint Miller
    # loops on 6-lane groups (MBLS_AV_FORM=grouped, r05)
    "av-default": ("av", {}, "", "av_grouped=0,av_onelane=1,av_pipelined=1"),
    "av-grouped": ("av", {"MBLS_AV_FORM": "grouped"}, "", "av_grouped=1,av_onelane=0,av_pipelined=0"),
    # three back-to-back pipelined calls; the use-once gate with its planned budget,
    # and squeezed to one byte so every H(m) dispatch must wait for the earlier ones
    "av-pipe": ("av_pipe", {}, "", "av_onelane=3,av_pipelined=3"),
    "av-pipe-gate-tight": ("av_pipe", {"MBLS_USE_ONCE_BUDGET": "1", "MBLS_EXPECT_GATE_WAITS": "1"}, "",
                           "av_onelane=3,av_pipelined=3"),
}


@pytest.mark.parametrize("case", list(CASES))
def test_knob_forms(case):
    scenario, knobs, form, paths = CASES[case]
    env = dict(os.environ, **knobs, MBLS_EXPECT_FORM=form, MBLS_EXPECT_PATHS=paths, MBLS_SCENARIO=scenario)
    mod = "tests._onelane_child" if scenario == "small" else "tests._forced_forms_child"
    r = subprocess.run([sys.executable, "-m", mod], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]


def test_deferred_launch_error_stays_with_its_engine():
    """a failed deferred launch on engine 1 does not fail engine 0's copies and
    frees; engine 1's synchronize reports it once; a d2h from engine 1's thread reads engine 0's
    deferred verdict after it ran."""
    env = dict(os.environ, MBLS_SCENARIO="defer_error", MBLS_G2_CRITICAL_KEYS="0")
    r = subprocess.run([sys.executable, "-m", "tests._forced_forms_child"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]


def test_two_engine_overwrite_right_after_a_call():
    """an input of a call enqueued on engine 0 overwritten right away from
    engine 1 -- synchronously (mbls_dev_memcpy_h2d drains EVERY engine) and stream-ordered
    (mbls_dev_memcpy_h2d_async) -- leaves the call's verdicts those of the original inputs."""
    env = dict(os.environ, MBLS_SCENARIO="overwrite")
    r = subprocess.run([sys.executable, "-m", "tests._forced_forms_child"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]


def test_two_engine_overwrite_of_a_deferred_table_call():
    """A pipelined table call leaves its signature decode + H(m) deferred (r04): its signatures
    overwritten from another engine right after the call -- mbls_dev_memcpy_h2d and the
    stream-ordered mbls_dev_memcpy_h2d_async -- must not reach the verdicts."""
    env = dict(os.environ, MBLS_SCENARIO="table_overwrite")
    r = subprocess.run([sys.executable, "-m", "tests._forced_forms_child"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]

"""rt_render_sharded's cross-rank agreement rule on the CPU (csrc/rt/keycheck.h through tools/keycheck_sim):
every call all-gathers each rank's (scene digest, call key) on every rank, and the words are checked in the
call when the rank's key is new (or in strict mode), else at its next call.  The scenarios: a steady loop of
frames (one immediate check, then deferred ones: no host round trip), every rank changing its arguments
together (checked in the call, on every rank), a genuine mismatch between ranks that all changed (every rank
fails in the call, before any frame collective), and the misuse of one rank changing its key alone (that
rank fails in the call; its peers fail at their next call's deferred check; strict mode fails them all in
the call).  A failed check poisons the communicator: every later call on it fails at once and
issues no collective, so no rank's all-gather is ever paired with a peer's pending frame collective.  The reference loop this check guards is main.rs:117-125 (one process, no ranks)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "keycheck_sim.cpp")


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("keycheck") / "keycheck_sim")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-o", exe, SRC], check=True, timeout=120)

    def run(world, strict, *calls):
        args = [str(world), "1" if strict else "0"] + [",".join(c) for c in calls]
        out = subprocess.run([exe] + args, check=True, capture_output=True, text=True, timeout=60).stdout
        return [line.split() for line in out.strip().split("\n")]
    return run


def test_steady_loop_checks_once_then_defers(sim):
    rows = sim(4, False, *[["a"] * 4] * 5)
    assert rows[0] == ["S"] * 4 + ["gather=same", "pairing=ok"]
    for r in rows[1:]:
        assert r == ["A"] * 4 + ["gather=same", "pairing=ok"]


def test_all_ranks_change_together(sim):
    rows = sim(3, False, ["a"] * 3, ["a"] * 3, ["b"] * 3, ["b"] * 3)
    assert [r[:3] for r in rows] == [["S"] * 3, ["A"] * 3, ["S"] * 3, ["A"] * 3]
    assert all(r[3] == "gather=same" for r in rows)


def test_mismatch_after_a_common_change_fails_every_rank_in_the_call(sim):
    # all ranks change their arguments at call 2, rank 2 to different ones: every rank checks in the call
    # (its key is new) and fails naming rank 2, before any frame collective; a corrected call 3 agrees
    rows = sim(4, False, ["a"] * 4, ["a"] * 4, ["b", "b", "c", "b"], ["b"] * 4)
    assert rows[2] == ["F2k"] * 4 + ["gather=same", "pairing=ok"]
    # every rank's communicator is poisoned by the failed check: the corrected call must re-create it
    assert rows[3] == ["X"] * 4 + ["gather=diverged", "pairing=ok"]


def test_scene_mismatch_is_named_as_scene(sim):
    rows = sim(2, False, ["1:a", "2:a"])
    assert rows[0] == ["F1s", "F1s", "gather=same", "pairing=ok"]


def test_lone_rank_change(sim):
    # misuse: rank 1 alone changes its key at call 2.  It checks in the call and fails; ranks 0 and 2 kept
    # their key, defer their check and issue the frame's collectives (which rank 1 never joins), then fail
    # at call 3's deferred check.  Every rank issued call 2's gather (one collective sequence).
    rows = sim(3, False, ["a"] * 3, ["a"] * 3, ["a", "b", "a"], ["a", "b", "a"], ["a", "b", "a"])
    assert rows[2] == ["A", "F1k", "A", "gather=same", "pairing=ok"]
    # call 3: rank 1's communicator is poisoned, so it issues no all-gather that ranks 0 and 2's queued
    # frame collectives of call 2 could be paired with (round 5 issued one: undefined); 0 and 2 fail their
    # deferred check, and from then on every rank fails at once
    assert rows[3] == ["P1k", "X", "P1k", "gather=diverged", "pairing=ok"]
    assert rows[4] == ["X", "X", "X", "gather=diverged", "pairing=ok"]


def test_strict_mode_fails_every_rank_in_the_call(sim):
    rows = sim(3, True, ["a"] * 3, ["a"] * 3, ["a", "b", "a"])
    assert rows[0][:3] == rows[1][:3] == ["S"] * 3
    assert rows[2] == ["F1k"] * 3 + ["gather=same", "pairing=ok"]


@pytest.mark.parametrize("world", [2, 5, 8])
def test_every_rank_sees_the_same_verdict_when_it_checks(sim, world):
    # randomised sequences: whenever two ranks check the same call's words, their verdicts agree, and a
    # call in which every rank's key is new either succeeds on all ranks or fails on all ranks
    import random
    rng = random.Random(world)
    calls = []
    for _ in range(40):
        base = rng.choice("abc")
        calls.append([base if rng.random() < 0.9 else rng.choice("abcd") for _ in range(world)])
    rows = sim(world, False, *calls)
    for call, row in zip(calls, rows):
        checked = [t for t in row[:world] if t[0] in "SF"]
        assert len(set(checked)) <= 1
        assert row[-1] == "pairing=ok"  # never a collective paired with one of another kind

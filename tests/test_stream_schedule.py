"""The streaming kernel's LDS ring schedule is race-free for every wave timing (CPU model,
tools/stream_schedule.py).

The model restates the kernel's op sequence (LDS-DMA pieces, counted vmcnt waits, barriers, LDS
reads of K / V / Q, output stores) for the 4-wave form (4 slots, 2 tiles ahead, a barrier every
step) and the 8-wave form (8 slots, 4 tiles ahead, a barrier every second step) over item
sequences of 1-3 items per workgroup, and checks read-after-DMA (covered wait + barrier),
DMA-after-read (barrier) and the own-Q and zero-image rules. Each deliberately broken schedule
below must be flagged, so the checker is not vacuous."""
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sched():
    spec = importlib.util.spec_from_file_location("stream_schedule", os.path.join(REPO, "tools", "stream_schedule.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("nw", [4, 8])
def test_shipped_schedule_is_race_free(sched, nw):
    n, bad = sched.sweep(nws=(nw,), max_items=3, tiles=(2, 4, 6, 16, 34))
    assert n == 2 * (5 + 25 + 125)
    assert not bad, bad[:3]


def test_long_item_runs(sched):
    """Many items per workgroup (the 64-call launch: 8+ items of 16 tiles), both forms."""
    for nw in (4, 8):
        for seq in ([16] * 9, [2] * 7, [2, 16, 2, 34, 4, 2]):
            assert not sched.check(sched.kernel_ops(nw, seq, False), nw)


@pytest.mark.parametrize("mutation,nw", [
    ("lead+2", 4), ("lead+2", 8), ("odd_wait_loose", 8), ("every_4th_barrier", 8), ("no_prologue_barrier", 4),
    ("no_prologue_barrier", 8), ("no_two_tile_wait", 8), ("first_wait_loose", 8), ("nw4_wait_loose", 4)])
def test_broken_schedules_are_flagged(sched, mutation, nw):
    assert (mutation, nw) in sched.MUTATIONS
    _, bad = sched.sweep(nws=(nw,), max_items=2, tiles=(2, 4, 16), mutate=mutation)
    assert bad, mutation

"""Host logic of bench.py that needs no GPU: the untimed settle-step count."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_settle_steps_fill_the_warmup_to_settle_ms():
    # 5 warmup steps of 0.5 ms: 2.5 ms done, 27.5 ms more = 55 steps
    assert bench.settle_steps_needed(2.5e-3, 5, 30.0) == 55
    # a warmup that already lasted long enough adds nothing
    assert bench.settle_steps_needed(0.17, 2, 30.0) == 0
    # partial steps round up, so the warmup lasts at least settle_ms
    assert bench.settle_steps_needed(1.0e-3, 1, 2.5) == 2


def test_settle_steps_disabled_and_capped():
    assert bench.settle_steps_needed(1e-3, 3, 0.0) == 0
    assert bench.settle_steps_needed(1e-3, 0, 30.0) == 0
    # microsecond steps (C2 issued eagerly) stop at the cap
    assert bench.settle_steps_needed(3e-6, 3, 30.0) == 2000
    assert bench.settle_steps_needed(3e-6, 3, 30.0, cap=500) == 500

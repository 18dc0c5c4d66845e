"""Host logic of bench.py that needs no GPU: the untimed settle-step count, the pass kernel names."""
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


def test_stencil_kernel_names_follow_the_launch_rules():
    """The rocprof names the bench looks its pass up by: the 4096^2 x 2 pass (537 MB)
    streams its stores, a 10-deep pass of <= 192 MiB (C3's 1024^2 x 2) stores
    through the caches (vk_stencil_ps10.hip), variant 30 is the vector ring."""
    whole = 16 * 4096 * 4096 * 2
    assert bench.stencil_kernel_name(20, 10, 'fma', whole) == 'vk_ps::k_diffuse_ps<10, 4, 2, true>'
    assert bench.stencil_kernel_name(20, 10, 'fma', 16 * 1024 * 1024 * 2) == 'vk_ps::k_diffuse_ps<10, 4, 2, true, 2>'
    assert bench.stencil_kernel_name(20, 9, 'fma', 16 * 1024 * 1024 * 2) == 'vk_ps::k_diffuse_ps<9, 4, 2, true>'
    assert bench.stencil_kernel_name(30, 10, 'fma', whole) == 'vk_ps::k_diffuse_ps<10, 4, 2, true, 4>'
    assert bench.stencil_kernel_name(6, 9, 'exact') == 'vk_nt::k_diffuse_wl<9, 6, false>'
    assert bench.stencil_kernel_name(6, 10, 'exact') == 'vk_nt::k_diffuse_wl<10, 3, false>'

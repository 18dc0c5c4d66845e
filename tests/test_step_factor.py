"""The DP45 step factor en^-0.2 as every DP45 kernel computes it (round 6:
vk_kinetics.hip dp::step_pow, the specialised templates, vk_kremling.hip): a
single-precision estimate from the hardware log2 / exp2 (modelled here as the
float32 result perturbed by up to +-2.5e-7, more than the instructions'
error), then two Newton steps on en * y^5 = 1 in double, en clamped to
[1e-30, 1e30].  Within a few ulp of scipy's error_norm ** (-1/5) over the whole
range, and the clamp changes no factor (callers cap it at [0.2, 10])."""

import numpy as np


def step_pow(en, jitter=0.0, seed=1):
    e = np.clip(en, 1e-30, 1e30)
    yf = np.exp2(np.float32(-0.2) * np.log2(e.astype(np.float32))).astype(np.float32)
    if jitter:
        yf = yf * (1 + np.random.default_rng(seed).uniform(-jitter, jitter, yf.shape).astype(np.float32))
    y = yf.astype(np.float64)
    for _ in range(2):
        y2 = y * y
        r = 1.0 - e * (y2 * y2 * y)
        y = (0.2 * y) * r + y
    return y


def test_step_factor_within_a_few_ulp_of_pow():
    en = np.concatenate([np.logspace(-29.9, 29.9, 100001),
                         np.random.default_rng(0).uniform(1e-3, 10.0, 50000)])
    for jitter in (0.0, 2.5e-7):
        y = step_pow(en, jitter)
        assert np.abs(y / en ** -0.2 - 1).max() < 2e-15


def test_clamp_changes_no_capped_factor():
    small = np.logspace(-300, -30, 1000)        # accepted steps: min(10, 0.9 y) = 10 either way
    assert (np.minimum(10.0, 0.9 * step_pow(small)) == 10.0).all()
    large = np.logspace(30, 300, 1000)          # rejected steps: max(0.2, 0.9 y) = 0.2 either way
    assert (np.maximum(0.2, 0.9 * step_pow(large)) == 0.2).all()

"""Tolerance mode of the fused stencil passes (vk_set_stencil_mode(1)).

The default mode is bit-identical with the reference's
``f += coef * scipy.ndimage.convolve(f, LAP, mode='reflect')``
(vivarium/processes/diffusion_field.py:385-394; tests/test_gpu_parity.py).
The tolerance mode contracts each cell-substep into
``fma(coef/c4, (N+S)+(E+W), C)`` on a field carried rescaled by c4^-stage
(c4 = 1 - 4coef; ``fma(coef, (N+S)+(E+W), c4*C)`` when |c4| < 1e-3) and writes
the final pass without the delta-then-accumulate re-read.  Bar: within 1e-13 relative (of the plane's
largest value) of the scipy goldens and of the exact mode after whole steps,
at every tile geometry; uniform planes still skipped exactly.
"""

import os

import numpy as np
import pytest

from oracle import cpu

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
TOL = 1e-13


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


class _mode:
    def __init__(self, mode, depth=None, rows=None, variant=-1):
        self.mode, self.depth, self.rows, self.variant = mode, depth, rows, variant

    def __enter__(self):
        from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
        self.prev = stencil_mode(self.mode)
        self.prev_d = stencil_depth(self.depth) if self.depth else None
        self.prev_k = stencil_kernel(self.variant, self.rows or 0)

    def __exit__(self, *exc):
        from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
        stencil_mode(self.prev)
        if self.prev_d:
            stencil_depth(self.prev_d)
        stencil_kernel(self.prev_k, 0)


def _rel(got, ref):
    return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-300))


@pytest.mark.parametrize("variant", [20, 40])
@pytest.mark.parametrize('depth', [3, 5, 7, 9, 10, 11, 13])   # 13: no pair-sum pass, the exact wave tiles
def test_fma_mode_vs_scipy_goldens(dev, depth, variant):
    from lens_amd.lattice import Lattice
    z = np.load(os.path.join(GOLDEN, 'stencil.npz'))
    with _mode('fma', depth, 16, variant):
        for shape in ('17x23', '64x64', '128x96'):
            f0 = z['f0_' + shape]
            nx, ny = f0.shape
            for dt in (1.0, 5.0, 10.0):
                lat = Lattice(['a', 'b'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                              initial={'a': f0, 'b': np.full((nx, ny), 2.5)})
                lat.diffuse(dt)
                got = lat.owned('a').cpu().numpy()
                assert _rel(got, z['f_%s_dt%g' % (shape, dt)]) < TOL, (shape, dt)
                assert np.array_equal(lat.owned('b').cpu().numpy(), np.full((nx, ny), 2.5))


@pytest.mark.parametrize("variant", [20, 40])
@pytest.mark.parametrize('depth,rows', [(9, 64), (7, 40), (11, 48), (9, 17), (10, 34), (10, 17), (10, 64), (5, 8), (9, 8)])
@pytest.mark.parametrize('shape', [(700, 1000), (333, 517), (260, 1296)])
def test_fma_mode_large_tiles_vs_c_oracle(dev, depth, rows, shape, variant):
    from lens_amd.lattice import Lattice
    rng = np.random.default_rng(9)
    nx, ny = shape
    f0 = rng.random((nx, ny)) + 0.5
    with _mode('fma', depth, rows, variant):
        lat = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
        lat.diffuse(1.0)
        got = lat.owned('a').cpu().numpy()
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, 5.0 * 0.01, 100)
    assert _rel(got, ref) < TOL
    assert not np.array_equal(got, f0)


@pytest.mark.parametrize('rows', [64, 34, 17])
@pytest.mark.parametrize('shape', [(700, 1000), (333, 517), (260, 1296), (300, 96), (200, 97), (128, 200)])
def test_aligned_tiles_bitwise_vs_variant20(dev, shape, rows):
    """Variant 70 (the 10-deep pass with 16 halo columns, 96 written: every tile's
    rows whole 128-B lines) computes every cell as variant 20 does, bit for bit,
    whatever the tile grid; and within 1e-13 of the C oracle."""
    from lens_amd.lattice import Lattice
    rng = np.random.default_rng(13)
    nx, ny = shape
    f0 = rng.random((nx, ny)) + 0.5
    got = {}
    for variant in (70, 20):
        with _mode('fma', 10, rows, variant):
            lat = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
            lat.diffuse(1.0)
            got[variant] = lat.owned('a').cpu().numpy()
    assert np.array_equal(got[70], got[20])
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, 5.0 * 0.01, 100)
    assert _rel(got[70], ref) < TOL


def test_depth10_full_c4_planes_vs_depth9(dev):
    """The tolerance mode's 10-deep whole-step plan (10 passes per 100 substeps,
    three buffers) against the 9-deep plan on the full 4096^2 x 2 planes, three
    steps (1e-13), and a plane that is uniform stays bit for bit."""
    from lens_amd import configs
    from lens_amd.lattice import Lattice
    n = 4096
    glc = configs.gaussian_bump_field((n, n))
    out = {}
    for depth in (9, 10):
        with _mode('fma', depth, 34):
            lat = Lattice(['glc__D_e', 'ac_e'], (n, n), (float(n), float(n)), 10.0, 5.0, device=dev,
                          initial={'glc__D_e': glc, 'ac_e': np.full((n, n), 0.25)})
            for _ in range(3):
                lat.diffuse(1.0)
            torch.cuda.synchronize()
            out[depth] = lat
    a, b = out[9].fields[0], out[10].fields[0]
    assert float((a - b).abs().max() / a.abs().max()) < TOL
    assert torch.equal(out[10].fields[1], torch.full_like(out[10].fields[1], 0.25))


def test_fma_mode_full_c4_planes_vs_exact_mode(dev):
    """4096^2 x 2 fields (C4), three steps: the tolerance mode against the
    bit-exact mode, plane by plane, and the switch back restores exactness."""
    from lens_amd import configs
    from lens_amd.lattice import Lattice
    n = 4096
    glc = configs.gaussian_bump_field((n, n))
    ac = np.random.default_rng(2).random((n, n)) * 1e-3
    lats = {}
    for mode in ('exact', 'fma'):
        with _mode(mode):
            lat = Lattice(['glc__D_e', 'ac_e'], (n, n), (float(n), float(n)), 10.0, 5.0, device=dev,
                          initial={'glc__D_e': glc, 'ac_e': ac})
            for _ in range(3):
                lat.diffuse(1.0)
            torch.cuda.synchronize()
            lats[mode] = lat
    for f in range(2):
        a = lats['exact'].fields[f]
        b = lats['fma'].fields[f]
        rel = float((a - b).abs().max() / a.abs().max())
        assert rel < TOL, (f, rel)
        assert not torch.equal(a, b)        # the modes do differ (in the last bits)


@pytest.mark.parametrize('depth,n_sub', [(10, 20), (9, 18)])
@pytest.mark.parametrize('coef', [0.05, 0.2497, 0.2498, 0.25])
def test_fma_mode_scaled_and_unscaled_forms_vs_c_oracle(dev, depth, n_sub, coef):
    """The tolerance mode carries the field rescaled by c4^-stage (c4 = 1 - 4coef)
    while |c4| >= 1e-3 and keeps the unscaled fma form nearer coef = 1/4: both
    sides of that cut (0.2497 scaled, 0.2498 and 0.25 unscaled) on a ragged
    plane with edge tiles, against the C oracle (1e-13)."""
    from lens_amd import native
    rng = np.random.default_rng(11)
    nx, ny = 333, 517
    f0 = rng.random((nx, ny)) + 0.5
    with _mode('fma', depth, 17):
        field = torch.tensor(f0, device=dev)
        w0, w1 = torch.empty_like(field), torch.empty_like(field)
        native.check(native._lib.vk_diffuse(
            native.ptr(field), native.ptr(w0), native.ptr(w1), 1, nx * ny, ny, 0, nx, 0, nx, 1, 1,
            0, n_sub, n_sub, coef, 0, native.stream_handle()), 'diffuse')
        got = field.cpu().numpy()
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, coef, n_sub)
    assert _rel(got, ref) < TOL, _rel(got, ref)
    assert not np.array_equal(got, f0)


def test_fma_mode_zero_coefficient_is_identity(dev):
    """coef = 0 (no diffusion): the scaled form is t + 0 * sum with c4^K = 1, so
    the field comes back bit for bit."""
    from lens_amd import native
    rng = np.random.default_rng(12)
    nx, ny = 300, 237
    f0 = rng.random((nx, ny)) * 5
    with _mode('fma', 10, 17):
        field = torch.tensor(f0, device=dev)
        w0, w1 = torch.empty_like(field), torch.empty_like(field)
        native.check(native._lib.vk_diffuse(
            native.ptr(field), native.ptr(w0), native.ptr(w1), 1, nx * ny, ny, 0, nx, 0, nx, 1, 1,
            0, 20, 20, 0.0, 0, native.stream_handle()), 'diffuse')
        assert np.array_equal(field.cpu().numpy(), f0)

"""The 10-deep pair-sum pass with the vertical stash (variants 60-62,
lens_amd/csrc/vk_stencil_ps.h PsStash): a workgroup's four waves take four
vertically adjacent 64-row chunks of one column tile, and each boundary's input
rows are read from HBM once and handed to the wave above through LDS.

Only where the rows come from changes, so every plane is bit for bit the
variant-20 pass's (tolerance mode, vivarium/processes/diffusion_field.py:385-394),
and within 1e-13 of the C oracle.  A launch whose rows are not whole 64-row
chunks falls back to variant 20.
"""

import numpy as np
import pytest

from oracle import cpu

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu
TOL = 1e-13


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


def _diffuse(dev, f0, variant, steps=1, rows=64, extra=None):
    from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel, stencil_mode
    nx, ny = f0.shape
    prev_m, prev_d = stencil_mode('fma'), stencil_depth(10)
    prev_k = stencil_kernel(variant, rows)
    try:
        init = {'a': f0}
        names = ['a']
        if extra is not None:
            init['b'] = extra
            names.append('b')
        lat = Lattice(names, (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial=init)
        for _ in range(steps):
            lat.diffuse(1.0)
        torch.cuda.synchronize()
        return [lat.owned(n).cpu().numpy() for n in names]
    finally:
        stencil_mode(prev_m)
        stencil_depth(prev_d)
        stencil_kernel(prev_k, 0)


def _rel(got, ref):
    return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-300))


# rows: 640 = 10 chunks (the last group holds 2), 256 = one group whose top and
# bottom chunks both see a reflected row, 64 = one chunk (no boundary), 1088 = 17
# chunks (a group of one); columns: ragged and 16-B-aligned widths, 1 to 12 tiles
@pytest.mark.parametrize('variant', [60, 61, 62])
@pytest.mark.parametrize('shape', [(640, 1000), (256, 517), (64, 300), (1088, 1296), (320, 108)])
def test_stash_pass_bitwise_vs_variant20_and_c_oracle(dev, variant, shape):
    rng = np.random.default_rng(21)
    f0 = rng.random(shape) + 0.5
    got = _diffuse(dev, f0, variant)[0]
    ref20 = _diffuse(dev, f0, 20)[0]
    assert np.array_equal(got, ref20)
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, 5.0 * 0.01, 100)
    assert _rel(got, ref) < TOL
    assert not np.array_equal(got, f0)


def test_stash_pass_falls_back_off_whole_chunks(dev):
    """700 rows are not whole 64-row chunks: the launch is variant 20's."""
    rng = np.random.default_rng(22)
    f0 = rng.random((700, 517)) + 0.5
    assert np.array_equal(_diffuse(dev, f0, 60)[0], _diffuse(dev, f0, 20)[0])


def test_stash_pass_full_c4_planes_three_steps(dev):
    """The bench's planes (4096^2 x 2, a Gaussian bump and a random plane), three
    whole steps: bit for bit variant 20."""
    from lens_amd import configs
    n = 4096
    glc = configs.gaussian_bump_field((n, n))
    ac = np.random.default_rng(2).random((n, n)) * 1e-3
    a = _diffuse(dev, glc, 60, steps=3, extra=ac)
    b = _diffuse(dev, glc, 20, steps=3, extra=ac)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_stash_pass_uniform_plane_and_unscaled_form(dev):
    """A uniform plane keeps its bits (the whole workgroup skips it); coef near 1/4
    takes the unscaled fma form, also through the stash."""
    from lens_amd import native
    from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
    rng = np.random.default_rng(23)
    f0 = rng.random((640, 517)) + 0.5
    a, b = _diffuse(dev, f0, 60, extra=np.full((640, 517), 2.5))
    assert np.array_equal(b, np.full((640, 517), 2.5))
    nx, ny = 640, 517
    out = {}
    for variant in (60, 20):
        prev_m, prev_d, prev_k = stencil_mode('fma'), stencil_depth(10), stencil_kernel(variant, 64)
        try:
            field = torch.tensor(f0, device=dev)
            w0, w1 = torch.empty_like(field), torch.empty_like(field)
            native.check(native._lib.vk_diffuse(
                native.ptr(field), native.ptr(w0), native.ptr(w1), 1, nx * ny, ny, 0, nx, 0, nx, 1, 1,
                0, 20, 20, 0.2499, 0, native.stream_handle()), 'diffuse')
            out[variant] = field.cpu().numpy()
        finally:
            stencil_mode(prev_m)
            stencil_depth(prev_d)
            stencil_kernel(prev_k, 0)
    assert np.array_equal(out[60], out[20])
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, 0.2499, 20)
    assert _rel(out[60], ref) < TOL

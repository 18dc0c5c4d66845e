"""Stage-split pair-sum passes (variant 40, vk_stencil_sp.h) against the
single-wave pair-sum passes (variant 20, vk_stencil_ps.h).

A split pass spreads the K stages of one tile over the waves of a workgroup
and hands rows between them through LDS; every cell still goes through the
same ps_stage arithmetic on the same operands.  Bar: BIT-identical with
variant 20 (itself within 1e-13 of scipy's convolve and of the exact mode,
tests/test_stencil_modes.py) -- every tile geometry, ragged planes, reflecting
edges, chunk heights that do not divide the plane, uniform planes (skipped),
the unscaled coefficient form (coef ~ 1/4), row bands, and the full C4 planes.
The reference update: vivarium/processes/diffusion_field.py:385-394.
"""

import numpy as np
import pytest

from oracle import cpu

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu
SPLIT = (40,)


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


class _kernel:
    def __init__(self, variant, rows, depth=10, mode='fma'):
        self.variant, self.rows, self.depth, self.mode = variant, rows, depth, mode

    def __enter__(self):
        from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
        self.prev = (stencil_mode(self.mode), stencil_depth(self.depth), stencil_kernel(self.variant, self.rows))

    def __exit__(self, *exc):
        from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
        stencil_mode(self.prev[0])
        stencil_depth(self.prev[1])
        stencil_kernel(self.prev[2], 0)


def _run(dev, variant, rows, f0, diffusion=5.0, steps=1, second=None):
    from lens_amd.lattice import Lattice
    nx, ny = f0.shape
    init = {'a': f0}
    mols = ['a']
    if second is not None:
        init['b'] = second
        mols.append('b')
    with _kernel(variant, rows):
        lat = Lattice(mols, (nx, ny), (float(nx), float(ny)), 10.0, diffusion, device=dev, initial=init)
        for _ in range(steps):
            lat.diffuse(1.0)
        torch.cuda.synchronize()
    return lat


@pytest.mark.parametrize('variant', SPLIT)
@pytest.mark.parametrize('rows', [0, 8, 33, 128, 300])    # 0: whole rounds of workgroups (auto)
@pytest.mark.parametrize('shape', [(700, 1000), (333, 517), (260, 1296), (17, 23), (64, 64), (40, 700), (129, 233)])
def test_split_pass_equals_pair_sum_bitwise(dev, variant, rows, shape):
    rng = np.random.default_rng(hash((variant, rows) + shape) % 2**32)
    f0 = rng.random(shape) + 0.5
    uni = np.full(shape, 0.75)
    ref = _run(dev, 20, 34, f0, second=uni, steps=2)
    got = _run(dev, variant, rows, f0, second=uni, steps=2)
    a, b = got.owned().cpu().numpy(), ref.owned().cpu().numpy()
    assert np.array_equal(a[0], b[0]), (variant, rows, shape, float(np.abs(a[0] - b[0]).max()))
    assert np.array_equal(a[1], uni)                 # a uniform plane is skipped exactly
    assert not np.array_equal(a[0], f0)


@pytest.mark.parametrize('variant', SPLIT)
@pytest.mark.parametrize('diffusion', [24.98, 25.0, 0.0, 12.5])
def test_split_pass_coefficient_forms(dev, variant, diffusion):
    """coef = diffusion * 0.01 on unit bins: 0.2498 / 0.25 take the unscaled form
    (|1 - 4 coef| < 1e-3), 0 is the identity, 0.125 the rescaled form."""
    rng = np.random.default_rng(3)
    f0 = rng.random((150, 301)) * 3
    ref = _run(dev, 20, 34, f0, diffusion=diffusion)
    got = _run(dev, variant, 64, f0, diffusion=diffusion)
    assert torch.equal(got.fields, ref.fields), variant
    if diffusion == 0.0:
        assert np.array_equal(got.owned('a').cpu().numpy(), f0)


@pytest.mark.parametrize('variant', SPLIT)
def test_split_pass_vs_c_oracle(dev, variant):
    """Independent of variant 20: the C oracle's exact-order stencil, 1e-13."""
    rng = np.random.default_rng(11)
    f0 = rng.random((333, 517)) + 0.5
    got = _run(dev, variant, 96, f0).owned('a').cpu().numpy()
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, 5.0 * 0.01, 100)
    assert float(np.abs(got - ref).max() / np.abs(ref).max()) < 1e-13


@pytest.mark.parametrize('variant', SPLIT)
def test_split_pass_row_bands_equal_whole_plane(dev, variant):
    """Row bands with one 100-deep halo block per step (the C4 bench at N > 1),
    stepped with the split passes, equal the whole plane bit for bit."""
    from lens_amd import native
    from lens_amd.distributed import row_bands
    from lens_amd.lattice import Lattice
    rng = np.random.default_rng(4)
    nx, ny = 300, 237
    f0 = rng.random((nx, ny)) * 5
    whole = _run(dev, 20, 34, f0)
    with _kernel(variant, 48):
        for world in (2, 3):
            lats = [Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                            row_band=b, halo=100, initial={'a': f0}) for b in row_bands(nx, world)]
            for r, lat in enumerate(lats):
                if not lat.edge_top:
                    nb = lats[r - 1]
                    lat.fields[:, lat.row_lo - 100:lat.row_lo].copy_(nb.fields[:, nb.row_hi - 100:nb.row_hi])
                if not lat.edge_bot:
                    nb = lats[r + 1]
                    lat.fields[:, lat.row_hi:lat.row_hi + 100].copy_(nb.fields[:, nb.row_lo:nb.row_lo + 100])
            for lat in lats:
                lo_min = lat.row_lo if lat.edge_top else 0
                hi_max = lat.row_hi if lat.edge_bot else lat.rows_local
                native.check(native._lib.vk_diffuse(
                    native.ptr(lat.fields), native.ptr(lat.work0), native.ptr(lat.work1), 1,
                    lat.field_stride, ny, lat.row_lo, lat.row_hi, lo_min, hi_max, int(lat.edge_top),
                    int(lat.edge_bot), 0, 100, 100, lat.diffusion * 0.01, 0, native.stream_handle()), 'diffuse')
            got = torch.cat([lat.owned('a') for lat in lats], 0).cpu().numpy()
            assert np.array_equal(got, whole.owned('a').cpu().numpy()), world


def test_split_pass_full_c4_planes(dev):
    """The bench's planes: 4096^2 x 2 (gaussian bump + zeros that fill in), two
    steps, variant 40 at its default chunk height against variant 20 at 34 rows."""
    from lens_amd import configs
    n = 4096
    glc = configs.gaussian_bump_field((n, n))
    ac = np.random.default_rng(2).random((n, n)) * 1e-3
    ref = _run(dev, 20, 34, glc, second=ac, steps=2)
    got = _run(dev, 40, 0, glc, second=ac, steps=2)
    assert torch.equal(got.fields, ref.fields)


@pytest.mark.parametrize('passes', [1, 3, 10])
@pytest.mark.parametrize('mode,variant', [('fma', 20), ('fma', 40), ('exact', 20)])
@pytest.mark.parametrize('world,halo', [(2, 100), (3, 100), (3, 50)])
def test_band_interior_then_edges_equals_whole_plane(dev, mode, variant, world, halo, passes):
    """vk_diffuse_part: a band's first block as the interior of its first
    `passes` passes (no halo needed: they run while the halo exchange is in
    flight), then their edges and the other passes whole, equals the whole plane
    bit for bit -- both arithmetic modes, the pair-sum and the stage-split
    kernels, one and two halo blocks per step."""
    from lens_amd import native
    from lens_amd.distributed import row_bands
    from lens_amd.lattice import Lattice, n_substeps
    rng = np.random.default_rng(7)
    nx, ny = 700, 203
    f0 = rng.random((nx, ny)) * 5
    g0 = np.full((nx, ny), 1.25)                    # a uniform plane: skipped in every part
    with _kernel(variant, 0, mode=mode):
        whole = Lattice(['a', 'b'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                        initial={'a': f0, 'b': g0})
        whole.diffuse(1.0)
        lats = [Lattice(['a', 'b'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, row_band=b,
                        halo=halo, initial={'a': f0, 'b': g0}) for b in row_bands(nx, world)]
        n_sub = n_substeps(1.0)
        mms = []
        for lat in lats:
            mms.append(lat.uniform_summary(None).clone())
        split = 0
        j = 0
        while j < n_sub:
            cnt = min(halo, n_sub - j)
            bufs = [lat.state_buffer(j) for lat in lats]
            for r, lat in enumerate(lats):          # the halo exchange before the block
                if not lat.edge_top:
                    nb, src = lats[r - 1], bufs[r - 1]
                    bufs[r][:, lat.row_lo - halo:lat.row_lo].copy_(src[:, nb.row_hi - halo:nb.row_hi])
                if not lat.edge_bot:
                    nb, src = lats[r + 1], bufs[r + 1]
                    bufs[r][:, lat.row_hi:lat.row_hi + halo].copy_(src[:, nb.row_lo:nb.row_lo + halo])
            for lat, mm in zip(lats, mms):
                lo_min = lat.row_lo if lat.edge_top else 0
                hi_max = lat.row_hi if lat.edge_bot else lat.rows_local
                coef = lat.diffusion * 0.01
                if j == 0 and lat._run_part(j, cnt, n_sub, coef, mm, lo_min, hi_max, native.VK_PART_INTERIOR,
                                            passes):
                    split += 1
                    assert lat._run_part(j, cnt, n_sub, coef, mm, lo_min, hi_max, native.VK_PART_EDGES, passes)
                else:
                    lat._run_block(j, cnt, n_sub, coef, mm, lo_min, hi_max)
            j += cnt
        torch.cuda.synchronize()
    assert split == world                           # every band's first block split
    got = torch.cat([lat.owned() for lat in lats], 1).cpu().numpy()
    assert np.array_equal(got, whole.owned().cpu().numpy()), (world, halo)


def test_part_refuses_blocks_it_cannot_split(dev):
    """The whole plane (no halo rows) and the odd-depth plan do not split:
    VK_ERR_LIMIT, nothing launched, the field unchanged."""
    from lens_amd import native
    from lens_amd.lattice import Lattice
    f0 = np.random.default_rng(1).random((64, 64))
    with _kernel(20, 0):
        lat = Lattice(['a'], (64, 64), (64.0, 64.0), 10.0, 5.0, device=dev, initial={'a': f0})
        mm = lat.uniform_summary(None)
        assert not lat._run_part(0, 100, 100, 0.05, mm, 0, 64, native.VK_PART_INTERIOR)
    torch.cuda.synchronize()
    assert np.array_equal(lat.owned('a').cpu().numpy(), f0)

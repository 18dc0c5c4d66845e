"""The coupled passes (vk_diffuse_coupled, Colony._coupled_step): the gather
riding on the first diffusion pass and the exchange on the final one must give
exactly what the three separate launches give (vk_gather, the passes,
vk_exchange_sorted) -- fields, external concentrations and every agent array
bit for bit, step after step.  Covered: 10-deep and odd-depth plans, the
vector-ring variant, ragged planes (width not a multiple of 16 or
of a tile), a plane narrower than one tile, several chunks per tile column,
bins crowded past one load batch, uniform planes (the acetate plane starts at
zero), both arithmetic modes (pair-sum and variant-6 / plain-store wave tiles),
graph replay, and the fallbacks (single-substep passes, agents out of bin order).
"""

import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


class _stencil:
    def __init__(self, mode, depth, kernel, rows):
        self.want = (mode, depth, kernel, rows)

    def __enter__(self):
        from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
        mode, depth, kernel, rows = self.want
        self.prev = (stencil_mode(mode), stencil_depth(depth), stencil_kernel(kernel, rows))

    def __exit__(self, *exc):
        from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
        mode, depth, kernel = self.prev
        stencil_mode(mode)
        stencil_depth(depth)
        stencil_kernel(kernel, 0)


def _pair(dev, nx, ny, n, crowd=0, seed=3, integrator='euler'):
    """Two identical sorted lattice colonies (glc_ac kinetics), one stepping
    through the coupled passes and one through the separate launches."""
    from lens_amd import configs
    from lens_amd.colony import Colony
    from lens_amd.lattice import Lattice
    from lens_amd.rate_law_compiler import compile_rate_laws
    cfg = configs.glc_ac_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    rng = np.random.default_rng(seed)
    bounds = (float(nx), float(ny))
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=seed)
    loc = np.stack([rng.uniform(0, bounds[0], n), rng.uniform(0, bounds[1], n)])
    if crowd:
        # `crowd` agents in three neighbouring bins of one row (runs longer than a
        # load batch, crossing batch boundaries), the rest spread out
        k = np.arange(crowd)
        loc[0, :crowd] = 0.5 + nx // 2
        loc[1, :crowd] = 0.5 + (k % 3) + 17
    glc = configs.gaussian_bump_field((nx, ny))
    out = []
    for fused in (True, False):
        lat = Lattice(['glc__D_e', 'ac_e'], (nx, ny), bounds, 10.0, 5.0, device=dev,
                      initial={'glc__D_e': glc, 'ac_e': np.zeros((nx, ny))})
        col = Colony(cfg, n, device=dev, integrator=integrator, environment=lat, table=t)
        col.set_agents(params=params, conc=conc, location=loc)
        col.gather_external()
        col.sort_by_bin()
        col.fuse_coupling = fused
        out.append((col, lat))
    return out


def _same(a, b, where):
    (ca, la), (cb, lb) = a, b
    n = ca.n
    for m in la.molecules:
        assert torch.equal(la.owned(m), lb.owned(m)), (where, m)
    for name in ('conc', 'flux', 'counts'):
        assert torch.equal(getattr(ca, name)[:, :n], getattr(cb, name)[:, :n]), (where, name)


CASES = {
    # name: (nx, ny, agents, crowd, mode, depth, kernel, rows)
    'd10_ragged': (40, 300, 3000, 0, 'fma', 10, 20, 8),
    'd9_odd_plan': (40, 300, 3000, 0, 'fma', 9, 20, 8),
    'd10_split_selected': (40, 300, 3000, 0, 'fma', 10, 40, 8),   # coupled passes run variant 20
    'd10_crowded': (33, 260, 2500, 90, 'fma', 10, 20, 12),
    'd10_narrow': (30, 50, 800, 40, 'fma', 10, 20, 0),
    'd7_tall_tiles': (70, 230, 4000, 0, 'fma', 7, 20, 64),
    'exact_d9': (40, 300, 3000, 0, 'exact', 9, 6, 8),
    'exact_d5_plain_stores': (33, 260, 2500, 90, 'exact', 5, 2, 12),
    'exact_d10_setting': (40, 300, 3000, 0, 'exact', 10, 20, 0),
}


@pytest.mark.parametrize('case', sorted(CASES))
def test_coupled_passes_equal_separate_launches(dev, case):
    nx, ny, n, crowd, mode, depth, kernel, rows = CASES[case]
    with _stencil(mode, depth, kernel, rows):
        a, b = _pair(dev, nx, ny, n, crowd)
        assert a[0]._couple is not None and a[1].coupled_plan_ok(1.0)
        for step in range(3):
            a[0].step(1.0)
            b[0].step(1.0)
            assert a[0].last_step_coupled and not b[0].last_step_coupled
            torch.cuda.synchronize()
            _same(a, b, (case, step))
        # the acetate plane was uniform (zero) before the first exchange: it must
        # have received the exchange without being diffused in that step
        assert float(a[1].owned('ac_e').abs().max()) > 0


def test_coupled_dopri5_graph_replay_equals_separate_launches(dev):
    with _stencil('fma', 10, 20, 8):
        a, b = _pair(dev, 40, 300, 3000, 30, integrator='dopri5')
        replay = a[0].capture(1.0, 3)
        replay()
        for _ in range(3):
            b[0].step(1.0)
        torch.cuda.synchronize()
        _same(a, b, 'graph')


def test_coupled_declined_single_substep_passes_and_unsorted(dev):
    """One launch per substep (depth 1) keeps the separate launches (a
    single-substep pass carries no coupling); agents that moved out of bin
    order drop the index until they are sorted again."""
    with _stencil('exact', 1, 6, 8):
        a, b = _pair(dev, 40, 300, 3000)
        assert not a[1].coupled_plan_ok(1.0)
        a[0].step(1.0)
        b[0].step(1.0)
        assert not a[0].last_step_coupled
        torch.cuda.synchronize()
        _same(a, b, 'depth 1')
    with _stencil('fma', 10, 20, 8):
        col, lat = a
        rng = np.random.default_rng(9)
        loc = np.stack([rng.uniform(0, 40.0, col.n), rng.uniform(0, 300.0, col.n)])
        col.set_agents(location=loc)                 # moved: no longer in bin order
        assert col._couple is None
        col.step(1.0)
        assert not col.last_step_coupled
        col.sort_by_bin()
        assert col._couple is not None and col.fuse_coupling
        col.step(1.0)
        assert col.last_step_coupled


def test_c4_coupled_step_equals_separate_launches(dev):
    """The bench's C4 colony (1M agents, 4096^2 x 2, bin order, the bench's
    stencil settings): one step through the coupled passes equals one through
    the separate launches, bit for bit."""
    import types
    import bench
    args = types.SimpleNamespace(workload='c4', integrator='euler', halo=0, exchange='sorted',
                                 generic_kernel=False, agents=None, overlap_kinetics=False, sort_agents=True)
    from test_configs import _bench_stencil
    with _bench_stencil():
        a = bench.build_rank(args, 0, 1, dev)[:2]
        assert a[0]._couple is not None
        a[0].fuse_coupling = True
        a[0].step(1.0)
        assert a[0].last_step_coupled
        torch.cuda.synchronize()
        fa = [a[1].owned(m).clone() for m in a[1].molecules]
        ca = a[0].conc[:, :a[0].n].clone()
        del a
        b = bench.build_rank(args, 0, 1, dev)[:2]
        b[0].fuse_coupling = False
        b[0].step(1.0)
        torch.cuda.synchronize()
        for f, m in zip(fa, b[1].molecules):
            assert torch.equal(f, b[1].owned(m)), m
        assert torch.equal(ca, b[0].conc[:, :b[0].n])

"""The exchange added inside the final diffusion pass (vk_diffuse_exchange,
Colony.exchange_in_pass; lens_amd/csrc/vk_stencil_ps.h ex_stage / ex_apply):
each wave stages its cells' agents in LDS and adds their counts / bva * 1000 to
a row, in agent order, before storing it.  The new planes, external
concentrations and agent arrays must equal the separate launches (the passes,
then vk_exchange_sorted: update_field_with_exchange, registry.py:149-183,
applied agent by agent) bit for bit, step after step.

Covered: ragged and narrow planes, chunk heights 8 / 17 / 64, bins crowded past
a load batch, a wave whose cells hold more agents than its LDS slots (the
post-store fallback), uniform planes (the acetate plane starts at zero), DP45
and Euler, graph replay, the bench's C4 colony at full size, and the guards
(variant 20 keeps the separate sweep; the exact mode; agents out of bin order).
"""

import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_coupled_gpu import _same, _stencil  # noqa: E402


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


def _pair(dev, nx, ny, n, crowd=0, seed=5, integrator='euler', crowd_cells=3):
    """Two identical sorted lattice colonies (glc_ac kinetics): the first adds the
    exchange in the final pass, the second runs the separate sweep."""
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
        # `crowd` agents in `crowd_cells` neighbouring bins of one row
        k = np.arange(crowd)
        loc[0, :crowd] = 0.5 + nx // 2
        loc[1, :crowd] = 0.5 + (k % crowd_cells) + 17
    glc = configs.gaussian_bump_field((nx, ny))
    out = []
    for inpass in (True, False):
        lat = Lattice(['glc__D_e', 'ac_e'], (nx, ny), bounds, 10.0, 5.0, device=dev,
                      initial={'glc__D_e': glc, 'ac_e': np.zeros((nx, ny))})
        col = Colony(cfg, n, device=dev, integrator=integrator, environment=lat, table=t)
        col.set_agents(params=params, conc=conc, location=loc)
        col.gather_external()
        col.sort_by_bin()
        col.exchange_in_pass = inpass
        out.append((col, lat))
    return out


CASES = {
    # name: (nx, ny, agents, crowd, crowd_cells, rows)
    'ragged_rows8': (40, 300, 3000, 0, 3, 8),
    'ragged_rows17': (70, 230, 4000, 0, 3, 17),
    'tall_rows64': (200, 390, 12000, 0, 3, 64),
    'crowded': (33, 260, 2500, 90, 3, 12),
    'narrow': (30, 50, 800, 40, 3, 0),
    'over_capacity': (128, 300, 3000, 1500, 40, 64),   # one region's cells hold too many agents: post-store path
    'crowded_rows64': (128, 300, 3000, 24, 16, 64),     # up to 4 agents a lane in the image path
    'edge_tiles_rows64': (192, 290, 5000, 0, 3, 64),    # a partial last tile (290 = 3 x 96 + 2)
}


@pytest.mark.parametrize('case', sorted(CASES))
def test_exchange_in_pass_equals_separate_sweep(dev, case):
    nx, ny, n, crowd, cells, rows = CASES[case]
    with _stencil('fma', 10, 70, rows):
        a, b = _pair(dev, nx, ny, n, crowd, crowd_cells=cells)
        assert a[0]._exchange_in_pass_ok(1.0) and not b[0]._exchange_in_pass_ok(1.0)
        for step in range(3):
            a[0].step(1.0)
            b[0].step(1.0)
            torch.cuda.synchronize()
            _same(a, b, (case, step))
        # the acetate plane was uniform (zero) before the first exchange: it must
        # have received the exchange without being diffused in that step
        assert float(a[1].owned('ac_e').abs().max()) > 0


def test_exchange_in_pass_dopri5_graph_replay(dev):
    with _stencil('fma', 10, 70, 17):
        a, b = _pair(dev, 70, 230, 4000, 30, integrator='dopri5')
        replay = a[0].capture(1.0, 3)
        replay()
        for _ in range(3):
            b[0].step(1.0)
        torch.cuda.synchronize()
        _same(a, b, 'graph')


def test_exchange_in_pass_guards(dev):
    """Variant 20 and the exact mode have no store path: the colony keeps the
    separate sweep; agents out of bin order drop the index until sorted again."""
    for want in (('fma', 10, 20, 8), ('exact', 10, 20, 0)):
        with _stencil(*want):
            a, b = _pair(dev, 40, 300, 3000)
            assert not a[0]._exchange_in_pass_ok(1.0)
            a[0].step(1.0)
            b[0].step(1.0)
            torch.cuda.synchronize()
            _same(a, b, want)
    with _stencil('fma', 10, 70, 8):
        col, lat = a
        rng = np.random.default_rng(9)
        col.set_agents(location=np.stack([rng.uniform(0, 40.0, col.n), rng.uniform(0, 300.0, col.n)]))
        assert not col._exchange_in_pass_ok(1.0)
        col.step(1.0)
        col.sort_by_bin()
        assert col._exchange_in_pass_ok(1.0)


def test_c4_exchange_in_pass_equals_separate_sweep(dev):
    """The bench's C4 colony (1M agents, 4096^2 x 2, bin order, the bench's
    stencil settings, DP45 with the fused gather): one step with the exchange in
    the final pass equals one with the separate sweep, bit for bit."""
    import types
    import bench
    args = types.SimpleNamespace(workload='c4', integrator='dopri5', halo=0, exchange='sorted',
                                 generic_kernel=False, agents=None, overlap_kinetics=False, sort_agents=True)
    from test_configs import _bench_stencil
    with _bench_stencil():
        a = bench.build_rank(args, 0, 1, dev)[:2]
        assert a[0]._exchange_in_pass_ok(1.0)
        # the bench's wave regions take the image path: only regions with a lane owning
        # four agents of a row fall back (about one in 40 at this density)
        img = a[0]._ex_image
        assert (img.tiles, img.rows) == (43, 64) and int(img.xbad.sum()) <= 0.05 * img.xbad.numel()
        a[0].step(1.0)
        torch.cuda.synchronize()
        fa = [a[1].owned(m).clone() for m in a[1].molecules]
        ca = a[0].conc[:, :a[0].n].clone()
        del a
        b = bench.build_rank(args, 0, 1, dev)[:2]
        b[0].exchange_in_pass = False
        b[0].step(1.0)
        torch.cuda.synchronize()
        for f, m in zip(fa, b[1].molecules):
            assert torch.equal(f, b[1].owned(m)), m
        assert torch.equal(ca, b[0].conc[:, :b[0].n])

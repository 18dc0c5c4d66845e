"""HIP-graph replay of a colony step (Colony.capture) against eager stepping (needs an MI355X)."""

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from lens_amd import configs  # noqa: E402
from lens_amd.rate_law_compiler import compile_rate_laws  # noqa: E402


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


def _colony(dev, n=5000, specialize=False):
    from lens_amd.colony import Colony
    cfg = configs.glc_lct_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    params, conc = configs.heterogeneous_colony(t, cfg, n)
    col = Colony(cfg, n, device=dev, integrator='dopri5', table=t, specialize=specialize)
    col.set_agents(params=params, conc=conc)
    col.count_attempts(True)
    return col


def _state(col):
    n = col.n
    return {k: v[..., :n].cpu().numpy().copy() for k, v in
            (('conc', col.conc), ('h', col.h_state), ('flux', col.flux), ('counts', col.counts),
             ('nsteps', col.nsteps), ('attempts', col.attempts.reshape(1)))}


@pytest.mark.parametrize('per_graph', [1, 4])
def test_graph_replay_equals_eager_steps(dev, per_graph):
    """C2-style colony (held externals, DP45): 8 steps replayed from a graph of
    `per_graph` steps give the eager steps' state bit for bit, and the replayer
    advances the colony clock."""
    eager, graphed = _colony(dev), _colony(dev)
    eager.step(1.0)                 # first use of the kernels in both colonies
    graphed.step(1.0)
    for _ in range(8):
        eager.step(1.0)
    before = _state(graphed)
    replay = graphed.capture(1.0, per_graph)
    torch.cuda.synchronize()
    assert np.array_equal(_state(graphed)['conc'], before['conc'])   # capture runs nothing
    for _ in range(8 // per_graph):
        replay()
    torch.cuda.synchronize()
    eager.check_status()
    graphed.check_status()
    a, b = _state(eager), _state(graphed)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert graphed.step_index == eager.step_index and graphed.time == eager.time


def test_capture_refuses_host_decided_steps(dev):
    """A lattice or division colony takes host decisions per step: capture refuses it."""
    from lens_amd.colony import Colony
    cfg = configs.glc_lct_config()
    col = Colony(cfg, 4, device=dev, integrator='euler', environment='nonspatial')
    with pytest.raises(ValueError):
        col.capture(1.0, 1)


def _lattice_colony(dev, n=3000, nx=200):
    from lens_amd.colony import Colony
    from lens_amd.lattice import Lattice
    cfg = configs.glc_ac_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    rng = np.random.default_rng(5)
    lat = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (float(nx), float(nx)), 10.0, 5.0, device=dev,
                  initial={'glc__D_e': configs.gaussian_bump_field((nx, nx)), 'ac_e': np.zeros((nx, nx))})
    params, conc = configs.heterogeneous_colony(t, cfg, n)
    col = Colony(cfg, n, device=dev, integrator='dopri5', environment=lat, table=t, specialize=True)
    col.set_agents(params=params, conc=conc, location=rng.uniform(0.0, float(nx), (2, n)))
    col.gather_external()
    return col


def test_graph_replay_lattice_colony(dev):
    """C3-style single-GPU lattice colony (kinetics, gather, 100 diffusion
    substeps with the uniform-plane skip on the still-uniform acetate plane,
    sorted exchange): 6 replayed steps equal 6 eager steps bit for bit."""
    eager, graphed = _lattice_colony(dev), _lattice_colony(dev)
    eager.step(1.0)
    graphed.step(1.0)
    for _ in range(6):
        eager.step(1.0)
    replay = graphed.capture(1.0, 3)
    replay()
    replay()
    torch.cuda.synchronize()
    eager.check_status()
    graphed.check_status()
    n = eager.n
    assert np.array_equal(eager.conc[:, :n].cpu().numpy(), graphed.conc[:, :n].cpu().numpy())
    assert np.array_equal(eager.counts[:, :n].cpu().numpy(), graphed.counts[:, :n].cpu().numpy())
    for m in eager.lattice.molecules:
        assert np.array_equal(eager.lattice.owned(m).cpu().numpy(), graphed.lattice.owned(m).cpu().numpy()), m


def test_graph_replay_refuses_moved_agents(dev):
    """Moving agents re-bins them (new occupancy buffers): a graph captured
    before holds the old ones, so its replay raises instead of scattering the
    exchange into stale bins."""
    col = _lattice_colony(dev, n=500, nx=64)
    col.step(1.0)
    replay = col.capture(1.0, 1)
    replay()
    rng = np.random.default_rng(9)
    col.set_agents(location=rng.uniform(0.0, 64.0, (2, col.n)))
    with pytest.raises(RuntimeError):
        replay()



def test_stamped_capture_equals_eager_and_stamps_are_ordered(dev):
    """Colony.capture(..., stamps=...) -- the bench's instrumented replay that
    splits a step into kinetics and the rest -- changes nothing: the replayed
    steps equal eager steps bit for bit, and every step's three timestamps are
    in order, the next step's first after its last."""
    import numpy as np
    from lens_amd import native
    a = _lattice_colony(dev)
    b = _lattice_colony(dev)
    stamps = torch.zeros(3 * 4, dtype=torch.int64, device=dev)
    replay = a.capture(1.0, 4, stamps=stamps)
    replay()
    for _ in range(4):
        b.step(1.0)
    torch.cuda.synchronize()
    assert torch.equal(a.conc, b.conc)
    assert torch.equal(a.lattice.fields, b.lattice.fields)
    s = stamps.cpu().numpy().reshape(4, 3)
    assert (np.diff(s, axis=1) > 0).all() and (s[1:, 0] > s[:-1, 2]).all()
    assert native._lib.vk_wall_clock_khz() > 0


@pytest.mark.parametrize('k', [1, 3, 10])
def test_multi_step_launch_equals_single_steps(dev, k):
    """Colony.step_many (vk_step_dopri5_multi): k held-colony steps in one
    launch equal k single steps bit for bit -- state, carried step size, and
    every step's fluxes, exchange counts and attempts -- also replayed from a
    graph (the C2 bench's form)."""
    a, b, c = (_colony(dev, specialize=True) for _ in range(3))
    flux, counts, nsteps = [], [], []
    for _ in range(2 * k):
        b.step(1.0)
        flux.append(b.flux[:, :b.n].clone())
        counts.append(b.counts[:, :b.n].clone())
        nsteps.append(b.nsteps[:b.n].clone())
    for rep in range(2):
        a.step_many(1.0, k)
        for s in range(k):
            assert torch.equal(a.flux_steps[s, :, :a.n], flux[rep * k + s])
            assert torch.equal(a.counts_steps[s, :, :a.n], counts[rep * k + s])
            assert torch.equal(a.nsteps_steps[s, :a.n], nsteps[rep * k + s])
    assert torch.equal(a.conc, b.conc) and torch.equal(a.h_state, b.h_state)
    assert torch.equal(a.flux, b.flux) and torch.equal(a.counts[:, :a.n], b.counts[:, :b.n])
    replay = c.capture(1.0, 2 * k, steps_per_launch=k)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(c.conc, b.conc) and torch.equal(c.h_state, b.h_state)
    # after replay the colony's views hold the last replayed step (not the
    # pre-capture buffers the graph never writes)
    assert torch.equal(c.flux[:, :c.n], b.flux[:, :b.n])
    assert torch.equal(c.counts[:, :c.n], b.counts[:, :b.n])
    assert torch.equal(c.nsteps[:c.n], b.nsteps[:b.n])
    a.check_status()
    c.check_status()


@pytest.mark.parametrize('steps', [1, 2, 5])
def test_overlapped_capture_equals_sequential_steps(dev, steps):
    """capture(overlap=True) of a single-GPU lattice colony overlaps step k's
    exchange with step k+1's kinetics (two counts buffers) and the uniform probe
    with the gather.  Replays of it, of the sequential capture (the default)
    and eager steps agree bit for bit -- fields, every agent array, the counts of
    the last step -- for odd and even steps per graph, and an eager step after
    the replays continues from the same state."""
    cols = [_lattice_colony(dev) for _ in range(3)]
    for c in cols:
        c.sort_by_bin()
        c.step(1.0)
    over = cols[0].capture(1.0, steps, overlap=True)
    seq = cols[1].capture(1.0, steps)
    for _ in range(2):
        over()
        seq()
        for _ in range(steps):
            cols[2].step(1.0)
    for c in cols:
        c.step(1.0)
    torch.cuda.synchronize()
    ref = cols[2]
    for c in cols[:2]:
        c.check_status()
        for name in ('conc', 'flux', 'counts', 'h_state', 'nsteps'):
            assert torch.equal(getattr(c, name)[..., :c.n], getattr(ref, name)[..., :ref.n]), name
        assert torch.equal(c.lattice.fields, ref.lattice.fields)


@pytest.mark.parametrize('sort', [False, True])
def test_fused_gather_equals_separate_gather(dev, sort):
    """vk_step_dopri5_gather (the kinetics launch gathering the next step's local
    environment) against vk_step_dopri5 + vk_gather: every agent array and both
    fields bit for bit after several lattice steps, eager and graph-replayed,
    with agents in generated and in bin order."""
    a, b, c = _lattice_colony(dev), _lattice_colony(dev), _lattice_colony(dev)
    a.fuse_gather = False
    assert b._gather_fused() and not a._gather_fused()
    for col in (a, b, c):
        if sort:
            col.sort_by_bin()
    for _ in range(4):
        a.step(1.0)
        b.step(1.0)
    replay = c.capture(1.0, 4)
    replay()
    torch.cuda.synchronize()
    n = a.n
    for col in (b, c):
        for name in ('conc', 'h_state', 'flux', 'counts', 'nsteps', 'status'):
            x, y = getattr(a, name), getattr(col, name)
            assert torch.equal(x[..., :n], y[..., :n]), name
        assert torch.equal(col.lattice.fields, a.lattice.fields)

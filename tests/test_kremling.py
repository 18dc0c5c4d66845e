"""Kremling 2007 transport: the reference's odeint path.

Oracle: oracle/kremling.py -- the restated RHS integrated by scipy odeint on
the reference's 100-point grid.  The reference holds no fixture for this
process (its test only runs it).  The restatement is pinned to the
reference's own code by tests/golden/kremling_ref.npz
(tests/golden/make_kremling_ref.py evaluates the reference file's
DEFAULT_PARAMETERS and its ``model`` closure, unchanged, in both regimes of
the G6P switch, and integrates that ``model`` with odeint on the reference's
grid): the oracle's RHS equals the reference's bit for bit, and the GPU
kernel's end states are checked against the reference model's odeint.  Truth
is tight odeint (rtol 1e-13); the literal reference call uses odeint's
default tolerances.  Bar (north star): |gpu - odeint| <= 1e-6 * |odeint|
+ 1e-12 per species; fluxes likewise; exchange counts equal to +-1 (counts
truncate a concentration difference, so a last-digit difference can flip an
integer boundary)."""

import os

import numpy as np
import pytest

from oracle import kremling as ok

torch = pytest.importorskip('torch')


def test_oracle_grid_and_shapes():
    t = ok.grid(1.0)
    assert len(t) == 100 and t[-1] == 99 * (0.01 / 3600)
    internal, fluxes, counts, sol = ok.step(ok.initial_state())
    assert internal.shape == (8,) and fluxes.shape == (4,) and counts.shape == (3,)
    assert sol[0, 11:].tolist() == [0.0] * 4


def test_params_layout_matches_reference_names():
    from lens_amd import kremling as lk
    for name in ok.DEFAULT_PARAMETERS:
        assert lk.KREMLING_PARAMETERS[name] == ok.DEFAULT_PARAMETERS[name]
    from lens_amd import native
    assert all(f in lk.KREMLING_PARAMETERS for f, _ in native.VkKremlingParams._fields_)


GOLDEN = os.path.join(os.path.dirname(__file__), 'golden', 'kremling_ref.npz')


def test_oracle_rhs_equals_reference_model():
    """oracle.kremling.rhs == the reference's own model(state, t) (evaluated
    from Kremling2007_transport.py:220-351 by make_kremling_ref.py), bit for
    bit, at 96 states across both regimes of the internal-G6P switch; and the
    restated DEFAULT_PARAMETERS are the reference's."""
    z = np.load(GOLDEN)
    assert tuple(z['keys']) == ok.STATE_KEYS
    assert dict(zip(z['param_names'], z['params'])) == {k: float(v) for k, v in ok.DEFAULT_PARAMETERS.items()}
    states = z['states']
    assert (states[:, 4] > 0.01).sum() == 48 and (states[:, 4] <= 0.01).sum() == 48
    got = np.array([ok.rhs(st, 0.0, ok.DEFAULT_PARAMETERS) for st in states])
    assert np.array_equal(got, z['dy'])


def test_oracle_step_equals_reference_odeint():
    """oracle.kremling.step (odeint of the restated RHS) against odeint of the
    reference model on the same grid and tolerances: identical RHS, so the
    same LSODA path."""
    z = np.load(GOLDEN)
    for j, i in enumerate(z['pick']):
        s = z['states'][i].copy()
        s[11:] = 0.0
        internal, fluxes, _, _ = ok.step(s, rtol=1e-13, atol=1e-16)
        assert np.array_equal(internal, z['end_tight'][j])
        assert np.array_equal(fluxes, z['flux_tight'][j])
        assert np.array_equal(ok.step(s)[0], z['end_default'][j])


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


def _close(got, ref, rel=1e-6, floor=1e-12):
    return np.all(np.abs(got - ref) <= rel * np.abs(ref) + floor)


@pytest.mark.gpu
@pytest.mark.parametrize('condition', ['glc_g6p', 'glc_lct_shift'])
def test_gpu_kremling_matches_odeint(dev, condition):
    from lens_amd.kremling import KremlingColony
    if condition == 'glc_g6p':
        s0 = ok.initial_state()
    else:
        s0 = ok.initial_state(ok.GLC_LCT_SHIFT_INTERNAL, ok.GLC_LCT_SHIFT_EXTERNAL)
    rng = np.random.default_rng(4)
    n = 64
    states = np.repeat(s0[:, None], n, axis=1)
    states[:8, 1:] *= rng.uniform(0.7, 1.3, (8, n - 1))
    states[8:11, 1:] *= rng.uniform(0.5, 1.5, (3, n - 1))
    vol = rng.uniform(0.5, 3.0, n)
    col = KremlingColony(n, device=dev)
    col.set_state(states[:11])
    col.volume.copy_(torch.from_numpy(vol))
    for step in range(3):
        col.step(1.0)
        col.check_status()
        got = col.state.cpu().numpy()
        flux = col.flux.cpu().numpy()
        counts = col.counts.cpu().numpy()
        for a in range(0, n, 9):
            internal, fl, cnt, _ = ok.step(states[:, a], volume_fL=vol[a], rtol=1e-13, atol=1e-16)
            assert _close(got[:8, a], internal), (condition, step, a, got[:8, a], internal)
            assert _close(flux[:, a], fl), (condition, step, a)
            assert np.abs(counts[:, a] - cnt).max() <= 1
            # the literal reference call (odeint default rtol = atol = 1.49e-8) carries up to
            # ~1.5e-6 relative error of its own on XP (measured against the tight odeint):
            # the GPU result is at least as close to the truth as the reference's own
            lit = ok.step(states[:, a], volume_fL=vol[a])[0]
            err_gpu = np.abs(got[:8, a] - internal)
            err_ref = np.abs(lit - internal)
            assert np.all(err_gpu <= np.maximum(1e-6 * np.abs(internal) + 1e-12, err_ref)), (err_gpu, err_ref)
        states[:8] = got[:8]     # internal := last row; external held (environment owns it)


@pytest.mark.gpu
def test_gpu_kremling_vs_reference_model_odeint(dev):
    """One GPU step from each of 12 fixture states (6 per regime) against odeint
    of the reference's own model (kremling_ref.npz): internal species and mean
    fluxes within the north-star 1e-6, or at least as close to the tight
    solution as the reference's literal (default-tolerance) call.  In the
    lactose-branch states the internal G6P starts below the model's 0.01 switch
    (:245) and crosses it within the second: the right-hand side jumps, and an
    integrator stepping over the jump at rtol 1e-8 (the GPU) or at odeint's
    defaults (the reference) lands off the tight solution -- the literal call's
    mean PYK flux by up to 3.5e-6 relative (kremling_ref.npz).  So the mean
    fluxes are held to 1e-6 or to twice the literal call's own error, whichever
    is larger."""
    from lens_amd.kremling import KremlingColony
    z = np.load(GOLDEN)
    states = z['states'][z['pick']].T.copy()          # [15, 12]
    n = states.shape[1]
    col = KremlingColony(n, device=dev)
    col.set_state(states[:11])
    col.step(1.0)
    col.check_status()
    got = col.state.cpu().numpy()[:8]
    flux = col.flux.cpu().numpy()
    for a in range(n):
        ref, fref = z['end_tight'][a], z['flux_tight'][a]
        for g, r, lit, k in ((got[:, a], ref, z['end_default'][a], 1.0), (flux[:, a], fref, z['flux_default'][a], 2.0)):
            err_gpu, err_ref = np.abs(g - r), np.abs(lit - r)
            assert np.all(err_gpu <= np.maximum(1e-6 * np.abs(r) + 1e-12, k * err_ref)), (a, g, r, err_gpu, err_ref)


@pytest.mark.gpu
def test_process_drop_in_update_dict(dev):
    from lens_amd.kremling import BatchedKremlingTransport, GLC_G6P_INTERNAL, GLC_G6P_MEDIA
    proc = BatchedKremlingTransport()
    assert proc.name == 'Kremling2007_transport'
    schema = proc.ports_schema()
    states = {'internal': {k: v['_default'] for k, v in schema['internal'].items()},
              'external': {k: v['_default'] for k, v in schema['external'].items()},
              'global': {'volume': 1.0}}
    upd = proc.next_update(1.0, states)
    internal, fl, cnt, _ = ok.step(ok.initial_state(), rtol=1e-13, atol=1e-16)
    assert set(upd['internal']) == set(GLC_G6P_INTERNAL)
    assert _close(np.array([upd['internal'][k] for k in ok.INTERNAL]), internal)
    assert set(upd['fluxes']) == {'glc__D_e', 'GLCpts', 'PPS', 'PYK'}
    assert set(upd['fields']) == {'GLC', 'G6P', 'LCTS'}
    assert [upd['fields'][m]['_value'] for m in ('GLC', 'G6P', 'LCTS')] == cnt.tolist()
    assert upd['fields']['GLC']['_updater']['updater'] == 'update_field_with_exchange'
    del GLC_G6P_MEDIA


@pytest.mark.gpu
def test_gpu_kremling_avogadro_is_a_parameter(dev):
    """millimolar_to_counts reads scipy.constants.N_A at run time
    (vivarium/library/flux_conversion.py:7,38): 6.022140857e23 under the scipy
    the reference fixtures were made with, 6.02214076e23 from scipy 1.4 on.  The
    kernel takes the constant as an argument; the exchange counts follow
    whichever is passed (oracle with the same constant, +-1 count)."""
    from lens_amd.kremling import KremlingColony
    s0 = ok.initial_state()
    n = 16
    vol = np.linspace(1e7, 3e7, n)        # counts ~1e8: the two constants differ by ~1.3e-7 of them
    got = {}
    for na in (6.022140857e23, 6.02214076e23):
        col = KremlingColony(n, device=dev, avogadro=na)
        col.set_state(np.repeat(s0[:11, None], n, axis=1))
        col.volume.copy_(torch.from_numpy(vol))
        col.step(1.0)
        col.check_status()
        got[na] = col.counts.cpu().numpy()
        for a in range(n):
            cnt = ok.step(s0, volume_fL=vol[a], rtol=1e-13, atol=1e-16, avogadro=na)[2]
            assert np.abs(got[na][:, a] - cnt).max() <= 1
    assert (got[6.022140857e23] != got[6.02214076e23]).any()


@pytest.mark.gpu
def test_gpu_kremling_parameter_sets_interleaved(dev):
    """Two colonies with different parameter sets -- one with the default
    integer exponents (n = 2, m = 1: repeated products), one with n = 1.5
    (the pow path) and another kgly -- stepped alternately on one stream: the
    library's per-set device parameter copies keep them apart, and each
    matches tight odeint on its own parameters."""
    from lens_amd.kremling import KremlingColony
    s0 = ok.initial_state()
    n = 16
    sets = [{}, {'n': 1.5, 'kgly': ok.DEFAULT_PARAMETERS['kgly'] * 1.3}]
    cols = [KremlingColony(n, device=dev, parameters=p) for p in sets]
    for c in cols:
        c.set_state(np.repeat(s0[:11, None], n, axis=1))
    for _ in range(2):
        for c in cols:
            c.step(1.0)
    torch.cuda.synchronize()
    state = s0.copy()
    for c, p in zip(cols, sets):
        c.check_status()
        got = c.state.cpu().numpy()
        params = dict(ok.DEFAULT_PARAMETERS, **p)
        st = s0.copy()
        for _ in range(2):
            internal = ok.step(st, rtol=1e-13, atol=1e-16, params=params)[0]
            st[:8] = internal
        assert _close(got[:8, 0], st[:8]), (p, got[:8, 0], st[:8])
        assert np.array_equal(got[:, 0], got[:, n - 1])
    del state
    assert not np.allclose(cols[0].state.cpu().numpy()[:8, 0], cols[1].state.cpu().numpy()[:8, 0])


@pytest.mark.gpu
def test_gpu_kremling_graph_capture_needs_a_cached_set(dev):
    """a parameter set's device copy is made with a synchronous
    hipMemcpy, which graph capture forbids.  A set seen for the first time
    while the stream captures is refused with a clear error; after one eager
    step with it, capture works and replay equals eager stepping bit for bit."""
    from lens_amd import native
    from lens_amd.kremling import KremlingColony
    s0 = ok.initial_state()
    n = 32
    fresh = {'kgly': ok.DEFAULT_PARAMETERS['kgly'] * 1.0001234}     # a set no other test uses
    a = KremlingColony(n, device=dev, parameters=fresh)
    a.set_state(np.repeat(s0[:11, None], n, axis=1))
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with pytest.raises(native.NativeError, match='graph capture'):
            with torch.cuda.graph(g, stream=s):
                a.step(1.0, carry_h=True)
    torch.cuda.synchronize()
    b = KremlingColony(n, device=dev, parameters=fresh)
    b.set_state(np.repeat(s0[:11, None], n, axis=1))
    a.set_state(np.repeat(s0[:11, None], n, axis=1))
    a.h_state.zero_()
    a.step(1.0, carry_h=True)                 # eager: caches the set
    b.step(1.0, carry_h=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        a.step(1.0, carry_h=True)
    g.replay()
    b.step(1.0, carry_h=True)
    torch.cuda.synchronize()
    assert torch.equal(a.state, b.state) and torch.equal(a.counts, b.counts)

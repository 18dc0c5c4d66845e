"""HIP path vs the oracle, through the C ABI (needs an MI355X)."""

import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from netcodec import decode_network, decode_conc  # noqa: E402
from table_eval import table_euler  # noqa: E402
from lens_amd import configs  # noqa: E402
from lens_amd.rate_law_compiler import compile_rate_laws  # noqa: E402
from oracle import cpu  # noqa: E402
from oracle import lattice as olat  # noqa: E402
from oracle.kinetics import OracleODE, OracleAgent, mmol_to_counts, replay_single_agent  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


def _soa(t, concs):
    return np.ascontiguousarray(np.array([[float(c.get(k, 0.0)) for c in concs] for k in t.species]))


def _engine(t, dev):
    from lens_amd.kinetics import KineticsEngine
    return KineticsEngine(t, dev)


def test_library_is_the_hip_build(dev):
    from lens_amd import native
    lib = native.load()
    assert lib.vk_abi_version() == 1
    assert os.path.samefile(native.LIB_PATH, os.path.join(os.path.dirname(native.__file__), 'lib',
                                                          'libvk_kinetics.so'))


def test_rate_fluxes_bitwise_vs_reference(dev, golden_fluxes):
    for case in golden_fluxes['cases']:
        rx, kp = decode_network(case['network'])
        t = compile_rate_laws(rx, kp)
        concs = [decode_conc(c) for c in case['concs']]
        n = len(concs)
        eng = _engine(t, dev)
        ld = n + 3  # exercise ld > n
        conc = np.zeros((t.n_species, ld))
        conc[:, :n] = _soa(t, concs)
        params = np.repeat(t.param_defaults[:, None], ld, axis=1)
        flux = eng.fluxes(torch.from_numpy(params).to(dev), torch.from_numpy(conc).to(dev), n_agents=n)
        got = flux.cpu().numpy()[:, :n]
        expect = np.array([[f[r] for f in case['fluxes']] for r in t.reaction_ids])
        assert np.array_equal(got, expect), case['name']


def test_euler_step_bitwise(dev, golden_fluxes):
    rng = np.random.default_rng(11)
    for case in golden_fluxes['cases']:
        rx, kp = decode_network(case['network'])
        t = compile_rate_laws(rx, kp)
        concs = [decode_conc(c) for c in case['concs']]
        n = len(concs)
        conc = _soa(t, concs)
        params = np.ascontiguousarray(np.repeat(t.param_defaults[:, None], n, axis=1))
        m2c = rng.uniform(1e5, 1e6, n)
        dt = 1.0
        eng = _engine(t, dev)
        c_dev = torch.from_numpy(conc.copy()).to(dev)
        delta = torch.zeros((t.n_dyn, n), dtype=torch.float64, device=dev)
        flux, counts, status = eng.euler(dt, torch.from_numpy(params).to(dev), c_dev,
                                         torch.from_numpy(m2c).to(dev), delta=delta)
        # delta mode leaves conc untouched
        assert np.array_equal(c_dev.cpu().numpy(), conc)
        flux2, counts2, _ = eng.euler(dt, torch.from_numpy(params).to(dev), c_dev,
                                      torch.from_numpy(m2c).to(dev))
        new = c_dev.cpu().numpy()
        for a in range(n):
            agent = OracleAgent(rx, kp)
            states = {}
            for (port, name), v in concs[a].items():
                states.setdefault(port, {})[name] = v
            fl, deltas, cnt = agent.next_update(dt, states, m2c[a])
            for s in range(t.n_dyn):
                port, name = t.species[s]
                assert delta.cpu().numpy()[s, a] == deltas[port][name]
                assert new[s, a] == conc[s, a] + deltas[port][name]
            assert counts.cpu().numpy()[:, a].tolist() == [cnt[e] for e in t.external_ids]
            assert flux.cpu().numpy()[:, a].tolist() == [fl[r] for r in t.reaction_ids]
        assert not status.cpu().numpy().any()


def test_c1_colony_reproduces_reference_csv(dev):
    """BASELINE config 1 on the GPU: 2520 Euler steps == convenience_kinetics.csv."""
    import csv
    from lens_amd.colony import Colony
    cfg = configs.glc_lct_config()
    col = Colony(cfg, 1, device=dev, integrator='euler', environment='nonspatial')
    rows = {int(float(r['time'])): r for r in csv.DictReader(open(os.path.join(GOLDEN, 'convenience_kinetics_subset.csv')))}
    for step in range(2521):
        if step in rows:
            snap = col.snapshot()
            row = rows[step]
            for port in ('internal', 'external'):
                for name, v in snap[port].items():
                    ref = float(row[port + '_' + name])
                    if port == 'internal':
                        assert abs(v[0] - ref) <= 1e-14 * abs(ref), (step, name)
                    else:
                        assert abs(v[0] - ref) <= 1e-15, (step, name)
        if step < 2520:
            col.step(1.0)


def _params_dict(t, cfg, pvec):
    kp = {}
    for (kind, rid, enz, *mol), v in zip(t.param_names, pvec):
        kp.setdefault(rid, {}).setdefault(enz, {})
        kp[rid][enz]['kcat_f' if kind == 'kcat' else mol[0]] = float(v)
    for rid in cfg['kinetic_parameters']:
        for enz, p in cfg['kinetic_parameters'][rid].items():
            for k, v in p.items():
                if v is None:
                    kp[rid][enz][k] = None
    return kp


@pytest.mark.parametrize('variant', [0, 1])
@pytest.mark.parametrize('name', ['glc_lct', 'glc_ac', 'glc_lct_transport'])
def test_dopri5_matches_odeint(dev, name, variant):
    """North-star bar: end states within 1e-6 relative of scipy odeint (LSODA).

    Tolerance: |gpu - odeint| <= 1e-6*|odeint| + 1e-10.  The absolute floor is
    100x the integrator's atol (1e-12): species driven to ~0 within the step
    (pep_c under the 7.5e4/s PTS kcat) are only resolved to atol, as by
    scipy's own RK45 at the same tolerances."""
    cfg = {'glc_lct': configs.glc_lct_config, 'glc_ac': configs.glc_ac_config,
           'glc_lct_transport': configs.glc_lct_transport_config}[name]()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    n = 300
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=5)
    m2c = np.full(n, mmol_to_counts())
    eng = _engine(t, dev)
    c_dev = torch.from_numpy(conc.copy()).to(dev)
    h = torch.zeros(n, dtype=torch.float64, device=dev)
    flux, counts, status, nsteps = eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev,
                                              torch.from_numpy(m2c).to(dev), h_state=h, variant=variant)
    assert not status.cpu().numpy().any()
    got = c_dev.cpu().numpy()
    fl = flux.cpu().numpy()
    for a in range(0, n, 23):
        ode = OracleODE(cfg['reactions'], _params_dict(t, cfg, params[:, a]))
        new, mean_flux, cnt = ode.step({k: conc[s, a] for s, k in enumerate(t.species)}, 1.0, m2c[a])
        for s in range(t.n_dyn):
            ref = new[t.species[s]]
            assert abs(got[s, a] - ref) <= 1e-6 * abs(ref) + 1e-10, (name, a, t.species[s], got[s, a], ref)
        for r, rid in enumerate(t.reaction_ids):
            assert abs(fl[r, a] - mean_flux[rid]) <= 1e-6 * abs(mean_flux[rid]) + 1e-10


def test_dopri5_matches_c_oracle_all_agents(dev):
    cfg = configs.glc_lct_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    n = 10_000                      # BASELINE config 2 size
    params, conc = configs.heterogeneous_colony(t, cfg, n)
    m2c = np.full(n, mmol_to_counts())
    eng = _engine(t, dev)
    c_dev = torch.from_numpy(conc.copy()).to(dev)
    flux, counts, status, nsteps = eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev,
                                              torch.from_numpy(m2c).to(dev))
    c_ref = conc.copy()
    f_ref, k_ref, s_ref, n_ref = cpu.step_dopri5(cpu.Desc(t), 1.0, params, c_ref, m2c)
    got = c_dev.cpu().numpy()
    rel = np.abs(got[:t.n_dyn] - c_ref[:t.n_dyn]) / (np.abs(c_ref[:t.n_dyn]) + 1e-300)
    assert rel.max() < 1e-10
    # same algorithm, same step sequence
    assert np.mean(nsteps.cpu().numpy() == n_ref) > 0.99


def test_dopri5_status_and_limits(dev):
    from lens_amd.native import NativeError
    cfg = configs.glc_lct_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    params, conc = configs.heterogeneous_colony(t, cfg, 64)
    eng = _engine(t, dev)
    c_dev = torch.from_numpy(conc).to(dev)
    _, _, status, nsteps = eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev,
                                      torch.full((64,), 7e5, dtype=torch.float64, device=dev),
                                      max_steps=1, rtol=1e-12, atol=1e-16)
    assert (status.cpu().numpy() & 1).any()
    # zero agents is a no-op
    eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev,
               torch.full((64,), 7e5, dtype=torch.float64, device=dev), n_agents=0)
    # a 50-species network exceeds the agent-per-thread variant
    big = configs.synthetic_network(n_species=60, n_reactions=40)
    tb = compile_rate_laws(big['reactions'], big['kinetic_parameters'])
    eb = _engine(tb, dev)
    pb = torch.from_numpy(np.repeat(tb.param_defaults[:, None], 8, axis=1)).to(dev)
    cb = torch.ones((tb.n_species, 8), dtype=torch.float64, device=dev)
    assert tb.n_dyn + tb.n_reactions > 32
    with pytest.raises(NativeError):
        eb.dopri5(1.0, pb, cb, torch.ones(8, dtype=torch.float64, device=dev), variant=0)
    with pytest.raises(NativeError):
        eb.dopri5(1.0, pb, cb, torch.ones(8, dtype=torch.float64, device=dev), variant=7)
    assert eb.default_variant() == 1
    with pytest.raises(ValueError):
        eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev[:, :10].contiguous(),
                   torch.ones(64, dtype=torch.float64, device=dev))


def _big_network(ns=50, nr=40, ne=10, n=160, seed=20261015):
    cfg = configs.synthetic_network(n_species=ns, n_reactions=nr, n_enzymes=ne, seed=seed)
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=seed + 1, sigma=0.2)
    return cfg, t, params, conc


@pytest.mark.parametrize('variant', [1, 3])
@pytest.mark.parametrize('shape', [(50, 40, 10), (30, 20, 6), (120, 90, 12), (90, 66, 33)])
def test_dopri5_wave_vs_c_oracle(dev, shape, variant):
    """Agent-per-wavefront DP45 (C5-size networks) == the C oracle's DP45 to
    rounding: same RHS arithmetic, same step control; only the order of the
    error norm's sum differs (a wave reduction).  Variant 1 walks the table,
    variant 3 is the network-specialised kernel (codegen.wave_source; the
    90-species network needs two rounds of 64 rate-law lanes; the padded
    operands of the 120-species one do not fit the register file, so
    specialize() keeps the table walk for it)."""
    from lens_amd import codegen
    cfg, t, params, conc = _big_network(*shape)
    n = conc.shape[1]
    assert t.n_dyn + t.n_reactions > 32
    m2c = np.full(n, mmol_to_counts())
    eng = _engine(t, dev)
    if variant == 3:
        eng.specialize()
        if not eng.specialized:
            assert codegen.wave_registers(t) > eng.WAVE_REGISTER_LIMIT
            variant = 1
    assert eng.default_variant() == variant
    c_dev = torch.from_numpy(conc.copy()).to(dev)
    h = torch.zeros(n, dtype=torch.float64, device=dev)
    flux, counts, status, nsteps = eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev,
                                              torch.from_numpy(m2c).to(dev), h_state=h)
    assert not status.cpu().numpy().any()
    c_ref = conc.copy()
    hr = np.zeros(n)
    f_ref, k_ref, s_ref, n_ref = cpu.step_dopri5(cpu.Desc(t), 1.0, params, c_ref, m2c, h_state=hr)
    got = c_dev.cpu().numpy()
    scale = np.abs(c_ref[:t.n_dyn]) + 1e-9 * np.abs(c_ref[:t.n_dyn]).max(axis=0)
    assert (np.abs(got[:t.n_dyn] - c_ref[:t.n_dyn]) / scale).max() < 1e-9
    assert np.mean(nsteps.cpu().numpy() == n_ref) > 0.95
    fl = flux.cpu().numpy()
    fscale = np.abs(f_ref) + 1e-9 * np.abs(f_ref).max(axis=0)
    assert (np.abs(fl - f_ref) / fscale).max() < 1e-9
    # exchange counts come from the flux integrals: equal up to a one-count
    # truncation flip where the integral sits on an integer boundary
    assert np.abs(counts.cpu().numpy() - k_ref).max() <= 1


def _two_enzyme_network(n=96, seed=20261016):
    """A C5-style network where every third reaction has a second catalyst:
    reactions sum several rate laws (no one-to-one rate law/reaction map)."""
    cfg = configs.synthetic_network(n_species=40, n_reactions=30, n_enzymes=8, seed=seed)
    rng = np.random.default_rng(seed)
    for i, (rid, spec) in enumerate(sorted(cfg['reactions'].items())):
        if i % 3:
            continue
        first = spec['catalyzed by'][0]
        second = ('internal', 'E%02d' % ((int(first[1][1:]) + 1) % 8))
        spec['catalyzed by'] = [first, second]
        p = dict(cfg['kinetic_parameters'][rid][first])
        p['kcat_f'] = float(10 ** rng.uniform(-1, 3))
        cfg['kinetic_parameters'][rid][second] = p
    # an enzyme's partition holds the substrates of every reaction it catalyses
    # (kinetic_rate_laws.py:84-95): each of its rate laws needs their Kms
    for rid, spec in cfg['reactions'].items():
        for enz in spec['catalyzed by']:
            p = cfg['kinetic_parameters'][rid][enz]
            for other in cfg['reactions'].values():
                if enz in other['catalyzed by']:
                    for m, c in other['stoichiometry'].items():
                        if c < 0 and m not in p:
                            p[m] = float(10 ** rng.uniform(-3, 1))
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=seed + 1, sigma=0.2)
    return cfg, t, params, conc


@pytest.mark.parametrize('pad,lds,split,wpe', [(0, 0, 0, 2), (1, 0, 0, 2), (1, 1, 0, 2), (1, 2, 0, 2), (1, 0, 1, 3),
                                              (0, 0, 1, 3), (1, 0, 1, 2)])
@pytest.mark.parametrize('net', ['c5', 'two_enzyme', 'wide'])
def test_dopri5_wave_spec_equals_generic_wave(dev, net, pad, lds, split, wpe):
    """The specialised wavefront kernel (variant 3) against the table walk
    (variant 1): the padded identities are exact and everything else is the
    same arithmetic in the same order, so states, fluxes, counts, step counts
    and carried step sizes agree bit for bit -- with the branch-free LDS
    publishes (pad = 1, padding lanes write a scratch slot), the operand
    tables in LDS (lds = 1, 2), and split denominators (split = 1: the second
    half of a heavy rate law's sets computed in lane l + 32 and added by lane l
    in set order; the 'wide' network has two rounds of rate laws, so the option
    does not apply and the engine keeps one lane per rate law)."""
    from lens_amd import codegen
    if net == 'c5':
        cfg, t, params, conc = _big_network(n=300)
    elif net == 'two_enzyme':
        cfg, t, params, conc = _two_enzyme_network()
        assert not codegen.wave_shape(t)['RX_IDENTITY'] and codegen.wave_shape(t)['RXM'] == 2
    else:
        cfg, t, params, conc = _big_network(90, 66, 33, n=64)
        assert codegen.wave_shape(t)['LR'] == 2
    n = conc.shape[1]
    m2c = torch.full((n,), mmol_to_counts(), dtype=torch.float64, device=dev)
    eng = _engine(t, dev)
    eng.WAVE_PAD_WRITES = pad
    eng.WAVE_LDS_OPS = lds
    eng.WAVE_SPLIT_DEN = split
    eng.WAVE_WAVES_PER_SIMD = wpe
    out = []
    for variant in (1, 3):
        if variant == 3:
            eng.specialize()
        c_dev = torch.from_numpy(conc.copy()).to(dev)
        h = torch.zeros(n, dtype=torch.float64, device=dev)
        flux, counts, status, nsteps = eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev, m2c, h_state=h,
                                                  variant=variant)
        out.append([x.cpu().numpy() for x in (c_dev, flux, counts, status, nsteps, h)])
    for a, b, name in zip(out[0], out[1], ('conc', 'flux', 'counts', 'status', 'nsteps', 'h')):
        assert np.array_equal(a, b), name
    assert not out[1][3].any()


def test_dopri5_wave_matches_odeint(dev):
    """North-star bar on a 50-species network: within 1e-6 relative of odeint."""
    cfg, t, params, conc = _big_network(n=24)
    n = conc.shape[1]
    m2c = np.full(n, mmol_to_counts())
    eng = _engine(t, dev)
    c_dev = torch.from_numpy(conc.copy()).to(dev)
    flux, counts, status, nsteps = eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev,
                                              torch.from_numpy(m2c).to(dev), rtol=1e-10, atol=1e-14)
    assert not status.cpu().numpy().any()
    got = c_dev.cpu().numpy()
    for a in range(0, n, 5):
        ode = OracleODE(cfg['reactions'], _params_dict(t, cfg, params[:, a]))
        new, mean_flux, cnt = ode.step({k: conc[s, a] for s, k in enumerate(t.species)}, 1.0, m2c[a])
        for s_ in range(t.n_dyn):
            ref = new[t.species[s_]]
            assert abs(got[s_, a] - ref) <= 1e-6 * abs(ref) + 1e-10, (a, t.species[s_], got[s_, a], ref)


def test_dopri5_wave_equals_lane_variant_small_network(dev):
    """Both kernels on glc_lct: same trajectory to rounding."""
    cfg = configs.glc_lct_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    n = 2000
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=3)
    m2c = torch.full((n,), mmol_to_counts(), dtype=torch.float64, device=dev)
    eng = _engine(t, dev)
    out = []
    for variant in (0, 1):
        c_dev = torch.from_numpy(conc.copy()).to(dev)
        flux, counts, status, nsteps = eng.dopri5(1.0, torch.from_numpy(params).to(dev), c_dev, m2c,
                                                  variant=variant)
        out.append((c_dev.cpu().numpy(), nsteps.cpu().numpy()))
    rel = np.abs(out[0][0] - out[1][0]) / (np.abs(out[0][0]) + 1e-300)
    assert rel[:t.n_dyn].max() < 1e-10
    assert np.mean(out[0][1] == out[1][1]) > 0.99


@pytest.mark.parametrize('variant,depth', [(2, 1), (2, 3), (2, 5), (2, 9), (2, 13), (2, 15), (3, 7), (3, 9),
                                           (3, 11), (6, 5), (6, 7), (6, 9), (6, 10), (6, 11), (6, 15), (20, 9), (20, 3),
                                           (20, 10)])
def test_stencil_bitwise_vs_scipy_convolve(dev, variant, depth):
    """Every kernel variant and temporal-blocking depth reproduces
    scipy.ndimage.convolve bit for bit."""
    from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel
    z = np.load(os.path.join(GOLDEN, 'stencil.npz'))
    prev = stencil_depth(depth)
    prev_k = stencil_kernel(variant, 16)
    try:
        for shape in ('17x23', '64x64', '128x96'):
            f0 = z['f0_' + shape]
            nx, ny = f0.shape
            for dt in (1.0, 5.0, 10.0):
                lat = Lattice(['a', 'b'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                              initial={'a': f0, 'b': np.full((nx, ny), 2.5)})
                n_sub = lat.diffuse(dt)
                assert n_sub == int(z['n_%s_dt%g' % (shape, dt)])
                assert np.array_equal(lat.owned('a').cpu().numpy(), z['f_%s_dt%g' % (shape, dt)]), (shape, dt)
                assert np.array_equal(lat.owned('b').cpu().numpy(), np.full((nx, ny), 2.5))  # uniform skip
    finally:
        stencil_depth(prev)
        stencil_kernel(prev_k, 0)


@pytest.mark.parametrize('variant,depth,rows', [(2, 9, 64), (2, 7, 128), (2, 11, 32), (2, 15, 256), (3, 9, 64),
                                                (3, 13, 48), (6, 9, 64), (6, 11, 48), (6, 7, 40), (6, 9, 17),
                                                (6, 9, 8), (20, 9, 34), (6, 10, 34), (6, 10, 17), (6, 10, 64)])
@pytest.mark.parametrize('shape', [(700, 1000), (333, 517)])
def test_stencil_large_tiles_vs_c_oracle(dev, variant, depth, rows, shape):
    """Multi-tile / multi-chunk geometry: interior tiles, ragged last tile and
    chunk, odd widths; pipeline fill / branch-free steady state / drain."""
    from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel
    rng = np.random.default_rng(8)
    nx, ny = shape
    f0 = rng.random((nx, ny))
    prev = stencil_kernel(variant, rows)
    prev_d = stencil_depth(depth)
    try:
        lat = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
        lat.diffuse(1.0)
    finally:
        stencil_kernel(prev, 0)
        stencil_depth(prev_d)
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, 5.0 * 0.01, 100)
    assert np.array_equal(lat.owned('a').cpu().numpy(), ref)


@pytest.mark.parametrize('dt', [0.095, 0.2, 0.3, 1.1, 0.55, 0.1])
def test_exact_depth10_block_counts_vs_c_oracle(dev, dt):
    """The exact mode's 10-deep plan for every block shape a step can have: 10
    substeps (dt 0.095: one pass would run in place, so the odd-depth plan takes
    it), 20 / 30 / 110 (10-deep passes, the last one re-reading the step-start
    field) and 55 / 11 (dt 0.55 / 0.1: not multiples of 10, odd depths) -- bit for
    bit against the C oracle."""
    from lens_amd.lattice import Lattice, n_substeps, stencil_depth, stencil_kernel
    rng = np.random.default_rng(21)
    nx, ny = 333, 517
    f0 = rng.random((nx, ny))
    prev_d, prev_k = stencil_depth(10), stencil_kernel(6, 34)
    try:
        lat = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
        n_sub = lat.diffuse(dt)
    finally:
        stencil_depth(prev_d)
        stencil_kernel(prev_k, 0)
    assert n_sub == n_substeps(dt, 0.01)
    ref = np.ascontiguousarray(f0.copy())
    cpu.diffuse(ref, 5.0 * 0.01, n_sub)
    assert np.array_equal(lat.owned('a').cpu().numpy(), ref)


def test_uniform_summary(dev):
    """vk_field_uniform: (v, v) for a one-valued plane, (-inf, inf) otherwise --
    including a single differing cell at the very end and a NaN plane."""
    from lens_amd.lattice import Lattice
    nx, ny = 300, 257
    planes = {'u': np.full((nx, ny), 3.25), 'z': np.zeros((nx, ny)), 'last': np.full((nx, ny), 1.0),
              'first': np.full((nx, ny), 1.0), 'nan': np.full((nx, ny), np.nan),
              'inf': np.full((nx, ny), np.inf), 'rnd': np.random.default_rng(1).random((nx, ny))}
    planes['last'][-1, -1] = 1.0 + 2 ** -52
    planes['first'][0, 0] = -0.0 + 2.0
    lat = Lattice(list(planes), (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial=planes)
    got = lat.uniform_summary().cpu().numpy().reshape(-1, 2)
    expect = {'u': (3.25, 3.25), 'z': (0.0, 0.0), 'inf': (np.inf, np.inf)}
    for f, name in enumerate(planes):
        lo, hi = got[f]
        if name in expect:
            assert (lo, hi) == expect[name], name
        else:
            assert lo == -np.inf and hi == np.inf, name
    # uniform planes come through a diffusion step unchanged, non-uniform ones move
    before = lat.owned().cpu().numpy().copy()
    lat.diffuse(1.0)
    after = lat.owned().cpu().numpy()
    for f, name in enumerate(planes):
        if name in ('u', 'z', 'inf'):
            assert np.array_equal(after[f], before[f]), name
    ref = np.ascontiguousarray(planes['rnd'].copy())
    cpu.diffuse(ref, 5.0 * 0.01, 100)
    assert np.array_equal(after[list(planes).index('rnd')], ref)


def test_single_substep_diffusion(dev):
    from lens_amd.lattice import Lattice
    rng = np.random.default_rng(2)
    f0 = rng.random((20, 30))
    lat = Lattice(['a'], (20, 30), (20.0, 30.0), 10.0, 5.0, device=dev, initial={'a': f0})
    lat.diffuse(0.005)   # one substep (dt < 0.01)
    ref = olat.diffuse(f0, 0.005, 5.0, (20, 30), (20.0, 30.0))
    assert np.array_equal(lat.owned('a').cpu().numpy(), ref)


def test_banded_diffusion_equals_whole(dev):
    """Row bands with k-deep halos (the multi-GPU decomposition) on one device."""
    from lens_amd.lattice import Lattice
    rng = np.random.default_rng(3)
    nx, ny = 97, 40
    f0 = rng.random((nx, ny)) * 5
    whole = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
    whole.diffuse(1.0)
    for world, halo in ((2, 8), (3, 5), (4, 1), (3, 16)):
        from lens_amd.distributed import row_bands
        bands = row_bands(nx, world)
        lats = [Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                        row_band=b, halo=halo, initial={'a': f0}) for b in bands]

        def make_ex(r):
            def ex(src, cnt):
                lat = lats[r]
                names = {id(lat.fields): 'fields', id(lat.work0): 'work0', id(lat.work1): 'work1'}
                which = names[id(src)]
                if not lat.edge_top:
                    nb = lats[r - 1]
                    s = getattr(nb, which)
                    src[:, lat.row_lo - halo:lat.row_lo].copy_(s[:, nb.row_hi - halo:nb.row_hi])
                if not lat.edge_bot:
                    nb = lats[r + 1]
                    s = getattr(nb, which)
                    src[:, lat.row_hi:lat.row_hi + halo].copy_(s[:, nb.row_lo:nb.row_lo + halo])
            return ex

        # lock-step: every band runs block j before any runs block j+1
        from lens_amd import native
        n_sub = 100
        coeff_dt = lats[0].diffusion * 0.01
        j = 0
        while j < n_sub:
            cnt = min(halo, n_sub - j)
            for r, lat in enumerate(lats):
                src = lat.fields if j == 0 else (lat.work0 if ((j - 1) & 1) == 0 else lat.work1)
                make_ex(r)(src, cnt)
            for lat in lats:
                lo_min = lat.row_lo if lat.edge_top else 0
                hi_max = lat.row_hi if lat.edge_bot else lat.rows_local
                native.check(native._lib.vk_diffuse(
                    native.ptr(lat.fields), native.ptr(lat.work0), native.ptr(lat.work1), 1,
                    lat.field_stride, ny, lat.row_lo, lat.row_hi, lo_min, hi_max, int(lat.edge_top),
                    int(lat.edge_bot), j, cnt, n_sub, coeff_dt, 0, native.stream_handle()), 'diffuse')
            j += cnt
        got = torch.cat([lat.owned('a') for lat in lats], 0).cpu().numpy()
        assert np.array_equal(got, whole.owned('a').cpu().numpy()), (world, halo)


@pytest.mark.parametrize('mode', ['fma', 'exact'])
def test_banded_depth10_plan_equals_whole(dev, mode):
    """The 10-deep block plan on row bands with one 100-deep halo block per step
    (the C4 bench at N > 1) equals the whole plane under the same plan bit for
    bit: the same cells, the same arithmetic.  In the exact mode every plan gives
    scipy's bits, so the whole plane also equals the depth-9 odd plan's."""
    from lens_amd import native
    from lens_amd.distributed import row_bands
    from lens_amd.lattice import Lattice, stencil_depth, stencil_mode
    rng = np.random.default_rng(4)
    nx, ny = 300, 237
    f0 = rng.random((nx, ny)) * 5
    prev_m, prev_d = stencil_mode(mode), stencil_depth(10)
    try:
        whole = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
        whole.diffuse(1.0)
        if mode == 'exact':
            stencil_depth(9)
            nine = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
            nine.diffuse(1.0)
            stencil_depth(10)
            assert np.array_equal(nine.owned('a').cpu().numpy(), whole.owned('a').cpu().numpy())
        for world in (2, 3):
            bands = row_bands(nx, world)
            lats = [Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                            row_band=b, halo=100, initial={'a': f0}) for b in bands]
            for r, lat in enumerate(lats):          # the one halo exchange of the step
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
        # shallower halos: blocks of 10 k substeps are 10-deep passes too, chained
        # through the buffers the halo exchanges read (work[(j-1)&1] before block j;
        # a block inside the step starts and ends in the same work buffer, so it
        # needs an even number of passes -- halo 30 would plan its middle blocks at
        # odd depths, within the tolerance but not bit for bit)
        for world, halo in ((3, 50), (3, 20), (2, 40)) + (((3, 30),) if mode == 'exact' else ()):
            bands = row_bands(nx, world)
            lats = [Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                            row_band=b, halo=halo, initial={'a': f0}) for b in bands]
            j = 0
            while j < 100:
                cnt = min(halo, 100 - j)
                name = 'fields' if j == 0 else ('work0' if ((j - 1) & 1) == 0 else 'work1')
                for r, lat in enumerate(lats):
                    src = getattr(lat, name)
                    if not lat.edge_top:
                        nb = getattr(lats[r - 1], name)
                        src[:, lat.row_lo - halo:lat.row_lo].copy_(nb[:, lats[r - 1].row_hi - halo:lats[r - 1].row_hi])
                    if not lat.edge_bot:
                        nb = getattr(lats[r + 1], name)
                        src[:, lat.row_hi:lat.row_hi + halo].copy_(nb[:, lats[r + 1].row_lo:lats[r + 1].row_lo + halo])
                for lat in lats:
                    lo_min = lat.row_lo if lat.edge_top else 0
                    hi_max = lat.row_hi if lat.edge_bot else lat.rows_local
                    native.check(native._lib.vk_diffuse(
                        native.ptr(lat.fields), native.ptr(lat.work0), native.ptr(lat.work1), 1,
                        lat.field_stride, ny, lat.row_lo, lat.row_hi, lo_min, hi_max, int(lat.edge_top),
                        int(lat.edge_bot), j, cnt, 100, lat.diffusion * 0.01, 0, native.stream_handle()), 'diffuse')
                j += cnt
            got = torch.cat([lat.owned('a') for lat in lats], 0).cpu().numpy()
            assert np.array_equal(got, whole.owned('a').cpu().numpy()), (world, halo)
    finally:
        stencil_mode(prev_m)
        stencil_depth(prev_d)


def test_lattice_colony_side_stream_overlap_is_exact(dev):
    """Kinetics + gather on the side stream beside the diffusion passes gives
    the same fields and agent state, bit for bit, as the one-stream order --
    stepped eagerly and replayed from a captured graph (the side stream forks
    from and joins the captured stream inside every step)."""
    from lens_amd.colony import Colony
    from lens_amd.lattice import Lattice
    cfg = configs.glc_ac_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    nx, n = 256, 20000
    rng = np.random.default_rng(21)
    loc = rng.uniform(0, float(nx), (2, n))
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=5)
    out = []
    for overlap, graph in ((False, False), (True, False), (True, True)):
        lat = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (float(nx), float(nx)), 10.0, 5.0, device=dev,
                      initial={'glc__D_e': configs.gaussian_bump_field((nx, nx)), 'ac_e': np.zeros((nx, nx))})
        col = Colony(cfg, n, device=dev, integrator='dopri5', environment=lat, table=t, specialize=True)
        col.overlap_kinetics = overlap
        col.set_agents(params=params, conc=conc, location=loc)
        col.gather_external()
        if graph:
            col.capture(1.0, 3)()
        else:
            for _ in range(3):
                col.step(1.0)
        torch.cuda.synchronize()
        out.append((lat.owned('glc__D_e').cpu().numpy(), lat.owned('ac_e').cpu().numpy(),
                    col.conc[:, :n].cpu().numpy(), col.counts[:, :n].cpu().numpy()))
    for got in out[1:]:
        for a, b in zip(out[0], got):
            assert np.array_equal(a, b)


def test_lattice_colony_step_vs_oracle(dev):
    """Gather (pre-step) -> diffusion -> agent-ordered exchange, bit-exact, with a
    bin shared by several agents."""
    from lens_amd.colony import Colony
    from lens_amd.lattice import Lattice
    cfg = configs.glc_ac_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    nx, ny, n = 24, 20, 200
    bounds = (24.0, 20.0)
    glc = configs.gaussian_bump_field((nx, ny))
    ac = np.zeros((nx, ny))
    rng = np.random.default_rng(9)
    loc = np.stack([rng.uniform(0, bounds[0], n), rng.uniform(0, bounds[1], n)])
    loc[:, 5] = loc[:, 3]  # agents 3 and 5 share a bin
    for exchange in ('sorted', 'atomic'):
        lat = Lattice(['glc__D_e', 'ac_e'], (nx, ny), bounds, 10.0, 5.0, device=dev,
                      initial={'glc__D_e': glc, 'ac_e': ac})
        col = Colony(cfg, n, device=dev, integrator='euler', environment=lat, table=t, exchange=exchange)
        params, conc = configs.heterogeneous_colony(t, cfg, n, seed=4)
        col.set_agents(params=params, conc=conc, location=loc)
        col.gather_external()
        conc0 = col.conc.cpu().numpy().copy()
        col.step(1.0)
        # oracle: Euler per agent (table order) + lattice_step in agent order
        m2c = col.m2c.cpu().numpy()
        counts = {m: [] for m in t.external_ids}
        for a in range(n):
            _, _, cnt = table_euler(t, conc0[:, a], params[:, a], 1.0, m2c[a])
            for e, m in enumerate(t.external_ids):
                counts[m].append(int(cnt[e]))
        new, local = olat.lattice_step({'glc__D_e': glc.copy(), 'ac_e': ac.copy()},
                                       [tuple(loc[:, a]) for a in range(n)], counts, (nx, ny), bounds,
                                       10.0, 1.0, 5.0)
        got_g = lat.owned('glc__D_e').cpu().numpy()
        if exchange == 'sorted':
            assert np.array_equal(got_g, new['glc__D_e'])
            assert np.array_equal(lat.owned('ac_e').cpu().numpy(), new['ac_e'])
        else:
            np.testing.assert_allclose(got_g, new['glc__D_e'], rtol=1e-14, atol=0)
        ext = col.species('external', 'glc__D_e').cpu().numpy()
        assert np.array_equal(ext, local['glc__D_e'])


def test_process_drop_in_update_dict(dev):
    from lens_amd.process import BatchedConvenienceKinetics
    from lens_amd.invoke import BatchedInvoke
    cfg = configs.glc_lct_config()
    proc = BatchedConvenienceKinetics(cfg)
    states = {'internal': dict(cfg['initial_state']['internal']),
              'external': {'glc__D_e': 3.0, 'lcts_e': 2.0},
              'fluxes': {}, 'fields': {}, 'global': {'mmol_to_counts': 733058.77, 'location': [0.5, 0.5]},
              'dimensions': {}}
    update = proc.next_update(1.0, states)
    agent = OracleAgent(cfg['reactions'], cfg['kinetic_parameters'])
    fl, deltas, counts = agent.next_update(1.0, states, 733058.77)
    assert update['fluxes'] == fl
    assert update['internal'] == {k: v for k, v in deltas['internal'].items()}
    assert {m: v['_value'] for m, v in update['fields'].items()} == counts
    assert update['fields']['glc__D_e']['_updater']['updater'] == 'update_field_with_exchange'
    # batched: many processes, one launch per (network, interval)
    inv = BatchedInvoke()
    procs = [BatchedConvenienceKinetics(cfg) for _ in range(50)]
    futs = []
    for i, p in enumerate(procs):
        st = {**states, 'external': {'glc__D_e': 0.1 * (i + 1), 'lcts_e': 1.0}}
        futs.append((inv(p, 1.0, st), st))
    for f, st in futs:
        got = f.get()
        fl, deltas, counts = agent.next_update(1.0, st, 733058.77)
        assert got['fluxes'] == fl and got['internal'] == deltas['internal']
        assert {m: v['_value'] for m, v in got['fields'].items()} == counts


@pytest.mark.parametrize('name', ['glc_lct', 'glc_ac', 'glc_lct_transport'])
def test_specialized_dopri5_bitwise_equals_generic(dev, name):
    """The hiprtc-specialised kernel evaluates the same operations in the same
    order as the table-walking kernel: identical end states and step counts."""
    cfg = {'glc_lct': configs.glc_lct_config, 'glc_ac': configs.glc_ac_config,
           'glc_lct_transport': configs.glc_lct_transport_config}[name]()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    n = 3000
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=12)
    m2c = torch.full((n,), mmol_to_counts(), dtype=torch.float64, device=dev)
    eng = _engine(t, dev)
    p = torch.from_numpy(params).to(dev)
    c0 = torch.from_numpy(conc.copy()).to(dev)
    c2 = torch.from_numpy(conc.copy()).to(dev)
    f0, k0, s0, n0 = eng.dopri5(1.0, p, c0, m2c, variant=0)
    eng.specialize()
    f2, k2, s2, n2 = eng.dopri5(1.0, p, c2, m2c)
    assert torch.equal(c0, c2) and torch.equal(f0, f2) and torch.equal(k0, k2)
    assert torch.equal(n0, n2) and torch.equal(s0, s2)

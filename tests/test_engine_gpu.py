"""A lattice colony through the Experiment-shaped loop on the GPU (needs an MI355X).

SURVEY §8 a9 + N2: the environment is ``BatchedDiffusionField`` (fields on
the device, vk_diffuse_delta + one gather), every agent runs
``BatchedConvenienceKinetics`` (all agents of a step in one launch through
``BatchedInvoke``) and a second process on another interval, and the agents'
``update_field_with_exchange`` updates land as one agent-ordered scatter per
field.  The same colony runs through ``oracle.experiment.OracleExperiment``
with the reference's process semantics (oracle rate laws, numpy diffusion,
one-agent-at-a-time exchange).  Euler kinetics: every agent state and every
field must agree bit for bit, at several intervals, with processes on 1, 2
and 3 s clocks.
"""

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

NX, NY, N = 20, 16, 40


class EnzymeExpression:
    """A second per-agent process on its own clock: EIIglc += rate * timestep
    (accumulate).  Plain Python: it runs the same under both loops."""
    name = 'enzyme_expression'

    def __init__(self, rate, time_step):
        self.rate, self.time_step = rate, time_step

    def local_timestep(self):
        return self.time_step

    def is_deriver(self):
        return False

    def ports_schema(self):
        return {'internal': {'EIIglc': {'_default': 0.0}}}

    def next_update(self, timestep, states):
        return {'internal': {'EIIglc': self.rate * timestep * (1.0 + states['internal']['EIIglc'])}}


def _colony(batched, dev, expression=True):
    from lens_amd import configs
    from lens_amd.process import BatchedConvenienceKinetics, BatchedDiffusionField
    from oracle.experiment import OracleConvenienceKinetics, OracleDiffusionField
    from oracle.kinetics import mmol_to_counts
    cfg = configs.glc_ac_config()
    rng = np.random.default_rng(3)
    locs = [[float(rng.uniform(0, NX)), float(rng.uniform(0, NY))] for _ in range(N)]
    locs[5] = list(locs[2])                                    # a shared bin
    glc = configs.gaussian_bump_field((NX, NY))
    env = {'molecules': ['glc__D_e', 'ac_e'], 'n_bins': [NX, NY], 'bounds': [float(NX), float(NY)],
           'depth': 10.0, 'diffusion': 5.0, 'time_step': 3.0,
           'initial_state': {'glc__D_e': glc, 'ac_e': np.zeros((NX, NY))}}
    processes = {'diffusion': BatchedDiffusionField(dict(env, device=dev)) if batched else OracleDiffusionField(env),
                 'agents': {}}
    topology = {'diffusion': {'agents': ('agents',), 'fields': ('fields',), 'dimensions': ('dimensions',)},
                'agents': {}}
    agents = {}
    for a in range(N):
        kin_cfg = dict(cfg, time_step=1.0)
        kin = BatchedConvenienceKinetics(kin_cfg) if batched else OracleConvenienceKinetics(kin_cfg)
        aid = 'a%02d' % a
        processes['agents'][aid] = {'kinetics': kin}
        topology['agents'][aid] = {
            'kinetics': {'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
                         'fields': ('..', '..', 'fields'), 'dimensions': ('..', '..', 'dimensions'),
                         'global': ('boundary',)}}
        if expression:
            processes['agents'][aid]['expression'] = EnzymeExpression(1e-4 * (1 + a % 3), 2.0)
            topology['agents'][aid]['expression'] = {'internal': ('internal',)}
        internal = {k: v * (1 + 0.01 * a) for k, v in cfg['initial_state']['internal'].items()}
        agents[aid] = {'internal': internal, 'fluxes': {},
                       'boundary': {'location': locs[a], 'mmol_to_counts': mmol_to_counts(1339.0 + a),
                                    'external': {'glc__D_e': 0.0, 'ac_e': 0.0}}}
    init = {'agents': agents,
            'dimensions': {'bounds': env['bounds'], 'n_bins': env['n_bins'], 'depth': env['depth']}}
    return processes, topology, init


def _to_host(x):
    if hasattr(x, 'cpu'):
        return x.cpu().numpy()
    return x


def _host_tree(t):
    if isinstance(t, dict):
        return {k: _host_tree(v) for k, v in t.items()}
    if isinstance(t, list):
        return [_host_tree(v) for v in t]
    x = _to_host(t)
    return x.copy() if isinstance(x, np.ndarray) else x


def _compare(a, b, path=()):
    if isinstance(b, dict):
        assert isinstance(a, dict) and sorted(a) == sorted(b), path
        for k in b:
            _compare(a[k], b[k], path + (k,))
    else:
        x, y = _to_host(a), _to_host(b)
        if isinstance(y, np.ndarray):
            assert np.array_equal(x, y), path
        else:
            assert x == y, (path, x, y)


def test_lattice_colony_through_the_loop_equals_reference_restatement():
    from lens_amd.engine import Experiment
    from lens_amd.invoke import BatchedInvoke
    from oracle.experiment import OracleExperiment
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    p, t, init = _colony(True, dev)
    gpu = Experiment({'processes': p, 'topology': t, 'initial_state': init, 'invoke': BatchedInvoke(dev)})
    p, t, init = _colony(False, dev)
    ref = OracleExperiment(p, t, init)
    for interval in (1.0, 4.0, 0.5, 5.5):
        gpu.update(interval)
        ref.update(interval)
        torch.cuda.synchronize()
        assert gpu.local_time == ref.local_time
        _compare(gpu.state['agents'], ref.state['agents'])
        _compare(gpu.state['fields'], ref.state['fields'])
    # the run exchanged with the field and diffused it
    ac = _to_host(gpu.state['fields']['ac_e'])
    assert ac.max() > 0 and np.count_nonzero(ac) > N


@pytest.mark.parametrize('expression', [False, True])
def test_columnar_agents_through_the_loop_equal_reference_restatement(expression):
    """The same colony with its agents held in columns (lens_amd.agent_store): with
    kinetics alone per agent the kinetics run is one scheduler entry, one pack
    from the columns and one column apply (and the diffusion process's agent
    leaves one column write); with a second process per agent the per-agent
    path runs over row views.  Both equal the oracle loop bit for bit."""
    from lens_amd.engine import Experiment
    from lens_amd.invoke import BatchedInvoke
    from oracle.experiment import OracleExperiment
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    p, t, init = _colony(True, dev, expression)
    gpu = Experiment({'processes': p, 'topology': t, 'initial_state': init, 'invoke': BatchedInvoke(dev),
                      'agent_columns': ('agents',)})
    p, t, init = _colony(False, dev, expression)
    ref = OracleExperiment(p, t, init)
    for interval in (1.0, 4.0, 0.5, 5.5):
        gpu.update(interval)
        ref.update(interval)
        torch.cuda.synchronize()
        assert gpu.local_time == ref.local_time
        _compare(gpu.state['agents'], ref.state['agents'])
        _compare(gpu.state['fields'], ref.state['fields'])
    groups = [e for e in gpu._sched_cache[3] if type(e).__name__ == '_Group']
    assert bool(groups) == (not expression)


def test_diffusion_field_process_update_dict_vs_oracle():
    """BatchedDiffusionField.next_update: the field deltas bit for bit (uniform
    fields: zero) and every agent's external = the pre-step field at its bin."""
    from lens_amd.process import BatchedDiffusionField
    from oracle.experiment import OracleDiffusionField
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    rng = np.random.default_rng(4)
    f0 = rng.random((33, 21)) * 4
    env = {'molecules': ['a', 'u'], 'n_bins': [33, 21], 'bounds': [66.0, 21.0], 'depth': 3.0, 'diffusion': 9.0,
           'initial_state': {'a': f0, 'u': np.full((33, 21), 2.0)}}
    agents = {str(k): {'boundary': {'location': [float(rng.uniform(-5, 70)), float(rng.uniform(0, 21))]}}
              for k in range(25)}
    for timestep in (1.0, 0.005, 2.5):
        got = BatchedDiffusionField(dict(env, device=dev)).next_update(
            timestep, {'fields': {'a': torch.from_numpy(f0).to(dev), 'u': torch.full((33, 21), 2.0,
                                                                                   dtype=torch.float64,
                                                                                   device=dev)},
                       'agents': agents})
        want = OracleDiffusionField(env).next_update(timestep, {'fields': {'a': f0, 'u': np.full((33, 21), 2.0)},
                                                                'agents': agents})
        assert np.array_equal(got['fields']['a'].cpu().numpy(), want['fields']['a']), timestep
        assert np.array_equal(got['fields']['u'].cpu().numpy(), np.zeros((33, 21)))
        assert got['agents'] == {k: {'boundary': {'external': {m: float(v) for m, v in
                                                               w['boundary']['external'].items()}}}
                                 for k, w in want['agents'].items()}


# ---------------------------------------------------------------------------
# the device-resident Colony on per-process clocks
# ---------------------------------------------------------------------------

def _lattice_colony(dev, integrator, n=60, nx=24, ny=20, seed=8):
    from lens_amd import configs
    from lens_amd.colony import Colony
    from lens_amd.lattice import Lattice
    from lens_amd.rate_law_compiler import compile_rate_laws
    cfg = configs.glc_ac_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    rng = np.random.default_rng(seed)
    loc = np.stack([rng.uniform(0, nx, n), rng.uniform(0, ny, n)])
    loc[:, 4] = loc[:, 1]
    params, conc = configs.heterogeneous_colony(t, cfg, n, seed=seed)
    glc = configs.gaussian_bump_field((nx, ny))
    lat = Lattice(['glc__D_e', 'ac_e'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev,
                  initial={'glc__D_e': glc, 'ac_e': np.zeros((nx, ny))})
    col = Colony(cfg, n, device=dev, integrator=integrator, environment=lat, table=t)
    col.set_agents(params=params, conc=conc, location=loc)
    col.gather_external()
    return cfg, t, col, lat, params, conc, loc, glc


@pytest.mark.parametrize('integrator', ['euler', 'dopri5'])
def test_colony_run_single_clock_equals_step(integrator):
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    _, _, a, la, *_ = _lattice_colony(dev, integrator)
    _, _, b, lb, *_ = _lattice_colony(dev, integrator)
    for _ in range(4):
        a.step(1.0)
        b.run(1.0, kinetics_dt=1.0, diffusion_dt=1.0)
    torch.cuda.synchronize()
    assert torch.equal(a.conc, b.conc) and torch.equal(a.counts, b.counts) and torch.equal(a.flux, b.flux)
    assert torch.equal(la.owned(), lb.owned())


def test_colony_run_multirate_equals_reference_loop():
    """Kinetics every 1 s, the diffusion field every 2.5 s (Euler): the device
    colony's schedule equals the restated Experiment.update with oracle
    processes, bit for bit, across several run() calls."""
    from oracle.experiment import OracleConvenienceKinetics, OracleDiffusionField, OracleExperiment
    from oracle.kinetics import params_dict
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    cfg, t, col, lat, params, conc, loc, glc = _lattice_colony(dev, 'euler')
    n, (nx, ny) = col.n, lat.n_bins
    m2c = col.m2c[:n].cpu().numpy()
    ext0 = col.conc[:, :n].cpu().numpy()
    env = {'molecules': ['glc__D_e', 'ac_e'], 'n_bins': [nx, ny], 'bounds': [float(nx), float(ny)],
           'depth': 10.0, 'diffusion': 5.0, 'time_step': 2.5,
           'initial_state': {'glc__D_e': glc, 'ac_e': np.zeros((nx, ny))}}
    processes = {'diffusion': OracleDiffusionField(env), 'agents': {}}
    topology = {'diffusion': {'agents': ('agents',), 'fields': ('fields',), 'dimensions': ('dimensions',)},
                'agents': {}}
    agents = {}
    for a in range(n):
        aid = 'a%03d' % a
        kp = params_dict(t.param_names, cfg, params[:, a])
        processes['agents'][aid] = {'kinetics': OracleConvenienceKinetics(dict(cfg, kinetic_parameters=kp,
                                                                               time_step=1.0))}
        topology['agents'][aid] = {'kinetics': {
            'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
            'fields': ('..', '..', 'fields'), 'dimensions': ('..', '..', 'dimensions'), 'global': ('boundary',)}}
        agents[aid] = {
            'internal': {k[1]: conc[s, a] for s, k in enumerate(t.species) if k[0] == 'internal'},
            'fluxes': {},
            'boundary': {'location': [loc[0, a], loc[1, a]], 'mmol_to_counts': m2c[a],
                         'external': {k[1]: ext0[s, a] for s, k in enumerate(t.species) if k[0] == 'external'}}}
    ref = OracleExperiment(processes, topology, {'agents': agents, 'dimensions': {
        'bounds': env['bounds'], 'n_bins': env['n_bins'], 'depth': env['depth']}})
    for interval in (3.0, 5.0, 1.5):
        col.run(interval, kinetics_dt=1.0, diffusion_dt=2.5)
        ref.update(interval)
        torch.cuda.synchronize()
        got = col.conc[:, :n].cpu().numpy()
        for s, (port, name) in enumerate(t.species):
            where = 'internal' if port == 'internal' else None
            want = np.array([ref.state['agents']['a%03d' % a]['internal' if where else 'boundary']
                             [name] if where else ref.state['agents']['a%03d' % a]['boundary']['external'][name]
                             for a in range(n)])
            assert np.array_equal(got[s], want), (interval, port, name)
        for f, m in enumerate(lat.molecules):
            assert np.array_equal(lat.owned(m).cpu().numpy(), ref.state['fields'][m]), (interval, m)


def _dividing_colony(batched, dev, n=24, seed=4):
    """growth_division_minimal's compartment (GrowthProtein + the MetaDivision
    deriver, daughters regenerated from the same compartment) with the
    convenience kinetics of the lattice colony above on every agent."""
    from lens_amd import configs
    from lens_amd.division import GrowthProtein, MetaDivision
    from lens_amd.process import BatchedConvenienceKinetics, BatchedDiffusionField
    from oracle.experiment import OracleConvenienceKinetics, OracleDiffusionField
    from oracle.kinetics import mmol_to_counts
    cfg = configs.glc_ac_config()
    rng = np.random.default_rng(seed)
    glc = configs.gaussian_bump_field((NX, NY))
    env = {'molecules': ['glc__D_e', 'ac_e'], 'n_bins': [NX, NY], 'bounds': [float(NX), float(NY)],
           'depth': 10.0, 'diffusion': 5.0, 'time_step': 2.0,
           'initial_state': {'glc__D_e': glc, 'ac_e': np.zeros((NX, NY))}}

    def compartment(agent_id):
        kin_cfg = dict(cfg, time_step=1.0)
        kin = BatchedConvenienceKinetics(kin_cfg) if batched else OracleConvenienceKinetics(kin_cfg)
        return {'processes': {'kinetics': kin, 'growth': GrowthProtein({'growth_rate': 0.08}),
                              'division': MetaDivision({'agent_id': agent_id, 'daughter_path': (),
                                                        'compartment': lambda c: compartment(c['agent_id'])})},
                'topology': {'kinetics': {'internal': ('internal',), 'external': ('boundary', 'external'),
                                          'fluxes': ('fluxes',), 'fields': ('..', '..', 'fields'),
                                          'dimensions': ('..', '..', 'dimensions'), 'global': ('boundary',)},
                             'growth': {'internal': ('internal',), 'global': ('boundary',)},
                             'division': {'global': ('boundary',), 'cells': ('..', '..', 'agents')}}}

    processes = {'diffusion': BatchedDiffusionField(dict(env, device=dev)) if batched else OracleDiffusionField(env),
                 'agents': {}}
    topology = {'diffusion': {'agents': ('agents',), 'fields': ('fields',), 'dimensions': ('dimensions',)},
                'agents': {}}
    agents = {}
    for a in range(n):
        aid = str(a)
        c = compartment(aid)
        processes['agents'][aid], topology['agents'][aid] = c['processes'], c['topology']
        internal = {k: v * (1 + 0.01 * a) for k, v in cfg['initial_state']['internal'].items()}
        internal['protein'] = c['processes']['growth'].initial_protein * float(rng.uniform(1.0, 1.9))
        agents[aid] = {'internal': internal, 'fluxes': {},
                       'boundary': {'location': [float(rng.uniform(0, NX)), float(rng.uniform(0, NY))],
                                    'mmol_to_counts': mmol_to_counts(1339.0 + a), 'volume': 1.0 + 0.01 * a,
                                    'divide': False, 'external': {'glc__D_e': 0.0, 'ac_e': 0.0}}}
    init = {'agents': agents,
            'dimensions': {'bounds': env['bounds'], 'n_bins': env['n_bins'], 'depth': env['depth']}}
    return processes, topology, init


def test_dividing_colony_through_batched_loop_equals_reference_restatement():
    """A growth_division_minimal-style colony (MetaDivision + GrowthProtein +
    BatchedConvenienceKinetics under BatchedInvoke, Euler) on the device
    lattice, through lens_amd.engine.Experiment, against the oracle loop
    (oracle kinetics, numpy diffusion, one-agent exchange): agent ids, their
    order, every agent state and both fields bit for bit after every interval,
    with divisions along the way (daughters appended in mother order, mothers
    deleted, their processes gone)."""
    import random
    from lens_amd.engine import Experiment
    from lens_amd.invoke import BatchedInvoke
    from oracle.experiment import OracleExperiment
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    intervals = (1.0, 3.0, 0.5, 4.5, 2.0, 5.0)

    def run(batched):
        np.random.seed(21)
        random.seed(21)
        p, t, init = _dividing_colony(batched, dev)
        exp = (Experiment({'processes': p, 'topology': t, 'initial_state': init, 'invoke': BatchedInvoke(dev)})
               if batched else OracleExperiment(p, t, init))
        out = []
        for interval in intervals:
            exp.update(interval)
            if batched:
                torch.cuda.synchronize()
            fields = {m: _to_host(v).copy() for m, v in exp.state['fields'].items()}
            # a deep copy: a loop may update nested stores (boundary.external) in place
            agents = _host_tree(exp.state['agents'])
            out.append((exp.local_time, list(exp.state['agents']), agents, fields,
                        sorted(exp.processes['agents'])))
        return out

    gpu, ref = run(True), run(False)
    for k, (g, r) in enumerate(zip(gpu, ref)):
        assert g[0] == r[0], k
        assert g[1] == r[1], (k, g[1], r[1])
        _compare(g[2], r[2], ('agents', k))
        _compare(g[3], r[3], ('fields', k))
        assert g[4] == r[4] == sorted(g[1])
    assert len(gpu[-1][1]) > 24                                # divisions happened

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


def _colony(batched, dev):
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
        processes['agents'][aid] = {'kinetics': kin, 'expression': EnzymeExpression(1e-4 * (1 + a % 3), 2.0)}
        topology['agents'][aid] = {
            'kinetics': {'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
                         'fields': ('..', '..', 'fields'), 'dimensions': ('..', '..', 'dimensions'),
                         'global': ('boundary',)},
            'expression': {'internal': ('internal',)}}
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

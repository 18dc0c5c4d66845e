"""The Experiment-shaped driver (lens_amd.engine) against the
literal restatement of the reference's loop (oracle.experiment), on CPU.

* the reference's own multi-rate scenario (experiment.py:1734-1801
  test_timescales: a 3.0 s and a 0.3 s process on one store) plus a 0.7 s
  process, run through both loops: identical states bit for bit;
* BASELINE config 1 (convenience kinetics + NonSpatialEnvironment deriver)
  through both loops reproduces the reference fixture convenience_kinetics.csv
  -- which pins the restated scheduler, update order and updaters.
"""

import csv
import os

import numpy as np
import pytest

from lens_amd import configs
from lens_amd.engine import Experiment
from lens_amd.process import Process
from oracle.experiment import (OracleConvenienceKinetics, OracleExperiment, OracleNonSpatialEnvironment,
                               nonspatial_dimensions)
from oracle.kinetics import mmol_to_counts

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


class Slow(Process):
    name = 'slow'
    defaults = {'timestep': 3.0}

    def ports_schema(self):
        return {'state': {'base': {'_default': 1.0}}}

    def local_timestep(self):
        return self.parameters['timestep']

    def next_update(self, timestep, states):
        return {'state': {'base': timestep * states['state']['base'] * 0.1}}


class Fast(Process):
    name = 'fast'
    defaults = {'timestep': 0.3}

    def ports_schema(self):
        return {'state': {'base': {'_default': 1.0}, 'motion': {'_default': 0.0}}}

    def local_timestep(self):
        return self.parameters['timestep']

    def next_update(self, timestep, states):
        return {'state': {'motion': timestep * states['state']['base'] * 0.001}}


class Odd(Process):
    name = 'odd'
    defaults = {'time_step': 0.7}

    def ports_schema(self):
        return {'state': {'motion': {'_default': 0.0}, 'tally': {'_default': 0.0, '_updater': 'set'}}}

    def next_update(self, timestep, states):
        return {'state': {'tally': states['state']['motion'] + timestep,
                          'motion': -0.5 * timestep * states['state']['motion']}}


def _timescales(loop, odd=True):
    processes = {'slow': Slow(), 'fast': Fast()}
    topology = {'slow': {'state': ('state',)}, 'fast': {'state': ('state',)}}
    if odd:
        processes['odd'] = Odd()
        topology['odd'] = {'state': ('state',)}
    init = {'state': {'base': 1.0, 'motion': 0.0}}
    if loop is OracleExperiment:
        return OracleExperiment(processes, topology, init)
    return Experiment({'processes': processes, 'topology': topology, 'initial_state': init})


@pytest.mark.parametrize('odd', [False, True])
def test_multirate_loop_equals_reference_restatement(odd):
    a, b = _timescales(Experiment, odd), _timescales(OracleExperiment, odd)
    for interval in (10.0, 3.3, 0.05, 6.65):
        a.update(interval)
        b.update(interval)
        assert a.state == b.state, interval
        assert a.local_time == b.local_time
    # the slow process really ran at its own rate: base grew 4 times in 10 s
    c = _timescales(OracleExperiment, False).update(10.0)
    base = 1.0
    for dt in (3.0, 3.0, 3.0, 1.0):
        base = base + dt * base * 0.1
    assert c.state['state']['base'] == base


def _c1(loop):
    cfg = configs.glc_lct_config()
    ports = ('internal', 'external', 'fluxes', 'fields', 'global', 'dimensions')
    processes = {'kinetics': OracleConvenienceKinetics(cfg),
                 'environment': OracleNonSpatialEnvironment({'volume_L': 1e-14})}
    topology = {'kinetics': {p: (p,) for p in ports},
                'environment': {p: (p,) for p in ('external', 'fields', 'dimensions', 'global')}}
    init = {'internal': dict(cfg['initial_state']['internal']),
            'external': dict(cfg['initial_state']['external']),
            'fields': {m: np.ones((1, 1)) for m in cfg['initial_state']['external']},
            'global': {'mmol_to_counts': mmol_to_counts(), 'location': [0.5, 0.5]},
            'dimensions': nonspatial_dimensions(1e-14), 'fluxes': {}}
    if loop is OracleExperiment:
        return OracleExperiment(processes, topology, init)
    return Experiment({'processes': processes, 'topology': topology, 'initial_state': init})


@pytest.mark.parametrize('loop', [Experiment, OracleExperiment])
def test_c1_through_the_loop_reproduces_reference_csv(loop):
    rows = {int(float(r['time'])): r for r in csv.DictReader(open(os.path.join(GOLDEN,
                                                                             'convenience_kinetics_subset.csv')))}
    exp = _c1(loop)
    for step in range(max(rows) + 1):
        if step in rows:
            for port in ('internal', 'external'):
                for name, v in exp.state[port].items():
                    ref = float(rows[step][port + '_' + name])
                    tol = 1e-14 * abs(ref) if port == 'internal' else 1e-15
                    assert abs(v - ref) <= tol, (step, port, name, v, ref)
        exp.update(1.0)


def test_c1_both_loops_bitwise():
    a, b = _c1(Experiment), _c1(OracleExperiment)
    for _ in range(50):
        a.update(1.0)
        b.update(1.0)
    for port in ('internal', 'external', 'fluxes'):
        assert a.state[port] == b.state[port]
    for m in a.state['fields']:
        assert np.array_equal(a.state['fields'][m], b.state['fields'][m])


class _FakeKineticsInvoke:
    """An invoke hook that returns seeded kinetics outputs for every
    BatchedConvenienceKinetics call, either as a future with ``raw()`` (the
    path BatchedInvoke takes in lens_amd.engine) or with ``get()`` only (the
    reference's protocol: the update dict of unpack_update)."""

    class _F:
        def __init__(self, out, with_raw):
            self.out = out
            if with_raw:
                self.raw = lambda: self.out

        def get(self, timeout=0):
            p, f, d, c = self.out
            return p.unpack_update(f, d, c)

    def __init__(self, with_raw, seed=5):
        self.with_raw = with_raw
        self.rng = np.random.default_rng(seed)

    def __call__(self, process, interval, states):
        from lens_amd.process import BatchedConvenienceKinetics
        if not isinstance(process, BatchedConvenienceKinetics):
            out = process.next_update(interval, states)
            return type('I', (), {'get': lambda self, timeout=0: out})()
        t = process.table
        out = (process, self.rng.normal(size=t.n_reactions).tolist(), self.rng.normal(size=t.n_dyn).tolist(),
               self.rng.integers(-50, 50, size=t.n_ext).tolist())
        return self._F(out, self.with_raw)


def test_direct_kinetics_apply_equals_update_dict():
    """engine.Experiment applies a BatchedInvoke result straight into the store
    (_apply_kinetics: cached store nodes and updaters) instead of building and
    walking the update dict.  Against the dict path on CPU -- seeded outputs,
    6 agents, host fields (the reference's update_field_with_exchange
    arithmetic), a missing flux leaf and 3 steps -- the stores are identical,
    value and type."""
    from lens_amd.process import BatchedConvenienceKinetics
    cfg = configs.glc_lct_config()
    states = []
    for with_raw in (True, False):
        procs, topo, agents = {'agents': {}}, {'agents': {}}, {}
        for a in range(6):
            aid = 'a%d' % a
            procs['agents'][aid] = {'kinetics': BatchedConvenienceKinetics(dict(cfg, time_step=1.0))}
            topo['agents'][aid] = {'kinetics': {
                'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
                'fields': ('..', '..', 'fields'), 'dimensions': ('..', '..', 'dimensions'), 'global': ('boundary',)}}
            agents[aid] = {'internal': dict(cfg['initial_state']['internal']), 'fluxes': {},
                           'boundary': {'location': [0.5 + a, 1.5], 'mmol_to_counts': 1e6 * (a + 1),
                                        'external': dict(cfg['initial_state']['external'])}}
        init = {'agents': agents, 'dimensions': {'bounds': [8.0, 4.0], 'n_bins': [8, 4], 'depth': 3.0},
                'fields': {m: np.ones((8, 4)) for m in cfg['initial_state']['external']}}
        exp = Experiment({'processes': procs, 'topology': topo, 'initial_state': init,
                          'invoke': _FakeKineticsInvoke(with_raw)})
        del exp.state['agents']['a3']['fluxes'][sorted(exp.state['agents']['a3']['fluxes'])[0]]
        exp.update(3.0)
        if with_raw:
            plans = [p['kinetics'].__dict__.get('_engine_kinetics_plan') for p in exp.processes['agents'].values()]
            assert len(plans) == 6 and all(e is not None and e[2] is not None for e in plans)
        states.append(exp.state)

    def same(x, y):
        if isinstance(x, dict):
            return isinstance(y, dict) and list(x) == list(y) and all(same(x[k], y[k]) for k in x)
        if isinstance(x, np.ndarray):
            return isinstance(y, np.ndarray) and np.array_equal(x, y)
        return type(x) is type(y) and (x == y or (x != x and y != y))

    assert same(states[0], states[1])
    assert not np.array_equal(states[0]['fields']['glc__D_e'], np.ones((8, 4)))     # the exchange landed


class _LeafWriter(Process):
    """Writes every listed agent's boundary.external leaves each step: rows of
    seeded values over a key list that grows after the first step (a key no
    agent had resolved yet), as an AgentLeafUpdate (``leaf_raw``) or as the
    reference's update dict only."""
    name = 'leaf_writer'

    def __init__(self, ids, with_raw):
        super().__init__({'time_step': 1.0})
        self.ids, self.with_raw, self.calls = ids, with_raw, 0
        self.rng = np.random.default_rng(11)

    def ports_schema(self):
        return {'agents': {'*': {'boundary': {'external': {
            'glc': {'_default': 0.0, '_updater': 'set'},
            'ac': {'_default': 0.0},                                   # accumulate
            'lac': {'_default': 1.0, '_updater': 'halve_then_add'}}}}}}

    def next_update_raw(self, timestep, states):
        from lens_amd.process import AgentLeafUpdate
        self.calls += 1
        keys = ['glc', 'ac'] if self.calls == 1 else ['glc', 'ac', 'lac', 'absent']
        rows = self.rng.normal(size=(len(self.ids), len(keys))).tolist()
        return AgentLeafUpdate({}, list(self.ids), ('boundary', 'external'), keys, rows)


class _LeafInvoke:
    def __init__(self, with_raw):
        self.with_raw = with_raw

    def __call__(self, process, interval, states):
        up = process.next_update_raw(interval, states)
        if self.with_raw:
            return type('L', (), {'get': lambda s, timeout=0: up.as_dict(), 'leaf_raw': lambda s: up})()
        return type('D', (), {'get': lambda s, timeout=0: up.as_dict()})()


def test_leaf_columns_apply_equals_update_dict():
    """Experiment._apply_leaves (an AgentLeafUpdate applied as columns, with its
    per-agent branch cache) against apply_update of the same update's dict: set,
    accumulate and a custom updater; a key list that grows on the second step;
    an agent id with no store, an agent without the branch and a leaf the store
    lacks -- identical stores after 3 steps."""
    states = []
    for with_raw in (True, False):
        agents = {'a%d' % i: {'boundary': {'external': {'glc': 1.0 * i, 'ac': 0.5, 'lac': 2.0}}} for i in range(5)}
        agents['a3'] = {'other': {}}                       # no boundary branch
        del agents['a2']['boundary']['external']['ac']     # a missing leaf
        ids = ['a0', 'a1', 'a2', 'a3', 'a4', 'ghost']
        exp = Experiment({'processes': {'w': _LeafWriter(ids, with_raw)}, 'topology': {'w': {'agents': ('agents',)}},
                          'initial_state': {'agents': agents}, 'invoke': _LeafInvoke(with_raw)})
        exp.updaters['halve_then_add'] = lambda cur, new, st: cur * 0.5 + new
        exp.update(3.0)
        states.append(exp.state)
    assert states[0] == states[1]
    assert 'absent' not in states[0]['agents']['a0']['boundary']['external']


def test_engine_caches_stay_out_of_process_copies():
    """The engine keeps per-process caches (store nodes, kinetics plans) in the
    process's __dict__; a deep copy or pickle of the process after a run carries
    None there, not the engine and its store (a shallow copy shares the entries,
    which check the process and its path before use)."""
    import copy
    import pickle
    from lens_amd.process import BatchedConvenienceKinetics
    cfg = configs.glc_lct_config()
    proc = BatchedConvenienceKinetics(dict(cfg, time_step=1.0))
    topo = {'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
            'fields': ('fields',), 'dimensions': ('dimensions',), 'global': ('boundary',)}
    init = {'internal': dict(cfg['initial_state']['internal']), 'fluxes': {},
            'boundary': {'location': [0.5, 0.5], 'mmol_to_counts': 1e6,
                         'external': dict(cfg['initial_state']['external'])},
            'dimensions': {'bounds': [2.0, 2.0], 'n_bins': [2, 2], 'depth': 1.0},
            'fields': {m: np.ones((2, 2)) for m in cfg['initial_state']['external']}}
    exp = Experiment({'processes': {'k': proc}, 'topology': {'k': topo}, 'initial_state': init,
                      'invoke': _FakeKineticsInvoke(True)})
    exp.update(2.0)
    assert proc.__dict__.get('_engine_state_nodes') is not None
    assert proc.__dict__.get('_engine_kinetics_plan') is not None
    for other in (copy.deepcopy(proc), pickle.loads(pickle.dumps(proc))):
        assert other.__dict__.get('_engine_state_nodes') is None
        assert other.__dict__.get('_engine_kinetics_plan') is None
        assert other.signature == proc.signature


def test_batched_invoke_groups_and_fills_futures(monkeypatch):
    """BatchedInvoke on the host side (the launch replaced): calls are grouped by
    (network, interval, integrator) in first-call order, each group is one
    _run_group call over its members in call order, every future receives its
    own agent's outputs, and the first get() / raw() flushes everything recorded."""
    from lens_amd import invoke as inv
    from lens_amd.process import BatchedConvenienceKinetics
    runs = []

    def fake_run_group(items, device=None, raw=False):
        runs.append([(it.process.tag, it.interval) for it in items])
        t = items[0].process.table
        return [(it.process, [float(it.process.tag)] * t.n_reactions, [0.0] * t.n_dyn, [it.process.tag] * t.n_ext)
                for it in items]

    monkeypatch.setattr(inv, '_run_group', fake_run_group)
    cfg_a, cfg_b = configs.glc_lct_config(), configs.glc_ac_config()
    procs = []
    for tag, (cfg, dt) in enumerate([(cfg_a, 1.0), (cfg_b, 1.0), (cfg_a, 1.0), (cfg_a, 2.0), (cfg_b, 1.0)]):
        p = BatchedConvenienceKinetics(dict(cfg, time_step=dt))
        p.tag = tag
        procs.append((p, dt, cfg))
    b = inv.BatchedInvoke()
    futs = []
    for p, dt, cfg in procs:
        states = {port: dict(vals) for port, vals in cfg['initial_state'].items()}
        states['global'] = {'mmol_to_counts': 1e6, 'location': [0.5, 0.5]}
        futs.append(b(p, dt, states))
    assert runs == []                                   # nothing launched before the first result is asked for
    p3, f3, _, c3 = futs[3].raw()
    assert p3 is procs[3][0] and f3[0] == 3.0 and c3[0] == 3
    assert runs == [[(0, 1.0), (2, 1.0)], [(1, 1.0), (4, 1.0)], [(3, 2.0)]]
    for k, fut in enumerate(futs):                      # the rest are already filled: no second launch
        assert fut.raw()[0] is procs[k][0] and fut.raw()[3][0] == k
        assert fut.get()['fluxes'] == dict.fromkeys(procs[k][0].table.reaction_ids, float(k))
    assert len(runs) == 3

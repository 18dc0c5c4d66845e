"""Division through the Process-API loop (CPU): lens_amd.engine.Experiment
against the oracle's restatement of the reference loop (oracle/experiment.py),
with growth_division_minimal's processes -- GrowthProtein and the MetaDivision
deriver (lens_amd/division.py; vivarium/compartments/growth_division_minimal.py,
growth_protein.py, meta_division.py) -- plus a second process on its own
clock.  Both loops draw the same random numbers (GrowthProtein's remainder,
``split`` of integer counts), so agent ids, their order and every state must
agree bit for bit after every interval.
"""

import os
import random
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lens_amd.division import GrowthProtein, MetaDivision, daughter_phylogeny_id  # noqa: E402
from lens_amd.engine import Experiment  # noqa: E402
from oracle.experiment import OracleExperiment  # noqa: E402


class Counter:
    """A plain per-agent process on a 2 s clock with an integer count that
    ``split`` divides (a random odd remainder) and a float that ``zero`` resets."""
    name = 'counter'

    def local_timestep(self):
        return 2.0

    def is_deriver(self):
        return False

    def ports_schema(self):
        return {'internal': {'tokens': {'_default': 7, '_divider': 'split'},
                             'age': {'_default': 0.0, '_divider': 'zero'}}}

    def next_update(self, timestep, states):
        return {'internal': {'tokens': 3, 'age': timestep}}


def compartment(agent_id, rate=0.05):
    return {'processes': {'growth': GrowthProtein({'growth_rate': rate}),
                          'counter': Counter(),
                          'division': MetaDivision({'agent_id': agent_id, 'daughter_path': (),
                                                    'compartment': lambda cfg: compartment(cfg['agent_id'], rate)})},
            'topology': {'growth': {'internal': ('internal',), 'global': ('boundary',)},
                         'counter': {'internal': ('internal',)},
                         'division': {'global': ('boundary',), 'cells': ('..', '..', 'agents')}}}


def colony(n=12, seed=5):
    rng = np.random.default_rng(seed)
    processes, topology, agents = {'agents': {}}, {'agents': {}}, {}
    for a in range(n):
        aid = str(a)
        c = compartment(aid)
        processes['agents'][aid] = c['processes']
        topology['agents'][aid] = c['topology']
        p0 = c['processes']['growth'].initial_protein
        agents[aid] = {'internal': {'protein': p0 * float(rng.uniform(1.0, 1.95)), 'tokens': 5 + a, 'age': 0.0},
                       'boundary': {'volume': 1.2 + 0.01 * a, 'divide': False}}
    return processes, topology, {'agents': agents}


def run(kind, intervals, seed=11):
    np.random.seed(seed)
    random.seed(seed)
    p, t, init = colony()
    cfg = {'processes': p, 'topology': t, 'initial_state': init}
    if kind == 'columns':                     # the agents held in columns (lens_amd.agent_store)
        cfg['agent_columns'] = ('agents',)
    exp = Experiment(cfg) if kind in ('engine', 'columns') else OracleExperiment(p, t, init)
    snaps = []
    for interval in intervals:
        exp.update(interval)
        snaps.append((exp.local_time, list(exp.state['agents']), repr(exp.state['agents']),
                      sorted(exp._walk(exp.processes, ()), key=lambda x: x[0]).__len__()))
    return snaps, exp


INTERVALS = (1.0, 2.0, 0.5, 3.5, 4.0, 1.0, 6.0)


@pytest.mark.parametrize('kind', ['engine', 'columns'])
def test_division_ids_order_and_states_equal_reference_loop(kind):
    got, eng = run(kind, INTERVALS)
    ref, orc = run('oracle', INTERVALS)
    assert len(got) == len(ref)
    for k, (g, r) in enumerate(zip(got, ref)):
        assert g[0] == r[0], k
        assert g[1] == r[1], (k, g[1], r[1])             # agent ids, in store order
        assert g[2] == r[2], k                           # every value, bit for bit (repr)
        assert g[3] == r[3], k                           # the process tree
    ids = got[-1][1]
    assert len(ids) > 12                                 # divisions happened
    # lineage: every agent descends from a root through daughter_phylogeny_id
    roots = {str(a) for a in range(12)}
    for aid in ids:
        assert aid[0] in roots or aid[:2] in roots and all(c in '01' for c in aid[len(aid.rstrip('01')):])
    # daughters are appended after the survivors, in mother order, and the mother is gone
    for aid in ids:
        if len(aid) > 1 and aid[:-1] not in ids:
            assert aid[:-1] + '0' in ids and aid[:-1] + '1' in ids
    # no process of a deleted mother is left in the tree
    assert set(eng.processes['agents']) == set(ids)


def test_divided_values_follow_the_schema_dividers():
    """One division checked by hand: protein and volume split in half, the
    integer count split with its odd remainder to one daughter, age zeroed,
    the divide flag reset (divider_set_false), the rest copied."""
    np.random.seed(0)
    random.seed(0)
    p, t, _ = colony(1)
    growth = p['agents']['0']['growth']
    init = {'agents': {'0': {'internal': {'protein': growth.divide_protein * 1.5, 'tokens': 9, 'age': 2.5},
                             'boundary': {'volume': 2.0, 'divide': True}}}}
    exp = Experiment({'processes': p, 'topology': t, 'initial_state': init})
    # the derivers ran at construction: the mother divided at once
    assert list(exp.state['agents']) == daughter_phylogeny_id('0')
    d0, d1 = (exp.state['agents'][k] for k in daughter_phylogeny_id('0'))
    for d in (d0, d1):
        assert d['internal']['protein'] == growth.divide_protein * 1.5 / 2
        assert d['boundary']['volume'] == 1.0
        assert d['boundary']['divide'] is False
        assert d['internal']['age'] == 0
    assert sorted([d0['internal']['tokens'], d1['internal']['tokens']]) == [4, 5]
    assert set(exp.processes['agents']) == set(daughter_phylogeny_id('0'))
    assert exp.processes['agents']['00']['division'].agent_id == '00'


@pytest.mark.parametrize('maker_first', [False, True])
@pytest.mark.parametrize('structure', ['generate', 'delete', 'add'])
def test_generate_delete_add_updates(structure, maker_first):
    """_generate, _delete and _add at a branch, engine vs oracle.  With the
    structural process first, its _delete lands before the deleted agent's own
    updates of the same batch, which Store.apply_update then drops
    (experiment.py:699-711) instead of failing."""
    class Maker:
        name = 'maker'

        def local_timestep(self):
            return 1.0

        def is_deriver(self):
            return False

        def ports_schema(self):
            return {'cells': {'*': {}}}

        def next_update(self, timestep, states):
            if structure == 'generate':
                c = compartment('new%d' % len(states['cells']))
                return {'cells': {'_generate': [{'path': ('new%d' % len(states['cells']),),
                                                 'processes': {'counter': c['processes']['counter']},
                                                 'topology': {'counter': c['topology']['counter']},
                                                 'initial_state': {'internal': {'tokens': 1}}}]}}
            if structure == 'delete':
                return {'cells': {'_delete': [(k,) for k in list(states['cells'])[:1]]}}
            return {'cells': {'_add': [{'path': ('added%d' % len(states['cells']),),
                                        'state': {'x': 1.0}}]}}

    def build(kind):
        np.random.seed(1)
        random.seed(1)
        p, t, init = colony(3)
        if maker_first:
            p, t = {'maker': Maker(), **p}, {'maker': {'cells': ('agents',)}, **t}
        else:
            p['maker'] = Maker()
            t['maker'] = {'cells': ('agents',)}
        return Experiment({'processes': p, 'topology': t, 'initial_state': init}) if kind == 'engine' else \
            OracleExperiment(p, t, init)

    def snaps(kind):                     # one loop after the other: they draw from one RNG
        exp = build(kind)
        out = []
        for _ in range(3):
            exp.update(1.0)
            out.append((list(exp.state['agents']), repr(exp.state['agents'])))
        return out

    a, b = snaps('engine'), snaps('oracle')
    assert a == b
    assert len(a[-1][0]) == {'generate': 6, 'delete': 0, 'add': 6}[structure]


def test_deleted_derivers_are_forgotten_after_their_pass():
    """A deriver deleted in one send_updates pass is skipped only in that pass:
    the ids of deleted processes must not outlive it, or a new process that
    reuses a freed object's id would never run (the engine and the oracle hold
    the deleted objects for the pass and start every pass afresh)."""
    for kind in ('engine', 'oracle'):
        np.random.seed(0)
        random.seed(0)
        p, t, init = colony(2)
        exp = Experiment({'processes': p, 'topology': t, 'initial_state': init}) if kind == 'engine' else \
            OracleExperiment(p, t, init)
        deriver = exp.processes['agents']['0']['division']
        stale = {id(deriver): deriver}
        if kind == 'engine':
            exp._deleted = stale
        else:
            exp.deleted = stale
        exp.state['agents']['0']['boundary']['divide'] = True
        exp.send_updates([])
        assert '0' not in exp.state['agents'] and '00' in exp.state['agents'], kind


def test_deleting_agents_forgets_their_cache_entries():
    """A dividing colony must not keep every deleted mother's port nodes (each holds
    the mother's state subtree), port paths, schema updaters or dividers: after
    the loop, the caches hold entries for live agents only."""
    np.random.seed(1)
    random.seed(1)
    p, t, init = colony(3)
    exp = Experiment({'processes': p, 'topology': t, 'initial_state': init})
    for _ in range(12):
        exp.update(1.0)
    live = set(exp.state['agents'])
    assert len(live) > 3                                # the colony divided
    for (ppath, port) in list(exp._port_nodes) + list(exp._port_paths):
        if len(ppath) > 1 and ppath[0] == 'agents':
            assert ppath[1] in live, ppath
    for path in list(exp.schema) + list(exp.dividers):
        if len(path) > 1 and path[0] == 'agents' and path[1] != '*':
            assert path[1] in live, path


def test_regenerated_path_takes_its_new_schema():
    """A path deleted and generated again with another updater uses the new one
    (the reference builds fresh Stores), not the deleted subtree's."""
    class Leaf:
        name = 'leaf'

        def __init__(self, updater):
            self.updater = updater

        def local_timestep(self):
            return 1.0

        def is_deriver(self):
            return False

        def ports_schema(self):
            return {'x': {'v': {'_default': 0.0, '_updater': self.updater}}}

        def next_update(self, timestep, states):
            return {'x': {'v': 2.0}}

    exp = Experiment({'processes': {'cells': {'a': {'leaf': Leaf('accumulate')}}},
                      'topology': {'cells': {'a': {'leaf': {'x': ('x',)}}}},
                      'initial_state': {'cells': {'a': {'x': {'v': 1.0}}}}})
    exp.update(1.0)
    assert exp.state['cells']['a']['x']['v'] == 3.0
    exp._delete_path(('cells', 'a'))
    exp._generate(('cells',), ('a',), {'leaf': Leaf('set')}, {'leaf': {'x': ('x',)}}, {'x': {'v': 1.0}})
    exp.update(1.0)
    assert exp.state['cells']['a']['x']['v'] == 2.0          # set, not accumulate


def test_derive_globals_reads_width_and_density_from_the_store():
    """derive_globals.py:133-135 takes density and width from states['global'] on
    every call, not from the process parameters: a store holding other values
    derives with those (the same formulas as a CellModel built with them)."""
    from lens_amd.cells import CellModel
    from lens_amd.division import AVOGADRO, DeriveGlobals
    dg = DeriveGlobals()
    default = dg.next_update(1.0, {'global': {'mass': 1500.0, 'width': 1, 'density': 1100.0}})['global']
    other = dg.next_update(1.0, {'global': {'mass': 1500.0, 'width': 0.8, 'density': 1000.0}})['global']
    vol, m2c, length, area = CellModel(width=0.8, density=1000.0, avogadro=AVOGADRO).derive(1500.0)
    assert (other['volume'], other['mmol_to_counts'], other['length'], other['surface_area']) == (vol, m2c, length, area)
    assert other['length'] != default['length']
    # a store without the two leaves falls back to the parameters
    assert dg.next_update(1.0, {'global': {'mass': 1500.0}})['global'] == default

"""Columnar agent store (lens_amd/agent_store.py): an AgentsNode behaves as the
dict of per-agent dicts it replaces -- reads, writes, missing keys, branches
replaced as a whole, deletion with row reuse, copies -- while its leaves live in
columns that batched code reads and writes as arrays."""

import copy

import numpy as np

from lens_amd.agent_store import AgentsNode, AgentView, to_dict


def sample():
    return {'a': {'internal': {'glc': 1.5, 'n': 3}, 'boundary': {'location': [1.0, 2.0], 'mass': np.float64(2.0)},
                  'fluxes': {}},
            'b': {'internal': {'glc': 2.5}, 'boundary': {'location': [3.0, 4.0], 'mass': np.float64(4.0)},
                  'fluxes': {}}}


def test_reads_match_the_dicts():
    ref = sample()
    node = AgentsNode(copy.deepcopy(ref))
    assert list(node) == ['a', 'b']
    assert to_dict(node['a']) == ref['a'] and node['b'] == ref['b']
    assert repr(node) == repr(ref)
    a = node['a']
    assert isinstance(a, dict) and isinstance(a['internal'], dict)
    assert type(a['internal']['glc']) is float and type(a['boundary']['mass']) is np.float64
    assert a['internal']['n'] == 3 and type(a['internal']['n']) is int
    assert 'n' in a['internal'] and 'n' not in node['b']['internal']
    assert node['b']['internal'].get('n', 7) == 7 and len(node['b']['internal']) == 1
    assert a['fluxes'] == {} and 'fluxes' in a and not a['fluxes']
    assert a['boundary']['location'] == [1.0, 2.0]


def test_writes_types_and_branch_replacement():
    node = AgentsNode(sample())
    a = node['a']
    a['internal']['glc'] = a['internal']['glc'] + 1.0
    assert a['internal']['glc'] == 2.5 and node['b']['internal']['glc'] == 2.5
    a['internal']['glc'] = 7                                  # an int: the column turns object
    assert type(node['a']['internal']['glc']) is int and type(node['b']['internal']['glc']) is float
    a['fluxes']['r1'] = np.float64(0.5)
    assert node['a']['fluxes'] == {'r1': 0.5} and 'r1' not in node['b']['fluxes']
    a['internal'] = {'x': 1.0}                                # a branch replaced as a whole
    assert to_dict(node['a']['internal']) == {'x': 1.0}
    del a['boundary']['mass']
    assert 'mass' not in node['a']['boundary'] and node['b']['boundary']['mass'] == 4.0


def test_rows_are_freed_and_reused_in_order():
    node = AgentsNode(sample())
    t = node.table
    row_a = node.row('a')
    del node['a']
    assert list(node) == ['b']
    node['c'] = {'internal': {'glc': 9.0}}
    assert node.row('c') == row_a                             # the freed row, at the end of the order
    assert list(node) == ['b', 'c'] and to_dict(node['c']) == {'internal': {'glc': 9.0}}
    assert 'boundary' not in node['c']                        # nothing of 'a' shows through
    for k in range(100):                                      # growth past the capacity
        node['x%d' % k] = {'internal': {'glc': float(k)}}
    assert node['x99']['internal']['glc'] == 99.0 and t.cap >= 102


def test_columns_gather_and_scatter():
    node = AgentsNode(sample())
    t = node.table
    rows = node.rows(['b', 'a'])
    assert t.gather(('internal', 'glc'), rows).tolist() == [2.5, 1.5]
    assert t.gather(('internal', 'n'), rows, default=-1.0).tolist() == [-1.0, 3.0]
    t.scatter(('internal', 'glc'), rows, np.array([5.0, 6.0]))
    assert node['a']['internal']['glc'] == 6.0 and node['b']['internal']['glc'] == 5.0
    t.scatter(('fluxes', 'r2'), rows, np.array([1.0, 2.0]), np_scalar=True)
    assert type(node['a']['fluxes']['r2']) is np.float64 and node['b']['fluxes']['r2'] == 1.0


def test_copies_are_plain_dicts():
    node = AgentsNode(sample())
    c = copy.deepcopy(node['a'])
    assert type(c) is dict and type(c['internal']) is dict
    node['a']['internal']['glc'] = 0.0
    assert c['internal']['glc'] == 1.5
    assert type(node.copy()['b']) is dict
    assert isinstance(node['a'], AgentView)

"""The Process-API dividing loop pinned to the reference's own fixture.

reference_data/colony_metrics.csv (tests/golden/colony_metrics.csv.gz) is what
the reference's colony_metrics experiment wrote
(vivarium/experiments/colony_metrics_experiment.py:183-213): two
growth_division_minimal agents (GrowthProtein + the TreeMass / DeriveGlobals
derivers it asks for + MetaDivision) at growth_rate 0.001, random.seed(1) and
np.random.seed(1), 2400 one-second steps, every step emitted.  Here the same
colony runs through lens_amd.engine.Experiment -- the reference's scheduler,
structural updates (_divide), dividers and deriver order restated over a dict
store -- with the reference's draw order (the two multibody angle draws of
single_agent_config, then one GrowthProtein draw per agent per step), and its
emitted data goes through the reference's timeseries -> CSV transforms.  The
CSV must equal the fixture byte for byte: agent ids and their order, the
division times, and mass / volume / width / length / surface_area / protein at
every row.  (tests/test_emitter.py pins the device Colony to the same file.)
"""

import gzip
import math
import os
import random

import numpy as np
import pytest

from lens_amd.division import growth_division_minimal
from lens_amd.emitter import ExperimentEmitter, process_path_timeseries_for_csv, save_flat_timeseries
from lens_amd.engine import Experiment

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
BOUNDS = (40, 40)
LOCATIONS = [[0.3, 0.3], [0.5, 0.5]]


def single_agent_config(location):
    """multibody_physics.py:298-318 (location given; the angle is a draw)."""
    width, length = 1, 2
    radius = width / 2
    volume = (length - width) * (math.pi * radius ** 2) + (4 / 3) * math.pi * radius ** 3
    return {'boundary': {'location': [loc * BOUNDS[n] for n, loc in enumerate(location)],
                         'angle': np.random.uniform(0, 2 * math.pi), 'volume': volume, 'length': length,
                         'width': width, 'mass': 1339.0, 'thrust': 0, 'torque': 0}}


def colony_metrics_experiment(invoke=None, columns=False):
    random.seed(1)
    np.random.seed(1)
    ids = ['0', '1']
    processes, topology = {'agents': {}}, {'agents': {}}
    for aid in ids:
        c = growth_division_minimal(aid, growth_rate=0.001)
        processes['agents'][aid] = c['processes']
        topology['agents'][aid] = c['topology']
    initial = {'agents': {aid: single_agent_config(loc) for aid, loc in zip(ids, LOCATIONS)}}
    config = {'processes': processes, 'topology': topology, 'initial_state': initial}
    if invoke is not None:
        config['invoke'] = invoke
    if columns:
        config['agent_columns'] = ('agents',)
    return Experiment(config)


def run_csv(tmp_path, invoke=None, steps=2400, columns=False):
    exp = colony_metrics_experiment(invoke, columns)
    em = ExperimentEmitter(exp, extra={'dimensions': {'depth': 3000.0}})
    em.emit()
    for _ in range(steps):
        exp.update(1.0)
        if invoke is not None and hasattr(invoke, 'flush'):
            invoke.flush()
        em.emit()
    flat = process_path_timeseries_for_csv(em.get_path_timeseries())
    save_flat_timeseries(flat, str(tmp_path), 'colony_metrics.csv')
    return open(os.path.join(str(tmp_path), 'colony_metrics.csv'), 'rb').read(), exp


def assert_same_csv(got, want):
    if got != want:
        import csv
        import io
        g = list(csv.reader(io.StringIO(got.decode())))
        w = list(csv.reader(io.StringIO(want.decode())))
        assert g[0] == w[0], ('header', [h for h in w[0] if h not in g[0]][:5], [h for h in g[0] if h not in w[0]][:5])
        for i, (a, b) in enumerate(zip(g, w)):
            assert a == b, ('row', i, [(h, x, y) for h, x, y in zip(w[0], a, b) if x != y][:5])
        assert len(g) == len(w)
    assert got == want


@pytest.mark.parametrize('columns', [False, True])
def test_process_api_loop_rebuilds_colony_metrics_csv_byte_for_byte(tmp_path, columns):
    """Per-agent dicts, and agents held in columns (lens_amd.agent_store)."""
    got, exp = run_csv(tmp_path, columns=columns)
    want = gzip.open(os.path.join(GOLDEN, 'colony_metrics.csv.gz'), 'rb').read()
    assert_same_csv(got, want)
    assert len(exp.state['agents']) > 2                  # the colony divided
    # the deleted mothers left no cache entries behind
    live = set(exp.state['agents'])
    assert all(p[1] in live for p in exp._emit_paths if len(p) > 1 and p[0] == 'agents')


@pytest.mark.gpu
def test_process_api_loop_with_batched_invoke_rebuilds_colony_metrics_csv(tmp_path):
    """The same loop with the reference's `invoke` hook set to BatchedInvoke (the
    GPU batching front end; these processes are host processes and pass
    through it in the reference's order)."""
    torch = pytest.importorskip('torch')
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from lens_amd.invoke import BatchedInvoke
    got, _ = run_csv(tmp_path, invoke=BatchedInvoke(device=torch.device('cuda', 0)))
    want = gzip.open(os.path.join(GOLDEN, 'colony_metrics.csv.gz'), 'rb').read()
    assert_same_csv(got, want)

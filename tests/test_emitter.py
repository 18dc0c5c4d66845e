"""Emitter wire format: raw data -> timeseries -> CSV exactly
as the reference's tooling lays it out, and -- end to end on the GPU -- the
reference's colony_metrics.csv rebuilt byte for byte from a device colony."""

import csv
import gzip
import io
import os

import numpy as np
import pytest

from lens_amd.emitter import (path_timeseries_from_data, process_path_timeseries_for_csv,
                              save_flat_timeseries, timeseries_from_data)

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def test_timeseries_and_csv_layout(tmp_path):
    data = {0.0: {'agents': {'a': {'boundary': {'mass': 1.5}}}, 'dimensions': {'depth': 3.0}},
            1.0: {'agents': {'a': {'boundary': {'mass': 2.5}}, 'b': {'boundary': {'mass': 7.0}}},
                  'dimensions': {'depth': 3.0}}}
    ts = timeseries_from_data(data)
    assert ts['agents']['a']['boundary']['mass'] == [1.5, 2.5]
    assert ts['agents']['b']['boundary']['mass'] == [7.0]
    assert ts['time'] == [0.0, 1.0]
    path = path_timeseries_from_data(data)
    flat = process_path_timeseries_for_csv(path)
    assert list(flat) == ['agents,a,boundary,mass', 'agents,b,boundary,mass', 'dimensions,depth', 'time']
    save_flat_timeseries(flat, str(tmp_path), 'x.csv')
    rows = list(csv.reader(open(tmp_path / 'x.csv')))
    # later-born agents' columns are padded from row 0 (vivarium/library/timeseries.py:53-69)
    assert rows[1] == ['1.5', '7.0', '3.0', '0.0'] and rows[2] == ['2.5', '', '3.0', '1.0']


torch = pytest.importorskip('torch')


@pytest.mark.gpu
def test_gpu_colony_rebuilds_reference_csv_byte_for_byte(tmp_path):
    """2 growth_division_minimal agents on the device, emitted every step through
    ColonyEmitter -> the reference's transforms -> CSV == reference_data/colony_metrics.csv."""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from lens_amd import configs
    from lens_amd.cells import CellModel
    from lens_amd.colony import Colony
    from lens_amd.emitter import ColonyEmitter
    dev = torch.device('cuda', 0)
    cm = CellModel(model='growth_protein', growth_rate=0.001, rng='stream', seed=1, setup_draws=2)
    col = Colony(configs.toy_config(), 2, device=dev, integrator='euler', cells=cm, agent_ids=['0', '1'])
    em = ColonyEmitter(col, species=[], cell_variables=['mass', 'volume', 'width', 'length', 'surface_area',
                                                         'protein'],
                       extra={'dimensions': {'depth': 3000.0}})
    em.emit()
    for _ in range(2400):
        col.step(1.0)
        em.emit()
    flat = process_path_timeseries_for_csv(em.get_path_timeseries())
    save_flat_timeseries(flat, str(tmp_path), 'colony_metrics.csv')
    got = open(tmp_path / 'colony_metrics.csv', 'rb').read()
    want = gzip.open(os.path.join(GOLDEN, 'colony_metrics.csv.gz'), 'rb').read()
    if got != want:
        g = list(csv.reader(io.StringIO(got.decode())))
        w = list(csv.reader(io.StringIO(want.decode())))
        assert g[0] == w[0], 'header'
        for i, (a, b) in enumerate(zip(g, w)):
            assert a == b, ('row', i, [(h, x, y) for h, x, y in zip(w[0], a, b) if x != y][:5])
        assert len(g) == len(w)
    assert got == want

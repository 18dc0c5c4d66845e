"""Emitter wire format for a device-resident colony.

The reference emits the whole Store tree every step (``Experiment.emit_data``,
vivarium/core/experiment.py:1328-1336) into an emitter; the in-memory
``TimeSeriesEmitter`` (vivarium/core/emitter.py:150-164) keeps
``{time: raw_data}`` and the analysis / golden-test tooling turns that into
timeseries (``timeseries_from_data``, ``path_timeseries_from_data``, :87-119),
then into CSV (``process_path_timeseries_for_csv`` + ``save_flat_timeseries``,
vivarium/library/timeseries.py:7-69) -- the format of the reference's
``reference_data/*.csv`` fixtures.

:class:`ColonyEmitter` produces exactly that raw data from the colony's SoA
rows, decimated (``emit_step``) and only for the requested variables, so the
reference's own plotting / comparison tools read our output unchanged.  The
device->host copy is the only cost; nothing is emitted inside the timed loop
unless the caller asks for it.
"""

from __future__ import annotations

import csv
import os
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

from lens_amd import native

# colony variable -> (store path under the agent, SoA source)
CELL_VARIABLES = {
    'mass': ('boundary', native.VK_CELL_MASS), 'volume': ('boundary', native.VK_CELL_VOLUME),
    'length': ('boundary', native.VK_CELL_LENGTH), 'surface_area': ('boundary', native.VK_CELL_SURFACE_AREA),
    'protein': ('internal', native.VK_CELL_PROTEIN),
}


class ColonyEmitter:
    """Collects ``{time: {'agents': {agent_id: {port: {variable: value}}}}}``.

    ``species``: (port, name) keys of the kinetics table to emit (default:
    every species); ``cell_variables``: names from :data:`CELL_VARIABLES`
    (plus ``'width'``) when the colony has a CellModel; ``boundary_port``:
    the store the cell variables live in (``'boundary'`` in the reference's
    lattice agents).  ``extra``: constant top-level entries emitted at every
    time (e.g. ``{'dimensions': {'depth': 3.0}}``)."""

    def __init__(self, colony, species: Optional[Iterable[Tuple[str, str]]] = None,
                 cell_variables: Optional[Iterable[str]] = None, emit_step: int = 1, extra=None):
        self.colony = colony
        t = colony.table
        self.species = list(t.species) if species is None else [tuple(k) for k in species]
        self.rows = [t.species.index(k) for k in self.species]
        self.cell_variables = list(cell_variables or [])
        self.emit_step = int(emit_step)
        self.extra = extra or {}
        self.saved_data: Dict[float, dict] = {}
        self._calls = 0

    def emit(self, time: Optional[float] = None):
        """Record the colony's state (every ``emit_step``-th call)."""
        self._calls += 1
        if (self._calls - 1) % self.emit_step:
            return
        col = self.colony
        time = col.time if time is None else time
        n = col.n
        conc = col.conc[self.rows, :n].cpu().numpy() if self.rows else np.zeros((0, n))
        cell = col.cell[:, :n].cpu().numpy() if self.cell_variables else None
        ids = col.agent_ids()
        agents = {}
        for a, aid in enumerate(ids):
            d: Dict[str, Dict[str, float]] = {}
            for (port, name), v in zip(self.species, conc[:, a]):
                d.setdefault(port, {})[name] = float(v)
            for var in self.cell_variables:
                if var == 'width':
                    d.setdefault('boundary', {})['width'] = col.cells.width
                    continue
                port, row = CELL_VARIABLES[var]
                d.setdefault(port, {})[var] = float(cell[row, a])
            agents[aid] = d
        data = {'agents': agents}
        data.update(self.extra)
        self.saved_data[time] = data

    def get_data(self):
        return self.saved_data

    def get_timeseries(self):
        return timeseries_from_data(self.saved_data)

    def get_path_timeseries(self):
        return path_timeseries_from_data(self.saved_data)


class ExperimentEmitter:
    """The in-memory timeseries emitter of the Process-API loop
    (:class:`lens_amd.engine.Experiment`): ``emit()`` records
    ``{time: experiment.emit_data() + extra}`` (Experiment.emit_data,
    vivarium/core/experiment.py:1328-1336; TimeSeriesEmitter, emitter.py:150-164)."""

    def __init__(self, experiment, extra=None):
        self.experiment = experiment
        self.extra = extra or {}
        self.saved_data: Dict[float, dict] = {}

    def emit(self, time: Optional[float] = None):
        data = self.experiment.emit_data()
        data.update(self.extra)
        self.saved_data[self.experiment.local_time if time is None else time] = data

    def get_data(self):
        return self.saved_data

    def get_path_timeseries(self):
        return path_timeseries_from_data(self.saved_data)


# ---------------------------------------------------------------------------
# the reference's raw-data -> timeseries -> CSV transforms (restated)
# ---------------------------------------------------------------------------

def _value_in_embedded_dict(data, timeseries):
    """vivarium/library/dict_utils.py:166-186 (time_index=None form)."""
    for key, value in data.items():
        if isinstance(value, dict):
            timeseries[key] = _value_in_embedded_dict(value, timeseries.get(key, {}))
        else:
            timeseries.setdefault(key, []).append(value)
    return timeseries


def timeseries_from_data(data):
    """vivarium/core/emitter.py:109-119."""
    embedded = {}
    for time, value in data.items():
        if isinstance(value, dict):
            embedded = _value_in_embedded_dict(value, embedded)
    embedded['time'] = list(data.keys())
    return embedded


def _path_dict(embedded, prefix=()):
    out = {}
    for key, value in embedded.items():
        if isinstance(value, dict):
            out.update(_path_dict(value, prefix + (key,)))
        else:
            out[prefix + (key,)] = value
    return out


def path_timeseries_from_data(data):
    """vivarium/core/emitter.py:87-95: {path tuple: [values]} + 'time'."""
    embedded = timeseries_from_data(data)
    times = embedded.pop('time')
    out = _path_dict(embedded)
    out['time'] = times
    return out


def process_path_timeseries_for_csv(path_ts):
    """vivarium/library/timeseries.py:7-51: tuple keys joined with ',', non-numeric dropped.

    This and :func:`save_flat_timeseries` restate the reference's helpers nearly
    line for line on purpose: they define the CSV wire format (key joining,
    which columns are dropped, row padding), and the GPU colony must rebuild
    ``reference_data/colony_metrics.csv`` byte for byte (tests/test_emitter.py)."""
    str_keys = {}
    for key, value in path_ts.items():
        if not isinstance(key, str):
            key = ','.join(key)
        str_keys[key] = value
    remove = [k for k, v in str_keys.items() if isinstance(v[0], list)]
    for k, v in str_keys.items():
        try:
            float(v[0])
        except (ValueError, TypeError):
            remove.append(k)
    for k in set(remove):
        del str_keys[k]
    return str_keys


def save_flat_timeseries(timeseries, out_dir, filename):
    """vivarium/library/timeseries.py:53-69: one column per key, rows padded from row 0."""
    n_rows = max(len(v) for v in timeseries.values())
    rows = [{} for _ in range(n_rows)]
    for key, val in timeseries.items():
        for i, elem in enumerate(val):
            rows[i][key] = elem
    with open(os.path.join(out_dir, filename), 'w') as f:
        writer = csv.DictWriter(f, timeseries.keys(), delimiter=',')
        writer.writeheader()
        writer.writerows(rows)

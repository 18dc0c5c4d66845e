"""Process-API drop-in: ``BatchedConvenienceKinetics``.

Same ``name``, ``defaults``, ``ports_schema``, ``derivers`` and
``next_update(timestep, states)`` contract as the reference
``ConvenienceKinetics`` (vivarium/processes/convenience_kinetics.py:56-352),
so it can replace it inside any Compartment / Experiment unchanged.  The
update dict it returns is the reference's, key for key:

* ``fluxes``: ``{reaction_id: flux}`` (updater ``set``),
* per non-external port: ``{state: delta}`` accumulated in the reference's
  order (``0 + sum_r coeff*flux*timestep``),
* ``fields``: ``{mol: {'_value': int count, '_updater': {'updater':
  'update_field_with_exchange', 'port_mapping': {...}}}}``.

The arithmetic runs on the GPU (``vk_step_euler`` through the C ABI).  A
single ``next_update`` call is a batch of one; :class:`lens_amd.invoke.
BatchedInvoke` gathers every agent's call of a timestep into one launch.

When the reference package is importable (its own Python 3.6-3.8
environment) the class derives from ``vivarium.core.process.Process`` and
registers in its ``process_registry``; otherwise from :class:`Process`
below, a restatement of that base class (vivarium/core/process.py:201-306).
"""

from __future__ import annotations

import copy
import hashlib
from typing import Any, Dict

import numpy as np

from lens_amd.rate_law_compiler import compile_rate_laws, RateLawTable

DEFAULT_TIME_STEP = 1.0


def deep_merge(dct, merge_dct):
    """vivarium/library/dict_utils.py:51-65 (mutates and returns dct)."""
    if dct is None:
        dct = {}
    if merge_dct is None:
        merge_dct = {}
    for k, v in merge_dct.items():
        if k in dct and isinstance(dct[k], dict) and isinstance(v, dict):
            deep_merge(dct[k], v)
        else:
            dct[k] = v
    return dct


class Process:
    """Restatement of vivarium.core.process.Process (process.py:201-306)."""

    defaults: Dict[str, Any] = {}
    registry: Dict[str, type] = {}

    def __init__(self, parameters=None):
        assert hasattr(self, 'name')
        if parameters is None:
            parameters = {}
        self.parameters = copy.deepcopy(self.defaults)
        self.config = {}
        self.schema_override = {}
        if '_schema' in parameters:
            self.schema_override = parameters.pop('_schema')
        self.parallel = False
        if '_parallel' in parameters:
            self.parallel = parameters.pop('_parallel')
        deep_merge(self.parameters, parameters)
        Process.registry.setdefault(self.name, type(self))

    def local_timestep(self):
        return self.parameters.get('time_step', DEFAULT_TIME_STEP)

    def ports(self):
        return {port: list(states.keys()) for port, states in self.ports_schema().items()}

    def default_state(self):
        state = {}
        for port, states in self.ports_schema().items():
            for key, value in states.items():
                if '_default' in value:
                    state.setdefault(port, {})[key] = value['_default']
        return state

    def is_deriver(self):
        return False

    def derivers(self):
        return {}

    def ports_schema(self):
        return {}

    def next_update(self, timestep, states):
        return {port: {} for port in self.ports()}


try:  # the reference's own environment: be a real vivarium Process
    from vivarium.core.process import Process as _VivariumProcess  # type: ignore
    ProcessBase = _VivariumProcess
except Exception:  # pragma: no cover - the reference is not installed here
    ProcessBase = Process


def _magnitude(x):
    """units.remove_units for a scalar (vivarium/library/units.py:37-65)."""
    return getattr(x, 'magnitude', x)


def table_signature(table: RateLawTable) -> str:
    """Processes whose compiled tables are structurally identical share one batch."""
    h = hashlib.sha1()
    h.update(repr((table.species, table.n_dyn, table.reaction_ids, table.external_ids,
                   table.param_names and [p[0] for p in table.param_names])).encode())
    for name, arr in table.arrays().items():
        h.update(name.encode())
        h.update(np.ascontiguousarray(arr).tobytes())
    return h.hexdigest()


class BatchedConvenienceKinetics(ProcessBase):
    """GPU-batched drop-in for ``ConvenienceKinetics``."""

    name = 'convenience_kinetics'
    defaults = {
        'reactions': {},
        'initial_state': {'internal': {}, 'external': {}},
        'kinetic_parameters': {},
        'port_ids': ['internal', 'external'],
        'added_port_ids': ['fluxes', 'fields', 'global'],
        'global_deriver_key': 'global_deriver',
    }

    def __init__(self, parameters=None):
        super().__init__(parameters)
        self.reactions = self.parameters['reactions']
        self.initial_state = self.parameters['initial_state']
        self.kinetic_parameters = self.parameters['kinetic_parameters']
        self.port_ids = self.parameters['port_ids'] + self.parameters['added_port_ids']
        self.table = compile_rate_laws(self.reactions, self.kinetic_parameters, self.port_ids)
        self.signature = table_signature(self.table)
        self.param_values = self.table.param_defaults.copy()

    # -- schema: convenience_kinetics.py:240-301 --------------------------------
    def ports_schema(self):
        schema = {port_id: {} for port_id in self.port_ids}
        for port, states in self.initial_state.items():
            for state_id in states:
                schema.setdefault(port, {})[state_id] = {
                    '_default': self.initial_state[port][state_id], '_emit': True}
        if 'external' in schema:
            schema['fields'] = {state_id: {'_default': np.ones((1, 1))}
                                for state_id in schema['external'].keys()}
        for rid in self.table.reaction_ids:
            schema['fluxes'][rid] = {'_default': 0.0, '_emit': False, '_updater': 'set'}
        schema['global'] = {
            'mmol_to_counts': {'_default': 0.0, '_emit': False},
            'location': {'_default': [0.5, 0.5]},
        }
        schema['dimensions'] = {
            'bounds': {'_default': [1, 1]},
            'n_bins': {'_default': [1, 1]},
            'depth': {'_default': 1},
        }
        return schema

    def derivers(self):
        return {
            self.parameters['global_deriver_key']: {
                'deriver': 'globals_deriver',
                'port_mapping': {'global': 'global'},
                'config': {'width': 1.0}}}

    # -- packing helpers shared with BatchedInvoke ----------------------------
    def pack_state(self, states):
        """One agent's species values (table order) and its mmol_to_counts, as
        Python floats."""
        groups = self.__dict__.get('_pack_groups')
        if groups is None:          # species grouped by port, in table order within each
            by_port = {}
            for i, (port, name) in enumerate(self.table.species):
                by_port.setdefault(port, []).append((i, name))
            groups = self._pack_groups = list(by_port.items())
            self._n_species = len(self.table.species)
        vals = [0.0] * self._n_species
        for port, members in groups:
            d = states.get(port)
            if isinstance(d, dict):
                get = d.get
                for i, name in members:
                    v = get(name, 0.0)
                    vals[i] = v if type(v) is float else float(getattr(v, 'magnitude', v))
        return vals, float(_magnitude(states['global']['mmol_to_counts']))

    def unpack_update(self, fluxes, deltas, counts):
        """Device outputs of one agent (sequences in table order) -> the
        reference's update dict (convenience_kinetics.py:316-349).  The inline
        ``_updater`` spec of the exchange is one shared, read-only dict."""
        t = self.table
        spec = self.__dict__.get('_exchange_spec')
        if spec is None:
            spec = self._exchange_spec = {
                'updater': 'update_field_with_exchange',
                'port_mapping': {'global': 'global', 'dimensions': 'dimensions'}}
            self._dyn_keys = t.species[:t.n_dyn]
        update = {port: {} for port in self.port_ids}
        update['fluxes'] = dict(zip(t.reaction_ids, map(np.float64, fluxes)))
        for (port, name), d in zip(self._dyn_keys, deltas):
            update.setdefault(port, {})[name] = d
        fields = update['fields']
        for mol, c in zip(t.external_ids, counts):
            fields[mol] = {'_value': c, '_updater': spec}
        return update

    def next_update(self, timestep, states):
        from lens_amd.invoke import run_batch
        return run_batch([(self, timestep, states)])[0]


# ---------------------------------------------------------------------------
# the environment side: DiffusionField drop-in and the batched exchange updater
# ---------------------------------------------------------------------------

def _bin_sites(locations, n_bins, bounds):
    """get_bin_site (vivarium/library/lattice_utils.py:34-40) for many agents: linear bins."""
    loc = np.asarray(locations, dtype=np.float64).reshape(-1, 2)
    i = np.mod(np.floor(loc[:, 0] * n_bins[0] / bounds[0]).astype(np.int64), n_bins[0])
    j = np.mod(np.floor(loc[:, 1] * n_bins[1] / bounds[1]).astype(np.int64), n_bins[1])
    return i * n_bins[1] + j


class AgentLeafUpdate:
    """An update that sets the same leaves under every agent -- ``rest`` (the
    update's other ports) plus, per agent id, ``agents[id][path...][key] = row[i]``
    -- kept as columns.  ``as_dict()`` spells it out as the reference's nested
    update dict; lens_amd.engine.Experiment applies it directly."""

    __slots__ = ('rest', 'ids', 'path', 'keys', 'rows')

    def __init__(self, rest, ids, path, keys, rows):
        self.rest, self.ids, self.path, self.keys, self.rows = rest, ids, tuple(path), keys, rows

    def as_dict(self):
        update = dict(self.rest)
        if self.ids:
            agents = {}
            for a, row in zip(self.ids, self.rows):
                leaf = dict(zip(self.keys, row))
                for k in reversed(self.path):
                    leaf = {k: leaf}
                agents[a] = leaf
            update['agents'] = agents
        return update


class BatchedDiffusionField(ProcessBase):
    """GPU drop-in for ``DiffusionField`` (vivarium/processes/diffusion_field.py:209-407).

    Same ``name``, ``defaults``, ``ports_schema`` and ``next_update``; the
    fields live on the GPU -- the ``fields`` store holds
    :class:`lens_amd.registry.DeviceField` values -- the delta of
    ``diffusion_delta`` (100 / 501 / 1001 substeps for dt = 1 / 5 / 10 s,
    uniform fields skipped) comes from ``vk_diffuse_delta`` and every agent's
    ``boundary.external`` from one ``vk_gather`` of the pre-step fields at the
    agents' bins.  The agents' ``update_field_with_exchange`` updates on those
    fields queue on the field and land in one agent-ordered launch
    (:mod:`lens_amd.registry`, bound into the reference's updater registry or
    :class:`lens_amd.engine.Experiment`)."""

    name = 'diffusion_field'
    defaults = {
        'time_step': 1,
        'molecules': ['glc'],
        'initial_state': {},
        'n_bins': [10, 10],
        'bounds': [10, 10],
        'depth': 3000.0,
        'diffusion': 5e-1,
        'gradient': {},
        'agents': {},
        'avogadro': 6.022140857e23,
    }

    def __init__(self, parameters=None):
        super().__init__(parameters)
        import torch
        from lens_amd import native
        from lens_amd.lattice import Lattice
        p = self.parameters
        self.molecule_ids = list(p['molecules'])
        self.n_bins = [int(p['n_bins'][0]), int(p['n_bins'][1])]
        self.bounds = [float(p['bounds'][0]), float(p['bounds'][1])]
        self.device = native.resolve_device(p.get('device'))
        self.lattice = Lattice(self.molecule_ids, self.n_bins, self.bounds, float(p['depth']), p['diffusion'],
                               device=self.device, avogadro=p['avogadro'])
        self.initial_agents = p['agents']
        self._torch = torch
        nf = len(self.molecule_ids)
        self._map = torch.arange(nf, dtype=torch.int32, device=self.device)   # plane f -> row f

    def ones_field(self):
        return self._torch.ones(self.n_bins, dtype=self._torch.float64, device=self.device)

    def _device_field(self, value):
        from lens_amd.registry import as_device_tensor
        return as_device_tensor(value, self.device).contiguous()

    def ports_schema(self):
        from lens_amd.registry import DeviceField
        local = {m: {'_default': 0.0, '_updater': 'set'} for m in self.molecule_ids}
        schema = {'agents': {}}
        for agent_id, states in self.initial_agents.items():
            schema['agents'][agent_id] = {'boundary': {'location': {'_value': states['boundary'].get('location', [])}}}
        schema['agents']['*'] = {'boundary': {
            'location': {'_default': [0.5 * b for b in self.bounds], '_updater': 'set'},
            'external': local}}
        init = self.parameters['initial_state']
        schema['fields'] = {
            m: {'_value': DeviceField(self._device_field(init[m]) if m in init else self.ones_field()),
                '_updater': 'accumulate', '_emit': True}
            for m in self.molecule_ids}
        schema['dimensions'] = {
            k: {'_value': self.parameters[k], '_updater': 'set', '_emit': True} for k in ('bounds', 'n_bins', 'depth')}
        return schema

    def next_update_raw(self, timestep, states):
        """:meth:`next_update`'s update before it is spelled out per agent: an
        :class:`AgentLeafUpdate` (lens_amd.engine.Experiment applies it without
        building one dict per agent; ``as_dict()`` is the reference's update)."""
        from lens_amd import native
        torch = self._torch
        fields = states['fields']
        lat = self.lattice
        with torch.cuda.device(self.device):
            for f, m in enumerate(self.molecule_ids):
                lat.fields[f].copy_(self._device_field(fields[m]))     # lands queued exchange first
            update = {}
            agents = states['agents']
            if agents:
                # pre-step fields at the agents' bins (get_local_environments,
                # diffusion_field.py:362-379): one vk_gather, one host copy
                ids = list(agents)
                n = len(ids)
                values_at = getattr(agents, 'values_at', None)      # columnar agents: one column read
                locs = (values_at(('boundary', 'location'), ids) if values_at is not None else
                        [agents[a]['boundary']['location'] for a in ids])
                bins = torch.from_numpy(_bin_sites(locs, self.n_bins, self.bounds).astype(np.int32)).to(self.device)
                vals = torch.empty((len(self.molecule_ids), n), dtype=torch.float64, device=self.device)
                native.check(native._lib.vk_gather(
                    native.ptr(lat.fields), lat.field_stride, native.ptr(bins), n, native.ptr(self._map),
                    native.ptr(self._map), int(self._map.numel()), native.ptr(vals), n, native.stream_handle()),
                    'vk_gather')
            delta = lat.diffuse_delta(timestep)
            update['fields'] = {m: delta[f] for f, m in enumerate(self.molecule_ids)}
            raw = AgentLeafUpdate(update, ids if agents else [], ('boundary', 'external'), list(self.molecule_ids),
                                  vals.cpu().numpy().T.tolist() if agents else [])
        return raw

    def next_update(self, timestep, states):
        return self.next_update_raw(timestep, states).as_dict()

"""Oracle (TEST INFRASTRUCTURE ONLY): the reference's multi-rate Experiment loop.

A literal restatement, over nested dicts instead of Store objects, of
  * Experiment.update ........ vivarium/core/experiment.py:1351-1450
    (per-process fronts; a process runs when its front time <= time, with
    timestep = min(front + local_timestep, interval) - front; the global
    step is the smallest timestep that ran; updates whose front lands by
    then are applied in front (first-appearance, depth-first) order; the
    derivers run after every applied step; the no-process-ran jump keeps
    the reference's use of the last loop path, :1414-1419)
  * send_updates / run_derivers (derivers with timestep 0) ... :1319-1349
  * Experiment.__init__'s initial deriver pass ................. :1247
  * Store.apply_update for value updates: branches recurse, leaves apply
    their schema updater or an inline {'_value', '_updater'} one, with a
    port_mapping state for update_field_with_exchange ........... :586-739
  * updaters accumulate / set / update_field_with_exchange .... vivarium/core/registry.py:117-183
  * topology paths relative to the process's parent, '..' steps up
    (normalize_path, experiment.py:1123-1130)
  * structural updates at a branch, in Store.apply_update's order
    (:628-697): _delete, _add, _generate (Store.generate :1017-1029) and
    _divide (the mother's values deep-copied, Store.divide_value :512-534
    with the schema's _divider per leaf -- registry.py:197-280 -- merged in
    per daughter, daughters generated in order at the end of the branch, the
    mother deleted, Store.delete_path :494-510); the loop walks the process
    tree every iteration (:1373-1391) and skips derivers deleted earlier in
    the same pass (:1321-1327)
Processes are invoked immediately (InvokeProcess, :1157-1167).  A '*' key in
a ports schema applies to every child of that store (DiffusionField's
agents schema, diffusion_field.py:292-302).
"""

from __future__ import annotations

import copy
import math
import random

import numpy as np

from oracle.kinetics import N_A_LEGACY, bin_site, bin_volume_L, count_to_mM

INFINITY = float('inf')


def normalize_path(path):
    progress = []
    for step in path:
        if step == '..' and progress:
            progress = progress[:-1]
        else:
            progress.append(step)
    return tuple(progress)


def update_accumulate(current, new, states):
    return current + new


def update_set(current, new, states):
    return new


def divide_set(state):
    return [state, state]


def divide_split(state):
    if isinstance(state, (int, np.integer)) and not isinstance(state, bool):
        remainder = state % 2
        half = int(state / 2)
        if random.choice([True, False]):
            return [half + remainder, half]
        else:
            return [half, half + remainder]
    elif state == float('inf') or state == 'Infinity':
        return [state, state]
    elif isinstance(state, (float, np.floating)):
        half = state / 2
        return [half, half]
    raise Exception('can not divide state {} of type {}'.format(state, type(state)))


def divide_zero(state):
    return [0, 0]


def divide_split_dict(state):
    if state is None:
        state = {}
    d1 = dict(list(state.items())[len(state) // 2:])
    d2 = dict(list(state.items())[:len(state) // 2])
    return [d1, d2]


DIVIDERS = {'set': divide_set, 'split': divide_split, 'split_dict': divide_split_dict, 'zero': divide_zero}


def dict_merge(dct, merge_dct):
    """vivarium/library/dict_utils.py deep_merge (mutates dct)."""
    for k, v in merge_dct.items():
        if k in dct and isinstance(dct[k], dict) and isinstance(v, dict):
            dict_merge(dct[k], v)
        else:
            dct[k] = v
    return dct


def make_update_field_with_exchange(avogadro=N_A_LEGACY):
    def update_field_with_exchange(current, new, states):
        location = states['global']['location']
        dims = states['dimensions']
        delta = np.zeros((dims['n_bins'][0], dims['n_bins'][1]), dtype=np.float64)
        i, j = bin_site(location, dims['n_bins'], dims['bounds'])
        delta[i, j] += count_to_mM(new, bin_volume_L(dims['n_bins'], dims['bounds'], dims['depth']), avogadro)
        return current + delta
    return update_field_with_exchange


class OracleExperiment:
    def __init__(self, processes, topology, initial_state, avogadro=N_A_LEGACY, updater_registry=None):
        """``updater_registry``: entries that replace the reference's updaters by
        name, as a maintainer replaces one in vivarium.core.registry.updater_registry
        (tests bind the device-aware update_field_with_exchange this way)."""
        self.processes = processes
        self.topology = topology
        self.state = _copy_tree(initial_state)
        self.updaters = {'accumulate': update_accumulate, 'set': update_set,
                         'update_field_with_exchange': make_update_field_with_exchange(avogadro)}
        self.updaters.update(updater_registry or {})
        self.schema = {}                      # store path (with '*' globs) -> updater name
        self._globs = []                      # the schema paths holding a '*'
        self.dividers = {}                    # store path (with '*' globs) -> _divider
        self.deleted = {}                     # processes removed during the current pass, by id (held)
        self.local_time = 0.0
        for path, proc in self._walk(processes, ()):
            for port, port_schema in proc.ports_schema().items():
                self._register(self.port_path(path, port), port_schema)
        self.send_updates([])                 # the derivers run once at t = 0

    # -- tree ------------------------------------------------------------------
    def _walk(self, node, path):
        out = []
        for key, value in node.items():
            if isinstance(value, dict):
                out += self._walk(value, path + (key,))
            else:
                out.append((path + (key,), value))
        return out

    def _topology_of(self, path):
        t = self.topology
        for key in path:
            t = t[key]
        return t

    def port_path(self, proc_path, port):
        return normalize_path(proc_path[:-1] + tuple(self._topology_of(proc_path)[port]))

    def get(self, path):
        v = self.state
        for key in path:
            v = v[key]
        return v

    def _register(self, path, schema):
        if not isinstance(schema, dict):
            return
        keys = [k for k in schema if not k.startswith('_')]
        if ('_default' in schema or '_value' in schema or '_updater' in schema or '_divider' in schema) and not keys:
            if '_updater' in schema:           # a schema without one keeps the store's updater
                self.schema.setdefault(path, schema['_updater'])
                if '*' in path and path not in self._globs:
                    self._globs.append(path)
            if '_divider' in schema:
                self.dividers.setdefault(path, schema['_divider'])
            if '*' not in path:
                node = self.state
                for key in path[:-1]:
                    node = node.setdefault(key, {})
                if path[-1] not in node:
                    node[path[-1]] = schema.get('_value', schema.get('_default'))
            return
        for k in keys:
            self._register(path + (k,), schema[k])

    def _updater_at(self, path):
        if path in self.schema:
            return self.schema[path]
        for pat in self._globs:                  # '*' patterns, in registration order
            if len(pat) == len(path) and all(p == '*' or p == q for p, q in zip(pat, path)):
                return self.schema[pat]
        return 'accumulate'

    # -- updates -------------------------------------------------------------
    def process_states(self, path, proc):
        return {port: self.get(self.port_path(path, port)) for port in proc.ports_schema()}

    def apply_update(self, update, proc_path):
        for port, value in update.items():
            self._apply(self.port_path(proc_path, port), value, proc_path)

    def _lookup(self, path):
        node = self.state
        for key in path:
            if not isinstance(node, dict) or key not in node:
                return None
            node = node[key]
        return node

    def _apply(self, path, update, proc_path):
        # Store.apply_update descends only into keys `inner` holds (experiment.py:699-711):
        # an update below a missing key (e.g. an agent deleted earlier in the same
        # batch) is dropped
        parent = self._lookup(path[:-1])
        if not isinstance(parent, dict) or path[-1] not in parent:
            return
        current = parent[path[-1]]
        inline = isinstance(update, dict) and '_updater' in update
        if isinstance(current, dict) and not inline:
            if '_delete' in update:
                for p in update['_delete']:
                    self.delete_path(path + tuple(p))
            if '_add' in update:
                for added in update['_add']:
                    target = normalize_path(path + tuple(added['path']))
                    node = self.state
                    for key in target[:-1]:
                        node = node.setdefault(key, {})
                    if isinstance(node.get(target[-1]), dict):
                        self.set_value(node[target[-1]], added['state'])
                    else:
                        node[target[-1]] = copy.deepcopy(added['state'])
            if '_generate' in update:
                for g in update['_generate']:
                    self.generate(path + tuple(g['path']), g['processes'], g['topology'], g['initial_state'])
            if '_divide' in update:
                divide = update['_divide']
                mother = divide['mother']
                mother_state = self.get(path + (mother,))
                initial_state = copy.deepcopy(mother_state)
                states = self.divide_value(path + (mother,), mother_state)
                for daughter, state in zip(divide['daughters'], states):
                    initial_state = dict_merge(initial_state, state)
                    self.generate(path + tuple(daughter['path']), daughter['processes'], daughter['topology'],
                                  daughter['initial_state'])
                    self.set_value(self.get(path + (daughter['daughter'],)), copy.deepcopy(initial_state))
                self.delete_path(path + (mother,))
            for key, value in update.items():
                if key in ('_delete', '_add', '_generate', '_divide'):
                    continue
                self._apply(path + (key,), value, proc_path)
            return
        states = None
        if inline:
            spec = update['_updater']
            name, mapping = (spec, None) if isinstance(spec, str) else (spec['updater'], spec.get('port_mapping'))
            value = update.get('_value')
            if mapping is not None:
                states = {up: self.get(self.port_path(proc_path, pp)) for up, pp in mapping.items()}
        else:
            name, value = self._updater_at(path), update
        parent[path[-1]] = self.updaters[name](current, value, states)

    # -- structure ----------------------------------------------------------------
    def set_value(self, node, value):
        """Store.set_value: values for keys the tree holds; others ignored."""
        for k, v in value.items():
            if k in node:
                if isinstance(node[k], dict) and isinstance(v, dict):
                    self.set_value(node[k], v)
                else:
                    node[k] = v

    def generate(self, target, processes, topology, initial_state):
        target = normalize_path(target)
        node = self.state
        for key in target:
            node = node.setdefault(key, {})
        pnode, tnode = self.processes, self.topology
        for key in target[:-1]:
            pnode = pnode.setdefault(key, {})
            tnode = tnode.setdefault(key, {})
        pnode.setdefault(target[-1], {}).update(processes)
        tnode.setdefault(target[-1], {}).update(topology)
        for ppath, proc in self._walk(processes, target):
            for port, port_schema in proc.ports_schema().items():
                self._register(self.port_path(ppath, port), port_schema)
        self.set_value(node, initial_state or {})

    def delete_path(self, path):
        parent = self.get(path[:-1])
        if path[-1] in parent:
            del parent[path[-1]]
        pnode = self.processes
        for key in path[:-1]:
            pnode = pnode.get(key, {})
        if path[-1] in pnode:
            lost = pnode.pop(path[-1])
            for _, proc in (self._walk(lost, ()) if isinstance(lost, dict) else [((), lost)]):
                self.deleted[id(proc)] = proc      # held: a new process must not reuse the id

    def divider_at(self, path):
        if path in self.dividers:
            return self.dividers[path]
        for pat, div in self.dividers.items():
            if '*' in pat and len(pat) == len(path) and all(p == '*' or p == q for p, q in zip(pat, path)):
                return div
        return None

    def divide_value(self, path, node):
        div = self.divider_at(path)
        if div:
            if isinstance(div, dict):
                states = {k: self.get(normalize_path(path[:-1] + tuple(p))) for k, p in div['topology'].items()}
                return div['divider'](node, states)
            return (DIVIDERS[div] if isinstance(div, str) else div)(node)
        if isinstance(node, dict):
            daughters = [{}, {}]
            for key, child in node.items():
                division = self.divide_value(path + (key,), child)
                if division:
                    for daughter, divided in zip(daughters, division):
                        daughter[key] = divided
            return daughters
        return None

    def send_updates(self, updates, derivers=None):
        self.deleted = {}                      # processes deleted during this pass
        for update, path in updates:
            self.apply_update(update, path)
        if derivers is None:
            derivers = [(p, s) for p, s in self._walk(self.processes, ()) if s.is_deriver()]
        for path, deriver in derivers:
            if id(deriver) in self.deleted:
                continue
            update = deriver.next_update(0, self.process_states(path, deriver))
            self.apply_update(update, path)

    # -- Experiment.update ---------------------------------------------------
    def update(self, interval):
        time = 0
        front = {}
        while time < interval:
            full_step = INFINITY
            everything = self._walk(self.processes, ())
            processes = [(p, s) for p, s in everything if not s.is_deriver()]
            derivers = [(p, s) for p, s in everything if s.is_deriver()]
            paths = {p for p, _ in processes}
            front = {p: f for p, f in front.items() if p in paths}
            for path, proc in processes:
                if path not in front:
                    front[path] = {'time': time, 'update': {}}
                process_time = front[path]['time']
                if process_time <= time:
                    future = min(process_time + proc.local_timestep(), interval)
                    timestep = future - process_time
                    update = (proc.next_update(timestep, self.process_states(path, proc)), path)
                    if timestep < full_step:
                        full_step = timestep
                    front[path]['time'] = future
                    front[path]['update'] = update
            if full_step == INFINITY:
                next_event = interval
                for _ in front.keys():
                    if front[path]['time'] < next_event:       # the reference's stale `path`
                        next_event = front[path]['time']
                time = next_event
            else:
                future = time + full_step
                updates = []
                for path, advance in front.items():
                    if advance['time'] <= future:
                        updates.append(advance['update'])
                        advance['update'] = {}
                self.send_updates(updates, derivers)
                time = future
                self.local_time += full_step
        return self


def _copy_tree(t):
    if isinstance(t, dict):
        return {k: _copy_tree(v) for k, v in t.items()}
    if isinstance(t, np.ndarray):
        return t.copy()
    if isinstance(t, list):
        return list(t)
    return t


# ---------------------------------------------------------------------------
# oracle processes
# ---------------------------------------------------------------------------

class OracleProcess:
    """The parts of vivarium.core.process.Process (process.py:201-306) the loop uses."""
    defaults = {}

    def __init__(self, parameters=None):
        self.parameters = dict(self.defaults)
        self.parameters.update(parameters or {})

    def local_timestep(self):
        return self.parameters.get('time_step', 1.0)

    def is_deriver(self):
        return False


class OracleConvenienceKinetics(OracleProcess):
    """ConvenienceKinetics (convenience_kinetics.py:240-352) on oracle.kinetics.OracleAgent."""

    def __init__(self, parameters):
        super().__init__(parameters)
        from oracle.kinetics import OracleAgent
        self.agent = OracleAgent(parameters['reactions'], parameters['kinetic_parameters'])
        self.initial_state = parameters.get('initial_state', {})

    def ports_schema(self):
        schema = {port: {} for port in ('internal', 'external', 'fluxes', 'fields', 'global', 'dimensions')}
        for port, states in self.initial_state.items():
            for k, v in states.items():
                schema[port][k] = {'_default': v}
        schema['fields'] = {k: {'_default': np.ones((1, 1))} for k in schema['external']}
        for rid in self.agent.model.reaction_ids:
            schema['fluxes'][rid] = {'_default': 0.0, '_updater': 'set'}
        # convenience_kinetics.py:269-285: declared, so a daughter's store holds them
        # (no divider: each daughter keeps the mother's value)
        schema['global'] = {'mmol_to_counts': {'_default': 0.0}, 'location': {'_default': [0.5, 0.5]}}
        schema['dimensions'] = {'bounds': {'_default': [1, 1]}, 'n_bins': {'_default': [1, 1]},
                                'depth': {'_default': 1}}
        return schema

    def next_update(self, timestep, states):
        st = {p: states[p] for p in ('internal', 'external')}
        m2c = states['global']['mmol_to_counts']
        fluxes, deltas, counts = self.agent.next_update(timestep, st, m2c)
        update = {'fluxes': dict(fluxes), 'internal': deltas['internal']}
        update['fields'] = {mol: {'_value': c, '_updater': {
            'updater': 'update_field_with_exchange',
            'port_mapping': {'global': 'global', 'dimensions': 'dimensions'}}} for mol, c in counts.items()}
        return update


class OracleDiffusionField(OracleProcess):
    """DiffusionField.next_update (diffusion_field.py:280-407): field deltas and each
    agent's external := the pre-step field at its bin."""
    defaults = {'time_step': 1.0}

    def __init__(self, parameters):
        super().__init__(parameters)
        self.molecules = list(parameters['molecules'])
        self.n_bins = list(parameters['n_bins'])
        self.bounds = list(parameters['bounds'])
        self.diffusion = parameters['diffusion']
        self.initial_state = parameters.get('initial_state', {})

    def ports_schema(self):
        return {
            'agents': {'*': {'boundary': {
                'location': {'_default': [0.5 * b for b in self.bounds], '_updater': 'set'},
                'external': {m: {'_default': 0.0, '_updater': 'set'} for m in self.molecules}}}},
            'fields': {m: {'_value': np.array(self.initial_state[m], dtype=np.float64) if m in self.initial_state
                           else np.ones(self.n_bins), '_updater': 'accumulate'} for m in self.molecules},
            'dimensions': {k: {'_value': self.parameters[k], '_updater': 'set'} for k in ('bounds', 'n_bins', 'depth')},
        }

    def next_update(self, timestep, states):
        from oracle.lattice import diffusion_delta
        fields = states['fields']
        update = {'fields': {m: diffusion_delta(fields[m], timestep, self.diffusion, self.n_bins, self.bounds)
                             for m in self.molecules}}
        agents = states['agents']
        if agents:
            update['agents'] = {
                aid: {'boundary': {'external': {
                    m: fields[m][bin_site(spec['boundary']['location'], self.n_bins, self.bounds)]
                    for m in self.molecules}}}
                for aid, spec in agents.items()}
        return update


class OracleNonSpatialEnvironment(OracleProcess):
    """NonSpatialEnvironment (nonspatial_environment.py:14-82): a deriver that sets
    external[mol] := fields[mol][0][0]; 1 x 1 fields of bin volume = volume."""

    def __init__(self, parameters):
        super().__init__(parameters)
        self.volume_L = parameters.get('volume_L', 1e-12)

    def is_deriver(self):
        return True

    def ports_schema(self):
        return {'external': {}, 'fields': {}, 'dimensions': {}, 'global': {}}

    def next_update(self, timestep, states):
        return {'external': {m: {'_updater': 'set', '_value': f[0][0]} for m, f in states['fields'].items()}}


def nonspatial_dimensions(volume_L):
    """The dimensions store NonSpatialEnvironment declares: 1 um x 1 um bins,
    depth = volume / (1 um^2) in um (the expression oracle.kinetics.replay_single_agent
    is pinned with against convenience_kinetics.csv)."""
    return {'depth': volume_L * 1e15, 'n_bins': [1, 1], 'bounds': [1.0, 1.0]}

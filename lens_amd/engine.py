"""Experiment-shaped driver: the reference's multi-rate update loop, batched.

``Experiment`` restates vivarium.core.experiment.Experiment (experiment.py:
1181-1450) over a nested-dict store, with the same scheduling semantics:

* processes are visited depth first (the order of the nested ``processes``
  dict); a process runs when its front time <= time, with timestep =
  min(front + local_timestep, interval) - front, and computes its update
  from the state at that moment (InvokeProcess / ``config['invoke']``,
  :1157-1178, 1282-1311);
* the global step is the smallest timestep that ran; the updates whose
  front lands by then are applied in front order (:1395-1435); the derivers
  run after every applied step and once at construction (:1247, 1319-1349);
* value updates follow Store.apply_update (:586-739): branches recurse,
  leaves apply the schema updater (accumulate by default) or an inline
  ``{'_value', '_updater'}`` one; ``update_field_with_exchange`` gets the
  agent's ``global`` / ``dimensions`` states through its port_mapping
  (registry.py:149-183);
* structural updates at a branch, in the reference's order (:628-697):
  ``_delete`` (paths), ``_add`` (path + state), ``_generate`` (path,
  processes, topology, initial_state: the processes join the tree and their
  ports' schemas register) and ``_divide`` (the mother's values are copied,
  each leaf's ``_divider`` splits them -- :mod:`lens_amd.division` -- the
  daughters are generated at the end of the branch in order, then the mother
  is deleted); the process tree is walked again after any of them, and a
  deriver deleted earlier in the same pass does not run (:1321-1327).

What is batched (SURVEY.md §8 a9 + N2):

* ``config['invoke'] = BatchedInvoke()`` turns every agent's
  ``BatchedConvenienceKinetics.next_update`` of a step into one kernel
  launch (lens_amd/invoke.py);
* ``update_field_with_exchange`` is :mod:`lens_amd.registry`'s device-aware
  updater, the one that also binds into the reference's own
  ``updater_registry``: on a device field (a
  :class:`lens_amd.registry.DeviceField`, as
  :class:`lens_amd.process.BatchedDiffusionField` keeps them) each agent's
  call only queues its (bin, count) on the field, and the queue lands in one
  agent-ordered scatter (``vk_exchange_sorted``) the first time anything reads
  the field -- the same additions in the same order, so the field is
  bit-identical to the reference's one-agent-at-a-time updater.
"""

from __future__ import annotations

import gc
from typing import Dict, List, Tuple

import numpy as np

from lens_amd.agent_store import AgentsNode, AgentView
from lens_amd.division import DIVIDERS
from lens_amd.process import deep_merge
from lens_amd.registry import DeviceField, make_update_field_with_exchange

INFINITY = float('inf')
_MISSING = object()
N_A_LEGACY = 6.022140857e23


def normalize_path(path) -> Tuple:
    """experiment.py:1123-1130 ('..' steps up)."""
    progress = []
    for step in path:
        if step == '..' and progress:
            progress = progress[:-1]
        else:
            progress.append(step)
    return tuple(progress)


def _accumulate(current, new, states):
    return current + new


def _set(current, new, states):
    return new


class _EngineCache(tuple):
    """An engine's per-process cache entry, kept in the process's ``__dict__``
    (one attribute read per use).  It holds store nodes and the engine itself,
    so copies and pickles of the process leave it out (None: rebuilt on use)."""
    __slots__ = ()

    def __copy__(self):
        return None

    def __deepcopy__(self, memo):
        return None

    def __reduce__(self):
        return (type(None), ())


class _InvokeNow:
    def __init__(self, process, interval, states):
        self.update = process.next_update(interval, states)

    def get(self, timeout=0):
        return self.update


_END = object()          # _PathIndex: marks a path's own entry in the trie


class _PathIndex:
    """The store / process paths the engine's caches hold entries for, as a trie, so
    that deleting a subtree drops exactly its entries in time proportional to the
    subtree (the reference drops them with the deleted Store objects,
    experiment.py:505-509).  Each path carries a set of tags (e.g. its ports)."""
    __slots__ = ('root',)

    def __init__(self):
        self.root = {}

    def add(self, path, tag=None):
        node = self.root
        for k in path:
            nxt = node.get(k)
            if nxt is None:
                nxt = node[k] = {}
            node = nxt
        tags = node.get(_END)
        if tags is None:
            tags = node[_END] = set()
        tags.add(tag)

    def pop_prefix(self, prefix):
        """Remove and return [(path, tags)] of every path under `prefix` (itself included)."""
        node = self.root
        for k in prefix[:-1]:
            node = node.get(k)
            if node is None:
                return []
        sub = node.pop(prefix[-1], None) if prefix else node
        if not prefix:
            self.root = {}
        out, stack = [], ([(tuple(prefix), sub)] if sub else [])
        while stack:
            p, n = stack.pop()
            for k, v in n.items():
                if k is _END:
                    out.append((p, v))
                else:
                    stack.append((p + (k,), v))
        return out


class Experiment:
    def __init__(self, config):
        self.processes = config['processes']
        self.topology = config['topology']
        self.invoke = config.get('invoke') or _InvokeNow
        self.avogadro = config.get('avogadro', N_A_LEGACY)
        self.state = _copy_tree(config.get('initial_state', {}))
        # config['agent_columns'] = ('agents',): the agents under that node live in
        # columns (lens_amd.agent_store) -- per-agent dicts become views of rows, and
        # batched processes read and write whole columns (_schedule, _apply_group)
        self.agent_columns = normalize_path(config['agent_columns']) if config.get('agent_columns') else None
        if self.agent_columns is not None:
            node = self.state
            for k in self.agent_columns[:-1]:
                node = node.setdefault(k, {})
            node[self.agent_columns[-1]] = AgentsNode(node.get(self.agent_columns[-1]) or {})
        self.schema: Dict[Tuple, str] = {}
        self._globs: List[Tuple] = []            # the schema paths holding a '*'
        self._port_paths: Dict[Tuple, Tuple] = {}
        self.updaters = {'accumulate': _accumulate, 'set': _set,
                         'update_field_with_exchange': make_update_field_with_exchange(self.avogadro)}
        self._ports: Dict[int, Tuple] = {}          # id(process) -> (process, its port names)
        self._updater_cache: Dict[Tuple, str] = {}  # resolved schema updater per leaf path
        self._leaf_updaters: Dict[Tuple, Dict] = {}  # branch path -> {leaf key: updater name}
        # (agents path, branch) -> {agent id: (version, its leaf branch node, its _leaf_updaters
        # entry, its branch path)}: no per-agent path tuple or walk while the structure stands
        self._agent_leaf_names: Dict[Tuple, Dict] = {}
        # (process path, port) -> (structure version, parent node, parent path, key): the
        # store node a port resolves to.  Value updates replace leaves only; the version
        # moves whenever a dict-valued node is replaced or the schema registers nodes, and
        # an entry from an older version is resolved again.
        self._port_nodes: Dict[Tuple, Tuple] = {}
        self._plans: Dict[Tuple, Tuple] = {}        # process path -> (version, process, kinetics plan)
        self._state_nodes: Dict[Tuple, Tuple] = {}  # process path -> (version, process, [(port, parent, key)])
        self._version = 0
        self._emit_paths: Dict[Tuple, bool] = {}    # store paths with _emit (ordered set)
        self._proc_index = _PathIndex()            # process paths with cached port entries (tag: port)
        self._schema_index = _PathIndex()          # store paths with a schema updater / divider
        self.dividers: Dict[Tuple, object] = {}   # store path (with '*' globs) -> schema _divider
        self._div_globs: List[Tuple] = []
        self._structure = 0                        # moves when processes join or leave the tree
        # processes deleted from the tree during the current send_updates, by id -- the
        # objects are held so that no new process can reuse a deleted one's id
        self._deleted = {}
        self._state_seen = None
        self.local_time = 0.0
        for path, proc in self._walk(self.processes, ()):
            for port, port_schema in proc.ports_schema().items():
                self._register(self.port_path(path, port), port_schema)
        self.send_updates([])

    # -- store -------------------------------------------------------------------
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
        key = (proc_path, port)
        p = self._port_paths.get(key)
        if p is None:
            p = self._port_paths[key] = normalize_path(proc_path[:-1] + tuple(self._topology_of(proc_path)[port]))
            self._proc_index.add(proc_path, port)
        return p

    def get(self, path):
        v = self.state
        for key in path:
            v = v[key]
        return v

    def _lookup(self, path):
        """The node at `path`, or None when a segment is missing: Store.apply_update
        descends only into keys its `inner` holds and drops the rest of an update
        (experiment.py:698-711), e.g. an update to an agent that an earlier update of
        the same batch deleted or divided."""
        v = self.state
        for key in path:
            if not isinstance(v, dict):
                return None
            v = v.get(key, _MISSING)
            if v is _MISSING:
                return None
        return v

    def _register(self, path, schema):
        if not isinstance(schema, dict):
            return
        self._version += 1
        self._clear_leaf_caches()
        keys = [k for k in schema if not k.startswith('_')]
        if ('_default' in schema or '_value' in schema or '_updater' in schema or '_divider' in schema or
                '_emit' in schema) and not keys:
            if '_updater' in schema or '_divider' in schema or schema.get('_emit'):
                self._schema_index.add(path)
            if schema.get('_emit'):
                self._emit_paths[path] = True       # Store.emit (experiment.py:299), in registration order
            if '_updater' in schema:           # a schema without one keeps the store's updater
                self.schema.setdefault(path, schema['_updater'])
                if '*' in path and path not in self._globs:
                    self._globs.append(path)
            if '_divider' in schema:
                self.dividers.setdefault(path, schema['_divider'])
                if '*' in path and path not in self._div_globs:
                    self._div_globs.append(path)
            if '*' not in path and ('_default' in schema or '_value' in schema):
                node = self.state
                for key in path[:-1]:
                    node = node.setdefault(key, {})
                if path[-1] not in node:
                    node[path[-1]] = schema.get('_value', schema.get('_default'))
            elif '*' not in path:
                node = self.state
                for key in path[:-1]:
                    node = node.setdefault(key, {})
                node.setdefault(path[-1], None)    # a store without a default holds None (Store.apply_defaults)
            return
        for k in keys:
            self._register(path + (k,), schema[k])

    def _updater_at(self, path):
        name = self._updater_cache.get(path)
        if name is None:
            name = self._updater_cache[path] = self._resolve_updater(path)
        return name

    def _resolve_updater(self, path):
        if path in self.schema:
            return self.schema[path]
        for pat in self._globs:                  # '*' patterns, in registration order
            if len(pat) == len(path) and all(p == '*' or p == q for p, q in zip(pat, path)):
                return self.schema[pat]
        return 'accumulate'

    # -- updates ---------------------------------------------------------------
    def _port_names(self, proc):
        # a process's ports_schema() is static once it is built (process.py:275-289);
        # the entry keeps the process alive, so its id cannot be reused
        entry = self._ports.get(id(proc))
        if entry is None or entry[0] is not proc:
            entry = self._ports[id(proc)] = (proc, tuple(proc.ports_schema()))
        return entry[1]

    def _port_node(self, proc_path, port):
        key = (proc_path, port)
        ent = self._port_nodes.get(key)
        if ent is None or ent[0] != self._version:
            path = self.port_path(proc_path, port)
            parent = self._lookup(path[:-1])
            ent = self._port_nodes[key] = (self._version, parent if isinstance(parent, dict) else None,
                                           path[:-1], path[-1])
            self._proc_index.add(proc_path, port)
        return ent

    def process_states(self, path, proc):
        # (parent node, key) per port, resolved once per (process path, structure version)
        # and kept on the process itself: one attribute read per call instead of a lookup
        # in a colony-sized dict keyed by path tuples (their hashes are not cached)
        pd = getattr(proc, '__dict__', None)
        ent = pd.get('_engine_state_nodes') if pd is not None else self._state_nodes.get(path)
        if ent is None or ent[0] is not self or ent[1] != path or ent[2] != self._version:
            nodes = []
            for port in self._port_names(proc):
                e = self._port_node(path, port)
                nodes.append((port, e[1], e[3]))
            ent = _EngineCache((self, path, self._version, nodes))
            if pd is not None:
                pd['_engine_state_nodes'] = ent
            else:
                self._state_nodes[path] = ent
        try:
            return {port: parent[key] for port, parent, key in ent[3]}
        except TypeError:
            missing = [port for port, parent, _ in ent[3] if parent is None]
            raise KeyError('process %s: no store for port(s) %s' % (path, missing)) from None

    def apply_update(self, update, proc_path):
        for port, value in update.items():
            _, parent, ppath, key = self._port_node(proc_path, port)
            if parent is None:          # the port's store is gone (deleted earlier in this batch)
                continue
            self._apply(parent, ppath, key, value, proc_path)

    def _apply(self, parent, ppath, key, update, proc_path):
        # parent = the store node at ppath holding `key` (branches pass their own node
        # down; leaf updater names are cached per (branch path, key), so a leaf
        # builds no path tuple once its branch has been seen)
        if key not in parent:
            return
        current = parent[key]
        inline = isinstance(update, dict) and '_updater' in update
        if isinstance(current, dict) and not inline:
            cpath = ppath + (key,)
            if isinstance(update, dict) and ('_delete' in update or '_add' in update or '_generate' in update or
                                             '_divide' in update):
                update = self._structural(cpath, update)
                current = parent.get(key, current)
            names = self._leaf_updaters.get(cpath)
            if names is None:
                names = self._leaf_updaters[cpath] = {}
            updaters = self.updaters
            for k, value in update.items():
                cur = current.get(k, _MISSING)
                if cur is _MISSING:
                    continue
                if isinstance(value, dict) or isinstance(cur, dict):     # inline updater or a branch
                    self._apply(current, cpath, k, value, proc_path)
                    continue
                name = names.get(k)                                      # a plain leaf, inlined
                if name is None:
                    name = names[k] = self._updater_at(cpath + (k,))
                new = current[k] = updaters[name](cur, value, None)
                if type(new) is dict:
                    self._version += 1
            return
        states = None
        if inline:
            spec = update['_updater']
            name, mapping = (spec, None) if isinstance(spec, str) else (spec['updater'], spec.get('port_mapping'))
            value = update.get('_value')
            if mapping is not None:
                states = {}
                for up, pp in mapping.items():
                    ent = self._port_node(proc_path, pp)
                    states[up] = ent[1].get(ent[3]) if ent[1] is not None else None
        else:
            names = self._leaf_updaters.get(ppath)
            if names is None:
                names = self._leaf_updaters[ppath] = {}
            name = names.get(key)
            if name is None:
                name = names[key] = self._updater_at(ppath + (key,))
            value = update
        new = parent[key] = self.updaters[name](current, value, states)
        if isinstance(current, dict) or isinstance(new, dict):
            self._version += 1          # a branch was replaced: cached port nodes below it are stale

    # -- structural updates (Store.apply_update, experiment.py:628-697) ----------------
    def _structural(self, cpath, update):
        """Apply the _delete / _add / _generate / _divide keys of an update at the
        branch ``cpath``, in the reference's order; returns the rest of the update."""
        if '_delete' in update:
            for path in update['_delete']:
                self._delete_path(cpath + tuple(path))
        if '_add' in update:
            for added in update['_add']:
                self._add_path(cpath, tuple(added['path']), added['state'])
        if '_generate' in update:
            for g in update['_generate']:
                self._generate(cpath, tuple(g['path']), g['processes'], g['topology'], g['initial_state'])
        if '_divide' in update:
            self._divide(cpath, update['_divide'])
        return {k: v for k, v in update.items() if k not in ('_delete', '_add', '_generate', '_divide')}

    def _clear_leaf_caches(self):
        self._updater_cache.clear()
        self._leaf_updaters.clear()
        for per_agent in self._agent_leaf_names.values():   # emptied in place: a running
            per_agent.clear()                               # _apply_leaves holds them
        self._agent_leaf_names.clear()

    def _structure_changed(self):
        self._version += 1
        self._structure += 1
        self._clear_leaf_caches()

    def _establish(self, path):
        node = self.state
        for key in path:
            if not isinstance(node.get(key), dict):
                node[key] = {}
            node = node[key]
        return node

    def _add_path(self, cpath, path, state):
        path = normalize_path(cpath + path)
        parent = self._establish(path[:-1])
        if isinstance(parent.get(path[-1]), dict):
            self._set_value(parent[path[-1]], state)
        else:
            parent[path[-1]] = _copy_tree(state)
        self._structure_changed()

    def _set_value(self, node, value):
        """Store.set_value: keys the tree does not hold are ignored."""
        for k, v in value.items():
            if k not in node:
                continue
            if isinstance(node[k], dict) and isinstance(v, dict):
                self._set_value(node[k], v)
            else:
                node[k] = _copy_tree(v)

    def _generate(self, cpath, path, processes, topology, initial_state):
        """Store.generate (experiment.py:1017-1029): the subtree at cpath + path, its
        processes in the process tree, their topology, their ports' schemas."""
        target = normalize_path(cpath + path)
        node = self._establish(target)
        pnode, tnode = self.processes, self.topology
        for key in target[:-1]:
            pnode = pnode.setdefault(key, {})
            tnode = tnode.setdefault(key, {})
        pnode.setdefault(target[-1], {}).update(processes)
        tnode.setdefault(target[-1], {}).update(topology)
        for ppath, proc in self._walk(processes, target):
            for port, port_schema in proc.ports_schema().items():
                self._register(self.port_path(ppath, port), port_schema)
        self._set_value(node, initial_state or {})
        self._structure_changed()

    def _delete_path(self, path):
        parent = self.get(path[:-1]) if path[:-1] else self.state
        if path[-1] not in parent:
            return
        del parent[path[-1]]
        pnode = self.processes
        for key in path[:-1]:
            pnode = pnode.get(key, {}) if isinstance(pnode, dict) else {}
        if isinstance(pnode, dict) and path[-1] in pnode:
            lost = pnode.pop(path[-1])
            for _, proc in (self._walk(lost, ()) if isinstance(lost, dict) else [((), lost)]):
                self._deleted[id(proc)] = proc
                self._ports.pop(id(proc), None)
        self._forget(path)
        self._structure_changed()

    def _forget(self, path):
        """Drop every cache entry under a deleted path: the port nodes and port paths
        of its processes (a port node holds its parent store node, i.e. the deleted
        subtree, alive), and the schema updaters and dividers registered under it, so
        that a path generated again later takes its new processes' topology and schema."""
        for ppath, ports in self._proc_index.pop_prefix(path):
            for port in ports:
                self._port_nodes.pop((ppath, port), None)
                self._port_paths.pop((ppath, port), None)
            self._state_nodes.pop(ppath, None)
            self._plans.pop(ppath, None)
        for spath, _ in self._schema_index.pop_prefix(path):
            self.schema.pop(spath, None)
            self.dividers.pop(spath, None)
            self._emit_paths.pop(spath, None)
            if spath in self._globs:
                self._globs.remove(spath)
            if spath in self._div_globs:
                self._div_globs.remove(spath)

    def _divider_at(self, path):
        if path in self.dividers:
            return self.dividers[path]
        for pat in self._div_globs:
            if len(pat) == len(path) and all(p == '*' or p == q for p, q in zip(pat, path)):
                return self.dividers[pat]
        return None

    def _divide_value(self, path, node):
        """Store.divide_value (experiment.py:512-534)."""
        div = self._divider_at(path)
        if div is not None:
            if isinstance(div, dict):
                base = path[:-1]
                states = {k: self.get(normalize_path(base + tuple(p))) for k, p in div['topology'].items()}
                return div['divider'](node, states)
            return (DIVIDERS[div] if isinstance(div, str) else div)(node)
        if isinstance(node, dict):
            daughters = [{}, {}]
            for key, child in node.items():
                division = self._divide_value(path + (key,), child)
                if division:
                    for daughter, value in zip(daughters, division):
                        daughter[key] = value
            return daughters
        return None

    def _divide(self, cpath, divide):
        mother = divide['mother']
        mpath = cpath + (mother,)
        mstate = self.get(mpath)
        initial_state = _copy_tree(mstate)
        states = self._divide_value(mpath, mstate)
        for daughter, state in zip(divide['daughters'], states):
            initial_state = deep_merge(initial_state, state)
            self._generate(cpath, tuple(daughter['path']), daughter['processes'], daughter['topology'],
                           daughter['initial_state'])
            self._set_value(self.get(cpath + (daughter['daughter'],)), initial_state)
        self._delete_path(mpath)

    def _kinetics_plan(self, proc_path, process):
        """Where a BatchedConvenienceKinetics update lands, resolved once per
        (process path, structure version): per output its store node, key and
        updater -- what apply_update finds by walking the update dict that
        unpack_update would build (internal deltas, fluxes, then the fields'
        inline update_field_with_exchange).  None when a target is not a plain
        leaf (the generic path handles it)."""
        pd = getattr(process, '__dict__', None)
        ent = pd.get('_engine_kinetics_plan') if pd is not None else self._plans.get(proc_path)
        if ent is not None and ent[0] == self._version and ent[1] is process and ent[3] is self and ent[4] == proc_path:
            return ent[2]
        t = process.table
        plan = None
        try:
            def leaves(port, names):
                _, parent, ppath, key = self._port_node(proc_path, port)
                node = parent.get(key, _MISSING) if parent is not None else _MISSING
                if node is _MISSING:
                    return [None] * len(names)           # no such port: apply_update skips it
                if not isinstance(node, dict):
                    raise LookupError
                cpath = ppath + (key,)
                out = []
                for k in names:
                    cur = node.get(k, _MISSING)
                    if cur is _MISSING:
                        out.append(None)                 # no such leaf: the update is dropped
                    elif isinstance(cur, dict):
                        raise LookupError
                    else:
                        fn = self.updaters[self._updater_at(cpath + (k,))]
                        # kind 0 / 1: the built-in accumulate / set, applied inline
                        out.append((node, k, fn, 0 if fn is _accumulate else (1 if fn is _set else 2)))
                return out
            dyn = [leaves(port, [name])[0] for port, name in t.species[:t.n_dyn]]
            flux = leaves('fluxes', t.reaction_ids)
            _, fparent, fppath, fkey = self._port_node(proc_path, 'fields')
            fnode = fparent.get(fkey, _MISSING) if fparent is not None else _MISSING
            if not isinstance(fnode, dict):
                raise LookupError                        # the generic path decides
            states = {}
            for up, pp in {'global': 'global', 'dimensions': 'dimensions'}.items():
                e = self._port_node(proc_path, pp)
                states[up] = e[1][e[3]]
            exch = self.updaters['update_field_with_exchange']
            site = getattr(exch, 'site', None)           # lens_amd.registry's updater: one bin per agent
            fields = []
            for mol in t.external_ids:
                cur = fnode.get(mol, _MISSING)
                if isinstance(cur, dict):
                    raise LookupError
                fields.append(None if cur is _MISSING else (fnode, mol))
            plan = (dyn, flux, fields, exch, states, site)
        except (LookupError, KeyError, TypeError):
            plan = None
        ent = _EngineCache((self._version, process, plan, self, proc_path))
        if pd is not None:
            pd['_engine_kinetics_plan'] = ent
        else:
            self._plans[proc_path] = ent
        return plan

    def _apply_kinetics(self, proc_path, process, fluxes, deltas, counts):
        plan = self._kinetics_plan(proc_path, process)
        if plan is None:
            self.apply_update(process.unpack_update(fluxes, deltas, counts), proc_path)
            return
        dyn, flux, fields, exch, states, site = plan
        bump = False
        # the updaters in apply_update's order; accumulate / set inline (a float or
        # numpy scalar sum / value is never a dict, so the structure cannot move)
        for tgt, d in zip(dyn, deltas):
            if tgt is not None:
                node, k, fn, kind = tgt
                if kind == 0:
                    node[k] = node[k] + d
                elif kind == 1:
                    node[k] = d
                else:
                    new = node[k] = fn(node[k], d, None)
                    bump |= type(new) is dict
        for tgt, f in zip(flux, fluxes):
            if tgt is not None:
                node, k, fn, kind = tgt
                if kind == 0:
                    node[k] = node[k] + np.float64(f)
                elif kind == 1:
                    node[k] = np.float64(f)
                else:
                    new = node[k] = fn(node[k], np.float64(f), None)
                    bump |= type(new) is dict
        where = None
        for tgt, c in zip(fields, counts):
            if tgt is not None:
                node, mol = tgt
                cur = node[mol]
                if site is not None and type(cur) is DeviceField:
                    # update_field_with_exchange on a device field, with the agent's
                    # bin derived once for all its molecules
                    if where is None:
                        where = site(states)
                    if cur._t.shape != where[2]:
                        raise ValueError('field shape %s does not match n_bins %s'
                                         % (cur.shape, list(where[2])))
                    cur.queue_exchange(where[0], int(c), where[1])
                    continue
                new = node[mol] = exch(cur, c, states)
                bump |= isinstance(new, dict)
        if bump:
            self._version += 1

    def _apply_leaves(self, proc_path, up):
        """Apply a :class:`lens_amd.process.AgentLeafUpdate` exactly as
        :meth:`apply_update` applies ``up.as_dict()`` -- the other ports, then for each
        agent the leaves under ``up.path`` with their schema updaters (a missing
        agent, branch or leaf is skipped) -- without building the per-agent dicts.
        An agent whose branch is not plain dicts goes through :meth:`_apply`."""
        if up.rest:
            self.apply_update(up.rest, proc_path)
        if not up.ids:
            return
        _, parent, ppath, key = self._port_node(proc_path, 'agents')
        if parent is None:
            return
        agents = parent.get(key, _MISSING)
        if not isinstance(agents, dict):
            self.apply_update(up.as_dict(), proc_path)
            return
        apath = ppath + (key,)
        if isinstance(agents, AgentsNode) and self._apply_leaves_columns(agents, apath, up):
            return
        updaters, keys, path = self.updaters, up.keys, up.path
        leaf_updaters = self._leaf_updaters
        by_agent = self._agent_leaf_names.get((apath, path))
        if by_agent is None:
            by_agent = self._agent_leaf_names[(apath, path)] = {}
        for aid, row in zip(up.ids, up.rows):
            # the agent's leaf branch, its path and its leaf updater names, kept per
            # agent until the store's structure moves (the port-node rule)
            ent = by_agent.get(aid)
            if ent is not None and ent[0] == self._version:
                node, names, cpath = ent[1], ent[2], ent[3]
            else:
                node = agents.get(aid, _MISSING)
                if node is _MISSING:
                    continue
                for k in path:
                    if not isinstance(node, dict):
                        break
                    node = node.get(k, _MISSING)
                    if node is _MISSING:
                        break
                if node is _MISSING:
                    continue
                if not isinstance(node, dict):
                    one = dict(zip(keys, row))
                    for k in reversed(path):
                        one = {k: one}
                    self._apply(agents, apath, aid, one, proc_path)
                    continue
                cpath = apath + (aid,) + path
                names = leaf_updaters.get(cpath)
                if names is None:
                    names = leaf_updaters[cpath] = {}
                by_agent[aid] = (self._version, node, names, cpath)
            for k, value in zip(keys, row):
                cur = node.get(k, _MISSING)
                if cur is _MISSING:
                    continue
                if isinstance(cur, dict):
                    self._apply(node, cpath, k, value, proc_path)
                    continue
                name = names.get(k)
                if name is None:
                    name = names[k] = self._updater_at(cpath + (k,))
                fn = updaters[name]
                if fn is _set:
                    node[k] = value
                    if type(value) is dict:
                        self._version += 1
                    continue
                new = node[k] = cur + value if fn is _accumulate else fn(cur, value, None)
                if type(new) is dict:
                    self._version += 1

    # -- columnar agents: whole-column application (lens_amd.agent_store) ---------------
    def _all_agents_resolve(self, apath, agents, leaf, name):
        """Whether every agent's ``leaf`` (a path below the agent) resolves to the
        schema updater ``name`` -- checked once per structure version."""
        cache = self.__dict__.setdefault('_resolve_cache', {})
        key = (apath, leaf, name)
        ent = cache.get(key)
        if ent is None or ent[0] != self._version:
            ok = all(self._updater_at(apath + (aid,) + leaf) == name for aid in agents)
            ent = cache[key] = (self._version, ok)
        return ent[1]

    def _apply_leaves_columns(self, agents, apath, up):
        """An AgentLeafUpdate on columnar agents as one column write per key, when
        that is what the per-agent walk would do: every agent present with the
        branch and every leaf a float that its schema sets (``set``).  False:
        nothing applied (the per-agent walk follows)."""
        from lens_amd.agent_store import _F
        t = agents.table
        cache = self.__dict__.get('_leaf_rows')
        if cache is not None and cache[0] is agents and cache[1] == self._version and cache[2] == up.ids:
            rows = cache[3]
        else:
            try:
                rows = agents.rows(up.ids)
            except KeyError:
                return False
            self._leaf_rows = (agents, self._version, list(up.ids), rows)
        path = up.path
        for i in range(1, len(path) + 1):
            m = t.present.get(path[:i])
            if m is None or not m[rows].all():
                return False
        leaves = []
        for k in up.keys:
            lp = path + (k,)
            if t.kind.get(lp) != _F or not t.present[lp][rows].all():
                return False
            if not self._all_agents_resolve(apath, agents, lp, 'set'):
                return False
            leaves.append(lp)
        vals = np.asarray(up.rows, dtype=np.float64).reshape(len(up.ids), len(leaves))
        if len(set(up.ids)) != len(up.ids):
            return False
        for j, lp in enumerate(leaves):
            t.cols[lp][rows] = vals[:, j]
            t.npf[lp][rows] = False                      # the row values are Python floats
        return True

    def _schedule(self, processes, front):
        """The scheduler's entries for ``processes`` (walk order): a run of two or
        more consecutive agent kinetics processes that can be applied as columns
        (:meth:`_kinetics_group`) becomes one group entry with one front; every
        other process is its own entry.  Only processes without a front yet are
        grouped (the caller builds groups at the start of an update call)."""
        sched = []
        run = []

        def close():
            if len(run) >= 2 and all(front.get(p) is None for p, _, _ in run):
                grp = self._kinetics_group(run)
                if grp is not None:
                    sched.append(grp)
                    run.clear()
                    return
            for p, proc, _ in run:
                sched.append((p, proc))
            run.clear()

        can = self.agent_columns is not None and hasattr(self.invoke, 'group_call')
        for path, proc in processes:
            key = self._group_key(path, proc) if can else None
            if key is None or (run and key != run[0][2]):
                close()
            if key is None:
                sched.append((path, proc))
            else:
                run.append((path, proc, key))
        close()
        return sched

    def _group_key(self, path, proc):
        from lens_amd.process import BatchedConvenienceKinetics
        if not isinstance(proc, BatchedConvenienceKinetics) or len(path) != len(self.agent_columns) + 2 or \
                path[:len(self.agent_columns)] != self.agent_columns:
            return None
        topo = self._topology_of(path)
        p = proc.parameters
        return (type(proc), proc.signature, path[-1], proc.local_timestep(), p.get('integrator', 'euler'),
                p.get('rtol', 1e-8), p.get('atol', 1e-12), p.get('max_steps', 100000),
                tuple(sorted((k, tuple(v)) for k, v in topo.items())))

    def _kinetics_group(self, run):
        """A group entry for a run of agent kinetics processes, or None if any
        member's outputs would not land as whole-column writes.  The members'
        per-agent plans (:meth:`_kinetics_plan`) must all be the same plan in
        column terms: every output a float leaf of the agent's own row with the same
        updater, every exchange on the same device fields."""
        from lens_amd.agent_store import _F
        agents = self.get(self.agent_columns)
        if not isinstance(agents, AgentsNode):
            return None
        t = agents.table
        procs = [proc for _, proc, _ in run]
        paths = [p for p, _, _ in run]
        aids = [p[len(self.agent_columns)] for p in paths]
        try:
            rows = agents.rows(aids)
        except KeyError:
            return None
        shape = None
        for path, proc, aid in zip(paths, procs, aids):
            plan = self._kinetics_plan(path, proc)
            if plan is None:
                return None
            dyn, flux, fields, exch, states, site = plan
            if site is None:
                return None
            row = agents.row(aid)
            cols = []
            for tgt in list(dyn) + list(flux):
                if tgt is None:
                    return None                     # a skipped output: the per-agent path decides
                node, k, fn, kind = tgt
                if not isinstance(node, AgentView) or node._r != row or kind == 2:
                    return None
                cols.append((node._p + (k,), kind))
            fl = []
            for ft in fields:
                if ft is None:
                    fl.append(None)
                    continue
                fnode, mol = ft
                if isinstance(fnode, AgentView):
                    return None
                fl.append((id(fnode), mol))
            loc = states.get('global')
            if not isinstance(loc, AgentView) or loc._r != row:
                return None
            sig = (tuple(cols), tuple(fl), id(states.get('dimensions')), loc._p)
            if shape is None:
                shape = sig
                first_plan = plan
            elif sig != shape:
                return None
        dyn_cols, fields = shape[0][:len(first_plan[0])], first_plan[2]
        flux_cols = shape[0][len(first_plan[0]):]
        for c, _ in shape[0]:
            if t.kind.get(c) != _F:
                return None
        topo = self._topology_of(paths[0])
        pack = []
        for port, name in procs[0].table.species:
            rel = topo.get(port)
            pack.append(None if rel is None else normalize_path(tuple(rel)) + (name,))
        gl = topo.get('global')
        if gl is None or any(r is not None and r[:1] == ('..',) for r in pack):
            return None
        return _Group(key=('__group__', paths[0], paths[-1], len(paths)), paths=paths, procs=procs, aids=aids,
                      rows=rows, table=t, pack=pack, m2c=normalize_path(tuple(gl)) + ('mmol_to_counts',),
                      loc=shape[3] + ('location',), dyn=dyn_cols, flux=flux_cols, fields=fields,
                      dims=first_plan[4]['dimensions'], exch=first_plan[3], version=self._version,
                      timestep=procs[0].local_timestep())

    def _invoke_group(self, g, timestep):
        """Pack the group's agents from the columns (the values pack_state reads
        per agent) and hand them to the invoke hook as one call."""
        t, rows = g.table, g.rows
        conc = np.empty((len(g.pack), len(rows)), dtype=np.float64)
        for i, c in enumerate(g.pack):
            conc[i] = 0.0 if c is None else t.gather(c, rows, 0.0)
        m = t.present.get(g.m2c)
        if m is None or not m[rows].all():
            raise KeyError('mmol_to_counts')
        m2c = t.gather(g.m2c, rows)
        # the parameters are re-read every call, as the per-agent path reads
        # process.param_values: an in-place change between update() calls reaches both
        params = np.stack([p.param_values for p in g.procs], axis=1)
        return self.invoke.group_call(g.procs, timestep, conc, m2c, params)

    def _apply_group(self, g, flux, delta, counts):
        """A group's kinetics outputs as column writes -- each agent's
        :meth:`_apply_kinetics` in agent order: internal deltas, fluxes, then the
        exchange queued on the device fields."""
        from lens_amd.agent_store import _F
        t, rows = g.table, g.rows
        if any(t.kind.get(c) != _F for c, _ in g.dyn + g.flux) or self._version != g.version:
            for i, (path, proc) in enumerate(zip(g.paths, g.procs)):
                self._apply_kinetics(path, proc, flux[:, i].tolist(), delta[:, i].tolist(),
                                     counts[:, i].tolist())
            return
        for (c, kind), d in zip(g.dyn, delta):
            col = t.cols[c]
            if kind == 0:
                col[rows] = col[rows] + d                 # float + float, or np.float64 + float
            else:
                col[rows] = d
                t.npf[c][rows] = False
        for (c, kind), f in zip(g.flux, flux):
            col = t.cols[c]
            col[rows] = col[rows] + f if kind == 0 else f
            t.npf[c][rows] = True                         # np.float64(f) (+ ...) in the per-agent path
        if not any(ft is not None for ft in g.fields):
            return
        loc = np.array([t.cols[g.loc][r] for r in rows.tolist()], dtype=np.float64).reshape(len(rows), 2)
        dims = g.dims
        nx, ny = int(dims['n_bins'][0]), int(dims['n_bins'][1])
        i = np.mod(np.floor(loc[:, 0] * nx / dims['bounds'][0]).astype(np.int64), nx)
        j = np.mod(np.floor(loc[:, 1] * ny / dims['bounds'][1]).astype(np.int64), ny)
        bins = (i * ny + j).tolist()
        _, bva, shape = g.exch.site({'global': {'location': [0.0, 0.0]}, 'dimensions': dims})
        for e, ft in enumerate(g.fields):
            if ft is None:
                continue
            fnode, mol = ft
            cur = fnode[mol]
            if type(cur) is not DeviceField:
                for a in range(len(rows)):          # a host field: the updater, agent by agent
                    states = {'global': {'location': loc[a].tolist()}, 'dimensions': dims}
                    cur = fnode[mol] = g.exch(fnode[mol], int(counts[e, a]), states)
                continue
            if cur._t.shape != shape:
                raise ValueError('field shape %s does not match n_bins %s' % (cur.shape, list(shape)))
            cur.queue_exchange_many(bins, counts[e], bva)

    def send_updates(self, updates, derivers=None):
        self._deleted = {}
        for update, path in updates:
            group = getattr(update, 'group_raw', None)
            if group is not None:
                self._apply_group(path, *group())
                continue
            raw = getattr(update, 'raw', None)
            leaves = getattr(update, 'leaf_raw', None)
            if raw is not None:
                self._apply_kinetics(path, *raw())       # BatchedInvoke: no update dict
            elif leaves is not None:
                self._apply_leaves(path, leaves())       # BatchedDiffusionField: columns
            else:
                self.apply_update(update.get(), path)
        if derivers is None:
            derivers = [(p, s) for p, s in self._walk(self.processes, ()) if s.is_deriver()]
        for path, deriver in derivers:
            if id(deriver) in self._deleted:          # removed by an earlier deriver's _divide / _delete
                continue
            self.apply_update(deriver.next_update(0, self.process_states(path, deriver)), path)

    def emit_data(self):
        """Store.emit_data (experiment.py:463-481): the values of the stores whose
        schema sets ``_emit``, as a nested dict (branches in the order their first
        emitted leaf was registered; a '*' in a path matches every child, in store
        order).  Stores that are gone are skipped."""
        out = {}

        def put(path, value):
            node = out
            for k in path[:-1]:
                node = node.setdefault(k, {})
            node[path[-1]] = value

        def expand(node, path, rest):
            if not rest:
                put(path, node)
                return
            if not isinstance(node, dict):
                return
            k = rest[0]
            if k == '*':
                for child, sub in node.items():
                    expand(sub, path + (child,), rest[1:])
            elif k in node:
                expand(node[k], path + (k,), rest[1:])
        for path in self._emit_paths:
            expand(self.state, (), path)
        return out

    # -- Experiment.update (experiment.py:1351-1450) ---------------------------------
    def update(self, interval):
        # Python's cyclic GC would traverse every agent's dicts over and over
        # while a step allocates its update dicts (40 % of the loop's host time
        # at 8k agents, scripts/invoke_profile.py): it is paused for the call;
        # reference counting still frees everything acyclic as it goes
        paused = gc.isenabled()
        gc.disable()
        try:
            return self._update(interval)
        finally:
            if paused:
                gc.enable()

    def _update(self, interval):
        if self.state is not self._state_seen:     # the whole store was replaced from outside
            self._state_seen = self.state
            self._version += 1
        time = 0
        front = {}
        # the reference re-walks the tree every iteration (:1373-1380) because a
        # _generate / _divide update can add processes; here it is walked again only
        # after such an update moved the structure
        seen = None
        sched = None
        while time < interval:
            if seen != self._structure:
                # the walk, kept while the process tree's structure stands (it moves with
                # every _generate / _delete / _divide; the tree is not edited otherwise)
                wc = self.__dict__.get('_walk_cache')
                if wc is not None and wc[0] == self._structure and wc[1] is self.processes:
                    processes, derivers = wc[2], wc[3]
                else:
                    everything = self._walk(self.processes, ())
                    processes = [(p, s) for p, s in everything if not s.is_deriver()]
                    derivers = [(p, s) for p, s in everything if s.is_deriver()]
                    self._walk_cache = (self._structure, self.processes, processes, derivers)
                if seen is None:
                    # columnar agents: runs of agent kinetics processes are scheduled as one
                    # entry each (one front, one invoke, one column apply), formed only here,
                    # at the start of the call, where every front starts at 0 -- and kept for
                    # the next call while the process list and the store's structure stand
                    cache = self.__dict__.get('_sched_cache')
                    if (cache is not None and cache[0] == self._structure and cache[1] == self._version and
                            cache[2] is processes):
                        sched = cache[3]
                    else:
                        sched = self._schedule(processes, front)
                        self._sched_cache = (self._structure, self._version, processes, sched)
                else:
                    # the structure moved mid-call: groups dissolve into their members, in
                    # place in the front order, with the group's front (and a pending update
                    # split per member); no regrouping until the next call
                    front = _dissolve_groups(front)
                    sched = processes
                if front:
                    live = {p for p, _ in processes}
                    front = {p: f for p, f in front.items() if p in live or p[0] == '__group__'}
                seen = self._structure
            full_step = INFINITY
            invoke, states_of = self.invoke, self.process_states
            last = None
            for entry in sched:
                if type(entry) is _Group:
                    key = entry.key
                    adv = front.get(key)
                    if adv is None:
                        adv = front[key] = {'time': time, 'update': None, 'group': entry}
                    process_time = adv['time']
                    if process_time <= time:
                        future = min(process_time + entry.timestep, interval)
                        timestep = future - process_time
                        pending = self._invoke_group(entry, timestep)
                        if timestep < full_step:
                            full_step = timestep
                        adv['time'] = future
                        adv['update'] = (pending, entry)
                    last = key
                    continue
                path, proc = entry
                adv = front.get(path)
                if adv is None:
                    adv = front[path] = {'time': time, 'update': None}
                process_time = adv['time']
                if process_time <= time:
                    future = min(process_time + proc.local_timestep(), interval)
                    timestep = future - process_time
                    pending = invoke(proc, timestep, states_of(path, proc))
                    if timestep < full_step:
                        full_step = timestep
                    adv['time'] = future
                    adv['update'] = (pending, path)
                last = path
            if full_step == INFINITY:
                next_event = interval
                for _ in front.keys():
                    if front[last]['time'] < next_event:   # the reference's stale `path` (:1414-1419)
                        next_event = front[last]['time']
                time = next_event
            else:
                future = time + full_step
                updates = []
                for path, advance in front.items():
                    if advance['time'] <= future and advance['update'] is not None:
                        updates.append(advance['update'])
                        advance['update'] = None
                self.send_updates(updates, derivers)
                time = future
                self.local_time += full_step
        return self


class _Group:
    """A scheduler entry for a run of agent kinetics processes handled as columns."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class _MemberUpdate:
    """Member i of a group's pending update, as a per-agent future (``raw()``)."""

    def __init__(self, pending, i, proc):
        self.pending, self.i, self.proc = pending, i, proc

    def raw(self):
        flux, delta, counts = self.pending.group_raw()
        i = self.i
        return self.proc, flux[:, i].tolist(), delta[:, i].tolist(), counts[:, i].tolist()

    def get(self, timeout=0):
        return self.proc.unpack_update(*self.raw()[1:])


def _dissolve_groups(front):
    """Front entries with every group replaced by its members' entries, in place
    in the order (a group's pending update split into per-member futures)."""
    out = {}
    for key, adv in front.items():
        g = adv.get('group') if isinstance(adv, dict) else None
        if g is None:
            out[key] = adv
            continue
        upd = adv['update']
        for i, (path, proc) in enumerate(zip(g.paths, g.procs)):
            out[path] = {'time': adv['time'],
                         'update': (_MemberUpdate(upd[0], i, proc), path) if upd is not None else None}
    return out


def _copy_tree(t):
    if isinstance(t, dict):
        return {k: _copy_tree(v) for k, v in t.items()}
    if isinstance(t, np.ndarray):
        return t.copy()
    if isinstance(t, DeviceField):
        return DeviceField(t.tensor.clone())
    if getattr(t, 'is_cuda', False):
        return t.clone()
    if isinstance(t, list):
        return list(t)
    return t

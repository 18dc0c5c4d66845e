"""Columnar (SoA) storage for the agents of a Process-API colony.

The reference keeps every agent's state as a tree of ``Store`` objects
(vivarium/core/experiment.py:203-1030); :class:`lens_amd.engine.Experiment`
restates it over nested dicts.  With tens of thousands of agents those
per-agent trees are what the per-agent loop spends its time walking, and
their cache footprint grows with the colony.

Here the subtree under one agents node (``Experiment(config['agent_columns']
= ('agents',))``) lives in columns instead: one column per leaf path below an
agent (``('internal', 'glc__D_e')``, ``('boundary', 'external', 'ac_e')`` ...),
one row per agent.  ``state['agents']`` is an :class:`AgentsNode` -- a dict of
agent id -> :class:`AgentView` in the colony's order -- and an
:class:`AgentView` is a dict-shaped view of one agent's row, so every process,
updater, divider and emitter that reads or writes per-agent dicts works
unchanged.  What changes is what batched code can do: read a leaf for every
agent as one array (:meth:`AgentTable.gather`) and write it back as one
(:meth:`AgentTable.scatter`) -- the engine's batched kinetics and leaf updates
do (lens_amd/engine.py).

Leaf values keep their Python types: Python floats and numpy float64 scalars
live in a float64 array (a per-cell flag remembers which of the two a cell
holds, so each reads back as it was written); any other value (ints, bools,
lists, device fields, quantities) lives in an object column.  Each path has a presence mask, so agents may hold different
sets of keys (missing keys behave as in a dict).
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

_F, _OBJ = 0, 2


class AgentTable:
    """The columns behind one :class:`AgentsNode`."""

    def __init__(self, capacity: int = 64):
        self.cap = max(16, int(capacity))
        self.trie: Dict = {}                        # key -> child trie (dict) or leaf path (tuple)
        self.cols: Dict[Tuple, object] = {}         # leaf path -> float64 array or list
        self.kind: Dict[Tuple, int] = {}
        self.npf: Dict[Tuple, np.ndarray] = {}      # float leaf path -> bool[cap]: the cell holds np.float64
        self.present: Dict[Tuple, np.ndarray] = {}  # every path (leaf or branch) -> bool[cap]
        self.free: List[int] = []
        self.rows = 0                               # rows handed out (high-water mark)

    # -- rows -------------------------------------------------------------------
    def _grow(self, need):
        if need <= self.cap:
            return
        cap = self.cap
        while cap < need:
            cap *= 2
        for p, c in self.cols.items():
            if isinstance(c, np.ndarray):
                n = np.zeros(cap, dtype=np.float64)
                n[:self.cap] = c
                self.cols[p] = n
            else:
                c.extend([None] * (cap - self.cap))
        for d in (self.present, self.npf):
            for p, m in d.items():
                n = np.zeros(cap, dtype=bool)
                n[:self.cap] = m
                d[p] = n
        self.cap = cap

    def new_row(self) -> int:
        if self.free:
            return self.free.pop()
        self._grow(self.rows + 1)
        self.rows += 1
        return self.rows - 1

    def free_row(self, row: int):
        for m in self.present.values():
            m[row] = False
        self.free.append(row)

    # -- paths ------------------------------------------------------------------
    def _node(self, prefix):
        node = self.trie
        for k in prefix:
            node = node[k]
        return node

    def _ensure_branch(self, prefix, key):
        node = self._node(prefix)
        child = node.get(key)
        if child is None:
            child = node[key] = {}
            self.present[prefix + (key,)] = np.zeros(self.cap, dtype=bool)
        elif isinstance(child, tuple):
            raise TypeError('agent store: %r is a leaf, not a branch' % (prefix + (key,),))
        return child

    def _ensure_leaf(self, prefix, key, value):
        node = self._node(prefix)
        path = prefix + (key,)
        child = node.get(key)
        if child is None:
            node[key] = path
            t = type(value)
            if t is float or t is np.float64:
                self.cols[path], self.kind[path] = np.zeros(self.cap, dtype=np.float64), _F
                self.npf[path] = np.zeros(self.cap, dtype=bool)
            else:
                self.cols[path], self.kind[path] = [None] * self.cap, _OBJ
            self.present[path] = np.zeros(self.cap, dtype=bool)
        elif isinstance(child, dict):
            raise TypeError('agent store: %r is a branch, not a leaf' % (path,))
        return path

    def _to_object(self, path):
        c, npf = self.cols[path], self.npf.pop(path)
        self.cols[path] = [np.float64(x) if f else x for x, f in zip(c.tolist(), npf.tolist())]
        self.kind[path] = _OBJ

    # -- one value --------------------------------------------------------------
    def get(self, path, row):
        c = self.cols[path]
        if self.kind[path] == _F:
            return c[row] if self.npf[path][row] else float(c[row])
        return c[row]

    def set(self, path, row, value):
        if self.kind[path] == _F:
            t = type(value)
            if t is float or t is np.float64:
                self.cols[path][row] = value
                self.npf[path][row] = t is np.float64
                self.present[path][row] = True
                return
            self._to_object(path)
        self.cols[path][row] = value
        self.present[path][row] = True

    def clear_below(self, path, row):
        """Mark ``path`` and everything under it absent for ``row``."""
        for p, m in self.present.items():
            if p[:len(path)] == path:
                m[row] = False

    # -- whole columns (the batched paths) -----------------------------------------
    def is_float(self, path) -> bool:
        return self.kind.get(path, _OBJ) != _OBJ

    def gather(self, path, rows, default=0.0):
        """float64 values of a float leaf for ``rows`` (``default`` where absent)."""
        c = self.cols.get(path)
        if c is None:
            return np.full(len(rows), default, dtype=np.float64)
        m = self.present[path][rows]
        if self.kind[path] == _OBJ:              # values of other types: float() each (the slow path)
            return np.array([float(getattr(c[r], 'magnitude', c[r])) if ok else default
                             for r, ok in zip(rows.tolist(), m.tolist())], dtype=np.float64)
        v = c[rows]
        if not m.all():
            v = np.where(m, v, default)
        return v

    def scatter(self, path, rows, values, np_scalar=False):
        """Set a leaf to float64 ``values`` for ``rows`` (the column is created as a
        Python-float column, or numpy-float64 with ``np_scalar``)."""
        if path not in self.cols:
            prefix, key = path[:-1], path[-1]
            node = self.trie
            for i, k in enumerate(prefix):
                node = self._ensure_branch(prefix[:i], k)
            self._ensure_leaf(prefix, key, 0.0)
        if self.kind[path] == _OBJ:
            conv = np.float64 if np_scalar else float
            col = self.cols[path]
            for r, v in zip(rows.tolist(), values.tolist()):
                col[r] = conv(v)
        else:
            self.cols[path][rows] = values
            self.npf[path][rows] = bool(np_scalar)
        self.present[path][rows] = True
        for i in range(1, len(path)):
            self.present[path[:i]][rows] = True


class AgentView(dict):
    """One agent's subtree (or a branch of it) as a dict-shaped view of its row.

    A ``dict`` subclass so that code testing ``isinstance(x, dict)`` treats it as
    a branch; it stores nothing itself -- every method reads and writes the
    table (the dict's own storage stays empty)."""

    __slots__ = ('_t', '_r', '_p', '_n')

    def __init__(self, table, row, prefix=(), node=None):
        dict.__init__(self)
        self._t, self._r, self._p = table, row, prefix
        self._n = table._node(prefix) if node is None else node

    # -- reading ----------------------------------------------------------------
    def __contains__(self, key):
        child = self._n.get(key)
        if child is None:
            return False
        return bool(self._t.present[child if isinstance(child, tuple) else self._p + (key,)][self._r])

    def __getitem__(self, key):
        child = self._n.get(key)
        if child is not None:
            if isinstance(child, tuple):
                if self._t.present[child][self._r]:
                    return self._t.get(child, self._r)
            elif self._t.present[self._p + (key,)][self._r]:
                return AgentView(self._t, self._r, self._p + (key,), child)
        raise KeyError(key)

    def get(self, key, default=None):
        child = self._n.get(key)
        if child is not None:
            if isinstance(child, tuple):
                if self._t.present[child][self._r]:
                    return self._t.get(child, self._r)
            elif self._t.present[self._p + (key,)][self._r]:
                return AgentView(self._t, self._r, self._p + (key,), child)
        return default

    def __iter__(self):
        t, r, p = self._t, self._r, self._p
        for k, child in list(self._n.items()):
            if t.present[child if isinstance(child, tuple) else p + (k,)][r]:
                yield k

    def keys(self):
        return list(self.__iter__())

    def __len__(self):
        return sum(1 for _ in self.__iter__())

    def __bool__(self):
        return any(True for _ in self.__iter__())

    def items(self):
        return [(k, self[k]) for k in self.__iter__()]

    def values(self):
        return [self[k] for k in self.__iter__()]

    # -- writing ----------------------------------------------------------------
    def __setitem__(self, key, value):
        t, r, p = self._t, self._r, self._p
        if isinstance(value, dict):
            self._t._ensure_branch(p, key)
            path = p + (key,)
            snapshot = list(value.items())           # the source may be a view of this row
            t.clear_below(path, r)
            t.present[path][r] = True
            sub = AgentView(t, r, path)
            for k, v in snapshot:
                sub[k] = v
        else:
            path = t._ensure_leaf(p, key, value)
            t.set(path, r, value)

    def __delitem__(self, key):
        if key not in self:
            raise KeyError(key)
        self._t.clear_below(self._p + (key,), self._r)

    def setdefault(self, key, default=None):
        if key not in self:
            self[key] = default
        return self[key]

    def pop(self, key, *default):
        if key in self:
            v = self[key]
            v = to_dict(v) if isinstance(v, AgentView) else v
            del self[key]
            return v
        if default:
            return default[0]
        raise KeyError(key)

    def update(self, other=(), **kw):
        for k, v in (other.items() if hasattr(other, 'items') else other):
            self[k] = v
        for k, v in kw.items():
            self[k] = v

    def clear(self):
        self._t.clear_below(self._p, self._r)
        if self._p:
            self._t.present[self._p][self._r] = True

    # -- as a plain dict ----------------------------------------------------------
    def copy(self):
        return to_dict(self)

    def __copy__(self):
        return to_dict(self)

    def __deepcopy__(self, memo):
        import copy
        return copy.deepcopy(to_dict(self), memo)

    def __reduce__(self):
        return (dict, (to_dict(self),))

    def __eq__(self, other):
        return to_dict(self) == (to_dict(other) if isinstance(other, AgentView) else other)

    def __ne__(self, other):
        return not self.__eq__(other)

    __hash__ = None

    def __repr__(self):
        return repr(to_dict(self))


def to_dict(x):
    """A plain nested dict snapshot of a view (other values unchanged)."""
    if isinstance(x, AgentView):
        return {k: to_dict(v) for k, v in x.items()}
    return x


class AgentsNode(dict):
    """The agents node: agent id -> :class:`AgentView`, in the colony's order (a
    real dict of views); assigning a plain dict stores it as a new row."""

    def __init__(self, agents=None, table=None):
        dict.__init__(self)
        self.table = table or AgentTable(len(agents or ()) + 16)
        for aid, state in (agents or {}).items():
            self[aid] = state

    def row(self, aid) -> int:
        return dict.__getitem__(self, aid)._r

    def rows(self, ids) -> np.ndarray:
        get = dict.__getitem__
        return np.fromiter((get(self, a)._r for a in ids), dtype=np.int64, count=len(ids))

    def values_at(self, path, ids):
        """The values of the leaf ``path`` (below each agent) for ``ids``, as a list --
        ``[self[a][path...] for a in ids]`` without the per-agent views."""
        t = self.table
        rows = self.rows(ids)
        m = t.present.get(path)
        if m is None or not m[rows].all():
            raise KeyError(path)
        c = t.cols[path]
        if t.kind[path] == _F:
            vals = c[rows].tolist()
            npf = t.npf[path][rows]
            if npf.any():
                vals = [np.float64(v) if f else v for v, f in zip(vals, npf.tolist())]
            return vals
        return [c[r] for r in rows.tolist()]

    def __setitem__(self, aid, value):
        t = self.table
        if isinstance(value, AgentView) and value._t is t and not value._p:
            old = dict.get(self, aid)
            if old is not None and old._r != value._r:
                t.free_row(old._r)
            dict.__setitem__(self, aid, value)
            return
        if not isinstance(value, dict):
            raise TypeError('an agent state must be a dict (got %s)' % type(value).__name__)
        snapshot = list(value.items())
        old = dict.get(self, aid)
        if old is not None:
            row = old._r
            t.clear_below((), row)
        else:
            row = t.new_row()
        view = AgentView(t, row, (), t.trie)
        for k, v in snapshot:
            view[k] = v
        dict.__setitem__(self, aid, view)

    def __delitem__(self, aid):
        view = dict.__getitem__(self, aid)
        dict.__delitem__(self, aid)
        self.table.free_row(view._r)

    def pop(self, aid, *default):
        if aid in self:
            v = to_dict(dict.__getitem__(self, aid))
            del self[aid]
            return v
        if default:
            return default[0]
        raise KeyError(aid)

    def setdefault(self, aid, default=None):
        if aid not in self:
            self[aid] = {} if default is None else default
        return dict.__getitem__(self, aid)

    def update(self, other=(), **kw):
        for k, v in (other.items() if hasattr(other, 'items') else other):
            self[k] = v
        for k, v in kw.items():
            self[k] = v

    def clear(self):
        for aid in list(self):
            del self[aid]

    def copy(self):
        return {k: to_dict(v) for k, v in self.items()}

    def __copy__(self):
        return self.copy()

    def __deepcopy__(self, memo):
        import copy
        return copy.deepcopy(self.copy(), memo)

    def __reduce__(self):
        return (dict, (self.copy(),))

    def __repr__(self):
        return repr(self.copy())

"""Batching ``invoke`` hook for the reference ``Experiment``.

``Experiment`` calls ``self.invoke(process, interval, states)`` for every
process that is due and consumes the result only through ``.get()`` inside
``send_updates`` (vivarium/core/experiment.py:1157-1178, 1230, 1282-1311,
1338-1341).  :class:`BatchedInvoke` exploits that: it records each
``BatchedConvenienceKinetics`` call (packing the agent's state into a host
SoA row immediately, since ``states`` are live store references), and the
first ``.get()`` of the step launches ONE kernel per (network, interval)
group for all recorded agents.  Other processes run immediately, as with the
reference's ``InvokeProcess``.

    experiment = Experiment({..., 'invoke': BatchedInvoke()})
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch

from lens_amd import native
from lens_amd.kinetics import KineticsEngine
from lens_amd.process import BatchedConvenienceKinetics

_ENGINES: Dict[Tuple[str, int], KineticsEngine] = {}


def engine_for(process: BatchedConvenienceKinetics, device=None) -> KineticsEngine:
    dev = native.resolve_device(device)
    key = (process.signature, dev.index if dev.index is not None else 0)
    eng = _ENGINES.get(key)
    if eng is None:
        eng = KineticsEngine(process.table, dev)
        _ENGINES[key] = eng
    return eng


class _Packed:
    __slots__ = ('process', 'interval', 'conc', 'm2c')

    def __init__(self, process, interval, states):
        self.process = process
        self.interval = float(interval)
        self.conc, self.m2c = process.pack_state(states)    # species values as a list, m2c


def _run_group(items: List[_Packed], device=None, raw: bool = False) -> List:
    p0 = items[0].process
    t = p0.table
    eng = engine_for(p0, device)
    n = len(items)
    dev = eng.device
    conc = torch.from_numpy(np.array([it.conc for it in items], dtype=np.float64).T.copy()).to(dev)
    params = torch.from_numpy(np.stack([it.process.param_values for it in items], axis=1)).to(dev).contiguous()
    m2c = torch.tensor([it.m2c for it in items], dtype=torch.float64, device=dev)
    delta = torch.zeros((t.n_dyn, n), dtype=torch.float64, device=dev)
    integrator = p0.parameters.get('integrator', 'euler')
    dt = items[0].interval
    if integrator == 'euler':
        flux, counts, status = eng.euler(dt, params, conc, m2c, delta=delta)
    elif integrator == 'dopri5':
        h = torch.tensor([getattr(it.process, '_h_state', 0.0) for it in items],
                         dtype=torch.float64, device=dev)
        flux, counts, status, _ = eng.dopri5(
            dt, params, conc, m2c, h_state=h, delta=delta,
            rtol=p0.parameters.get('rtol', 1e-8), atol=p0.parameters.get('atol', 1e-12),
            max_steps=p0.parameters.get('max_steps', 100000))
        for it, hv in zip(items, h.cpu().numpy()):
            it.process._h_state = float(hv)
    else:
        raise ValueError('unknown integrator %r' % integrator)
    st = status.cpu().numpy()
    if st.any():
        bad = int(np.flatnonzero(st)[0])
        raise FloatingPointError('agent %d: kernel status %d (1=max steps, 2=step underflow, '
                                 '4=non-finite)' % (bad, int(st[bad])))
    # agent-major Python lists in one conversion each (no per-element numpy scalars)
    flux_l = flux.t().cpu().tolist()
    delta_l = delta.t().cpu().tolist()
    counts_l = counts.t().cpu().tolist()
    if raw:
        return [(it.process, f, d, c) for it, f, d, c in zip(items, flux_l, delta_l, counts_l)]
    return [it.process.unpack_update(f, d, c) for it, f, d, c in zip(items, flux_l, delta_l, counts_l)]


def _run_arrays(procs, interval, conc, m2c, params, device=None):
    """One launch for a group of agents given as arrays (conc [species, n], m2c
    [n], params [P, n]): what _run_group computes from per-agent packs, returned
    as host arrays (flux [R, n], delta [ND, n], counts [E, n])."""
    p0 = procs[0]
    t = p0.table
    eng = engine_for(p0, device)
    n = len(procs)
    dev = eng.device
    conc_d = torch.from_numpy(np.ascontiguousarray(conc)).to(dev)
    params_d = torch.from_numpy(np.ascontiguousarray(params)).to(dev)
    m2c_d = torch.from_numpy(np.ascontiguousarray(m2c)).to(dev)
    delta = torch.zeros((t.n_dyn, n), dtype=torch.float64, device=dev)
    integrator = p0.parameters.get('integrator', 'euler')
    if integrator == 'euler':
        flux, counts, status = eng.euler(interval, params_d, conc_d, m2c_d, delta=delta)
    elif integrator == 'dopri5':
        h = torch.tensor([getattr(p, '_h_state', 0.0) for p in procs], dtype=torch.float64, device=dev)
        flux, counts, status, _ = eng.dopri5(
            interval, params_d, conc_d, m2c_d, h_state=h, delta=delta,
            rtol=p0.parameters.get('rtol', 1e-8), atol=p0.parameters.get('atol', 1e-12),
            max_steps=p0.parameters.get('max_steps', 100000))
        for p, hv in zip(procs, h.cpu().tolist()):
            p._h_state = hv
    else:
        raise ValueError('unknown integrator %r' % integrator)
    st = status.cpu().numpy()
    if st.any():
        bad = int(np.flatnonzero(st)[0])
        raise FloatingPointError('agent %d: kernel status %d (1=max steps, 2=step underflow, '
                                 '4=non-finite)' % (bad, int(st[bad])))
    return flux.cpu().numpy(), delta.cpu().numpy(), counts.cpu().numpy()


class _GroupFuture:
    """A group call's outputs (lens_amd.engine.Experiment's columnar agents):
    ``group_raw()`` = (flux [R, n], delta [ND, n], counts [E, n]) host arrays."""
    __slots__ = ('owner', 'result')

    def __init__(self, owner):
        self.owner = owner
        self.result = None

    def group_raw(self):
        if self.result is None:
            self.owner.flush()
        return self.result

    def get(self, timeout=0):
        raise TypeError('a group call has no single update dict (use group_raw)')


def run_batch(calls, device=None) -> List[dict]:
    """Evaluate [(process, interval, states)] in as few launches as possible."""
    packed = [_Packed(p, dt, s) for p, dt, s in calls]
    groups: Dict[Tuple[str, float, str], List[int]] = {}
    for i, it in enumerate(packed):
        key = (it.process.signature, it.interval, it.process.parameters.get('integrator', 'euler'))
        groups.setdefault(key, []).append(i)
    out: List[dict] = [None] * len(packed)
    for idx in groups.values():
        res = _run_group([packed[i] for i in idx], device)
        for i, r in zip(idx, res):
            out[i] = r
    return out


class _Future:
    """One recorded call's result: filled in by the owner's flush (the first
    ``get()`` / ``raw()`` of the step launches every recorded call)."""
    __slots__ = ('owner', 'result')

    def __init__(self, owner):
        self.owner = owner
        self.result = None

    def get(self, timeout=0):
        """The reference's update dict (convenience_kinetics.py:316-349)."""
        process, f, d, c = self.raw()
        return process.unpack_update(f, d, c)

    def raw(self):
        """(process, fluxes, deltas, counts) -- the same outputs before they are
        packed into the update dict; lens_amd.engine.Experiment applies them
        straight into the store (same updaters, same order)."""
        if self.result is None:
            self.owner.flush()
        return self.result


class _Immediate:
    def __init__(self, update):
        self.update = update

    def get(self, timeout=0):
        return self.update


class _ImmediateLeaves:
    """A process's :class:`lens_amd.process.AgentLeafUpdate`: ``get()`` is the
    reference's update dict, ``leaf_raw()`` the columns (lens_amd.engine.Experiment)."""

    def __init__(self, raw):
        self.raw_update = raw

    def get(self, timeout=0):
        return self.raw_update.as_dict()

    def leaf_raw(self):
        return self.raw_update


class BatchedInvoke:
    """Drop-in value for ``Experiment(config['invoke'])``."""

    def __init__(self, device=None):
        self.device = device
        self._pending = []
        self._groups = []

    def __call__(self, process, interval, states):
        if not isinstance(process, BatchedConvenienceKinetics):
            raw = getattr(process, 'next_update_raw', None)
            if raw is not None:
                return _ImmediateLeaves(raw(interval, states))
            return _Immediate(process.next_update(interval, states))
        fut = _Future(self)
        self._pending.append((fut, _Packed(process, interval, states)))
        return fut

    def group_call(self, procs, interval, conc, m2c, params):
        """Record a whole group of agents' calls, packed as arrays by the caller
        (lens_amd.engine.Experiment with columnar agents); launched with the
        step's other calls at the first ``get()``."""
        fut = _GroupFuture(self)
        self._groups.append((fut, procs, float(interval), conc, m2c, params))
        return fut

    def flush(self):
        """Launch every recorded call: one kernel per (network, interval,
        integrator) group; each future receives its agent's outputs."""
        groups, self._groups = self._groups, []
        for fut, procs, interval, conc, m2c, params in groups:
            fut.result = _run_arrays(procs, interval, conc, m2c, params, self.device)
        if not self._pending:
            return
        pending, self._pending = self._pending, []
        groups: Dict[Tuple, List[Tuple[_Future, _Packed]]] = {}
        for fut, it in pending:
            key = (it.process.signature, it.interval, it.process.parameters.get('integrator', 'euler'))
            groups.setdefault(key, []).append((fut, it))
        for members in groups.values():
            res = _run_group([it for _, it in members], self.device, raw=True)
            for (fut, _), r in zip(members, res):
                fut.result = r

"""The Process-API loop with its agents held in columns (Experiment(config
['agent_columns'] = ('agents',)), lens_amd/agent_store.py) against the
per-agent dict store: the same states, bit for bit and type for type, with
the batched paths on (one scheduler entry, one pack and one column apply for a
run of agent kinetics processes; one column write for the diffusion process's
agent leaves) -- including a colony whose structure changes in the middle of
an update call (the groups dissolve into their members).  The kernels are
replaced by seeded stand-ins (scripts/engine_host_ab.py), so this runs on the
CPU; tests/test_engine_gpu.py runs the real launches."""

import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'scripts'))
import engine_host_ab as hab  # noqa: E402


def _fields(exp):
    return [(list(f._bins), list(f._counts), f._bva) for f in exp.state['fields'].values()]


@pytest.mark.parametrize('n', [1, 7, 300])
def test_columns_equal_dicts_kinetics_and_diffusion(n):
    a, b = hab.make(n, False), hab.make(n, True)
    for interval in (1.0, 3.0, 0.5, 2.0):
        a.update(interval)
        b.update(interval)
        assert repr(a.state['agents']) == repr(b.state['agents'])
        assert _fields(a) == _fields(b)
        assert a.local_time == b.local_time
    if n > 1:
        sched = b._sched_cache[3]
        assert any(type(e).__name__ == '_Group' for e in sched)       # the batched path ran


class Culler:
    """Deletes the first agent every 2 s (structure changes mid-call)."""
    name = 'culler'

    def local_timestep(self):
        return 2.0

    def is_deriver(self):
        return False

    def ports_schema(self):
        return {'cells': {'*': {}}}

    def next_update(self, timestep, states):
        return {'cells': {'_delete': [(k,) for k in list(states['cells'])[:1]]}}


def test_columns_equal_dicts_when_agents_leave_mid_call():
    from lens_amd.engine import Experiment
    exps = []
    for columns in (False, True):
        p, t, init = hab.build(40)
        p['culler'], t['culler'] = Culler(), {'cells': ('agents',)}
        cfg = {'processes': p, 'topology': t, 'initial_state': init, 'invoke': hab.StubInvoke()}
        if columns:
            cfg['agent_columns'] = ('agents',)
        exp = Experiment(cfg)
        for m in list(exp.state['fields']):
            exp.state['fields'][m] = hab.host_field()
        exps.append(exp)
    a, b = exps
    for interval in (5.0, 1.0, 4.0):
        a.update(interval)
        b.update(interval)
        assert list(a.state['agents']) == list(b.state['agents'])
        assert repr(a.state['agents']) == repr(b.state['agents'])
        assert _fields(a) == _fields(b)
    assert len(b.state['agents']) < 40


def test_columnar_loop_is_flat_in_the_colony_size():
    """Host cost per agent-step (CPU time, stand-in kernels) stays within 1.6x
    from 200 to 6400 agents (the dict store grows ~1.5x over a shorter range);
    a loose bound for a shared CI host -- scripts/engine_host_ab.py times it."""
    import gc
    import time
    per = []
    for n in (200, 6400):
        exp = hab.make(n, True)
        exp.update(1.0)
        best = float('inf')
        for _ in range(3):
            gc.collect()
            t0 = time.process_time()
            exp.update(2.0)
            best = min(best, time.process_time() - t0)
        per.append(best / (2 * n))
    assert per[1] < 1.6 * per[0] + 2e-6, per


def test_group_reads_parameters_changed_in_place():
    """A cached scheduler group re-reads its members' param_values on every call,
    as the per-agent path reads process.param_values: an in-place change between
    update() calls reaches the columnar launch too."""
    seen = []

    class Recording(hab.StubInvoke):
        def flush(self):
            for _, procs, _, _, _, params in self._groups:
                seen.append(params.copy())
            super().flush()

    p, t, init = hab.build(8)
    from lens_amd.engine import Experiment
    exp = Experiment({'processes': p, 'topology': t, 'initial_state': init, 'invoke': Recording(),
                      'agent_columns': ('agents',)})
    for m in list(exp.state['fields']):
        exp.state['fields'][m] = hab.host_field()
    exp.update(1.0)
    assert seen, 'the batched path did not run'
    proc = p['agents']['a00003']['kinetics']
    proc.param_values[0] = 12345.0
    seen.clear()
    exp.update(1.0)
    assert seen and any((s == 12345.0).any() for s in seen)

"""Host cost of lens_amd.engine.Experiment's per-agent loop on the CPU, no GPU:
scripts/invoke_throughput.py's colony (glc_ac kinetics per agent, one
diffusion-field process over all agents), with the device work replaced by
stand-ins that keep the host side of the path -- BatchedInvoke's packing of
every agent's state, the direct kinetics apply with device-field exchange
queueing, and the diffusion process's AgentLeafUpdate of every agent's
externals.  The kernels' results are seeded random numbers.  For A/B of engine
changes on a quiet host (the GPU boxes' host timing varies +-50 %).

    python scripts/engine_host_ab.py [n_agents ...]
"""
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lens_amd.invoke import BatchedInvoke  # noqa: E402
from lens_amd.process import AgentLeafUpdate, Process  # noqa: E402
from lens_amd.registry import DeviceField  # noqa: E402

NX = NY = 64


def host_field():
    """A DeviceField over a host tensor: queue_exchange works, nothing reads it."""
    f = object.__new__(DeviceField)
    f._t = torch.zeros((NX, NY), dtype=torch.float64)
    f._bins, f._counts, f._bva = [], [], None
    return f


class StubInvoke(BatchedInvoke):
    """BatchedInvoke whose launch is replaced by seeded outputs."""

    def __init__(self):
        super().__init__(None)
        self.rng = np.random.default_rng(3)

    def _pool(self, table):
        pool = self.__dict__.get('pool')
        if pool is None:     # 64 seeded outputs, reused in turn (the stand-in costs next to nothing)
            pool = self.pool = [(self.rng.normal(size=table.n_reactions).tolist(),
                                 (1e-3 * self.rng.normal(size=table.n_dyn)).tolist(),
                                 self.rng.integers(-50, 50, size=table.n_ext).tolist()) for _ in range(64)]
        return pool

    def flush(self):
        pending, self._pending = self._pending, []
        groups, self._groups = self._groups, []
        for i, (fut, it) in enumerate(pending):
            fut.result = (it.process,) + self._pool(it.process.table)[i & 63]
        for fut, procs, interval, conc, m2c, params in groups:     # columnar agents: agent i = call i
            pool = self._pool(procs[0].table)
            sel = [pool[i & 63] for i in range(len(procs))]
            fut.result = (np.array([x[0] for x in sel]).T.copy(), np.array([x[1] for x in sel]).T.copy(),
                          np.array([x[2] for x in sel], dtype=np.int64).T.copy())


class StubDiffusion(Process):
    """BatchedDiffusionField's host side: every agent's externals as one
    AgentLeafUpdate; the fields' queued exchange is dropped (no device)."""
    name = 'stub_diffusion'

    def __init__(self, fields):
        super().__init__({'time_step': 1.0})
        self.fields = fields
        self.rng = np.random.default_rng(4)

    def ports_schema(self):
        return {'agents': {'*': {'boundary': {'external': {m: {'_default': 0.0, '_updater': 'set'}
                                                           for m in self.fields}}}},
                'fields': {m: {'_default': None} for m in self.fields},
                'dimensions': {}}

    def next_update_raw(self, timestep, states):
        for f in states['fields'].values():
            f._bins.clear()
            f._counts.clear()
        ids = list(states['agents'])
        rows = self.rng.random((len(ids), len(self.fields))).tolist()
        return AgentLeafUpdate({}, ids, ('boundary', 'external'), list(self.fields), rows)

    def next_update(self, timestep, states):
        return self.next_update_raw(timestep, states).as_dict()


def build(n):
    from lens_amd import configs
    from lens_amd.process import BatchedConvenienceKinetics
    from invoke_throughput import mmol_to_counts
    cfg = configs.glc_ac_config()
    rng = np.random.default_rng(1)
    mols = ['glc__D_e', 'ac_e']
    processes = {'diffusion': StubDiffusion(mols), 'agents': {}}
    topology = {'diffusion': {'agents': ('agents',), 'fields': ('fields',), 'dimensions': ('dimensions',)},
                'agents': {}}
    agents = {}
    for a in range(n):
        aid = 'a%05d' % a
        processes['agents'][aid] = {'kinetics': BatchedConvenienceKinetics(dict(cfg, time_step=1.0))}
        topology['agents'][aid] = {'kinetics': {
            'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
            'fields': ('..', '..', 'fields'), 'dimensions': ('..', '..', 'dimensions'), 'global': ('boundary',)}}
        agents[aid] = {'internal': dict(cfg['initial_state']['internal']), 'fluxes': {},
                       'boundary': {'location': [float(rng.uniform(0, NX)), float(rng.uniform(0, NY))],
                                    'mmol_to_counts': mmol_to_counts(1339.0),
                                    'external': {'glc__D_e': 0.0, 'ac_e': 0.0}}}
    init = {'agents': agents, 'fields': {m: None for m in mols},
            'dimensions': {'bounds': [float(NX), float(NY)], 'n_bins': [NX, NY], 'depth': 10.0}}
    return processes, topology, init


def make(n, columns):
    from lens_amd.engine import Experiment
    p, t, init = build(n)
    cfg = {'processes': p, 'topology': t, 'initial_state': init, 'invoke': StubInvoke()}
    if columns:
        cfg['agent_columns'] = ('agents',)
    exp = Experiment(cfg)
    for m in list(exp.state['fields']):      # after the initial state's copy (it clones device fields)
        exp.state['fields'][m] = host_field()
    return exp


def main():
    """COLUMNS=1: the agents held in columns (lens_amd.agent_store); COLUMNS=both:
    both stores, and their states after the timed calls must be equal."""
    from lens_amd.engine import Experiment  # noqa: F401
    sizes = [int(x) for x in sys.argv[1:]] or [500, 2000, 8000, 32000]
    reps = int(os.environ.get('REPS', '5'))
    mode = os.environ.get('COLUMNS', '0')
    for n in sizes:
        if mode == 'both':
            a, b = make(n, False), make(n, True)
            for _ in range(3):
                a.update(1.0)
                b.update(1.0)
            fa = [list(f._bins) + list(f._counts) for f in a.state['fields'].values()]
            fb = [list(f._bins) + list(f._counts) for f in b.state['fields'].values()]
            same = repr(a.state['agents']) == repr(b.state['agents']) and fa == fb
            print('agents %6d  dict store == columns: %s' % (n, same), flush=True)
            continue
        exp = make(n, mode == '1')
        exp.update(1.0)
        best = float('inf')
        for _ in range(reps):
            gc.collect()
            t0 = time.process_time()          # this process's CPU time: steadier than wall time on a shared host
            exp.update(3.0)
            best = min(best, time.process_time() - t0)
        print('agents %6d  %.2f us of CPU per agent-step (min of %d calls of 3 steps)%s'
              % (n, best / (3 * n) * 1e6, reps, '  [columns]' if mode == '1' else ''), flush=True)


if __name__ == '__main__':
    main()

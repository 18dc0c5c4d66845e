"""Host cost of the Experiment-shaped loop (lens_amd.engine) per agent-step, on CPU.

Every agent has a stub process with BatchedConvenienceKinetics' port shape
(internal species accumulate, fluxes set, external / global / dimensions read)
that returns a fixed update, so what is timed is the loop itself: scheduling,
state views, update application (the part of the Process-API path that stays
Python).  No GPU is touched.

    python scripts/engine_overhead.py [n_agents ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lens_amd import configs  # noqa: E402
from lens_amd.engine import Experiment  # noqa: E402
from lens_amd.process import Process  # noqa: E402

CFG = configs.glc_lct_config()
INTERNAL = dict(CFG['initial_state']['internal'])
EXTERNAL = dict(CFG['initial_state']['external'])
FLUXES = list(CFG['kinetic_parameters'])


class StubKinetics(Process):
    name = 'stub_kinetics'
    defaults = {'time_step': 1.0}

    def ports_schema(self):
        return {'internal': {k: {'_default': v} for k, v in INTERNAL.items()},
                'external': {k: {'_default': v} for k, v in EXTERNAL.items()},
                'fluxes': {r: {'_default': 0.0, '_updater': 'set'} for r in FLUXES},
                'global': {'mmol_to_counts': {'_default': 0.0}, 'location': {'_default': [0.5, 0.5]}},
                'dimensions': {'bounds': {'_default': [1, 1]}, 'n_bins': {'_default': [1, 1]},
                               'depth': {'_default': 1.0}}}

    def local_timestep(self):
        return self.parameters['time_step']

    def next_update(self, timestep, states):
        return {'internal': {k: 1e-9 * timestep for k in states['internal']},
                'fluxes': {r: 1e-3 for r in FLUXES}}


def build(n):
    processes = {'agents': {}}
    topology = {'agents': {}}
    for a in range(n):
        aid = 'a%05d' % a
        processes['agents'][aid] = {'kinetics': StubKinetics()}
        topology['agents'][aid] = {'kinetics': {
            'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
            'global': ('boundary',), 'dimensions': ('..', '..', 'dimensions')}}
    return {'processes': processes, 'topology': topology, 'initial_state': {}}


def main():
    for n in [int(x) for x in sys.argv[1:]] or [500, 2000, 8000]:
        exp = Experiment(build(n))
        exp.update(1.0)
        t0 = time.perf_counter()
        steps = 3
        exp.update(float(steps))
        dt = time.perf_counter() - t0
        print('agents %d  %.1f us of loop per agent-step' % (n, dt / (n * steps) * 1e6), flush=True)


if __name__ == '__main__':
    main()

"""Throughput of the Process-API path (lens_amd.engine.Experiment + BatchedInvoke +
BatchedDiffusionField): every agent keeps its own process object and dict
state, as under the reference's Experiment.  glc_ac network, 64x64 lattice,
kinetics and diffusion every 1 s.  Prints agent-steps/s (the reference's own
engine: 59-154 us of Python per agent-step).

    python scripts/invoke_throughput.py [n_agents ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

NX = NY = 64


def mmol_to_counts(volume_fL, avogadro=6.022140857e23):
    return avogadro * volume_fL * 1e-15 * 1e-3


def build(n, dev):
    from lens_amd import configs
    from lens_amd.process import BatchedConvenienceKinetics, BatchedDiffusionField
    cfg = configs.glc_ac_config()
    rng = np.random.default_rng(1)
    glc = configs.gaussian_bump_field((NX, NY))
    env = {'molecules': ['glc__D_e', 'ac_e'], 'n_bins': [NX, NY], 'bounds': [float(NX), float(NY)],
           'depth': 10.0, 'diffusion': 5.0, 'time_step': 1.0,
           'initial_state': {'glc__D_e': glc, 'ac_e': np.zeros((NX, NY))}}
    processes = {'diffusion': BatchedDiffusionField(dict(env, device=dev)), 'agents': {}}
    topology = {'diffusion': {'agents': ('agents',), 'fields': ('fields',), 'dimensions': ('dimensions',)},
                'agents': {}}
    agents = {}
    for a in range(n):
        kin_cfg = dict(cfg, time_step=1.0)
        aid = 'a%05d' % a
        processes['agents'][aid] = {'kinetics': BatchedConvenienceKinetics(kin_cfg)}
        topology['agents'][aid] = {'kinetics': {
            'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
            'fields': ('..', '..', 'fields'), 'dimensions': ('..', '..', 'dimensions'), 'global': ('boundary',)}}
        agents[aid] = {'internal': dict(cfg['initial_state']['internal']), 'fluxes': {},
                       'boundary': {'location': [float(rng.uniform(0, NX)), float(rng.uniform(0, NY))],
                                    'mmol_to_counts': mmol_to_counts(1339.0),
                                    'external': {'glc__D_e': 0.0, 'ac_e': 0.0}}}
    init = {'agents': agents, 'dimensions': {'bounds': env['bounds'], 'n_bins': env['n_bins'], 'depth': env['depth']}}
    return processes, topology, init


def main():
    from lens_amd.engine import Experiment
    from lens_amd.invoke import BatchedInvoke
    dev = torch.device('cuda', 0)
    for n in [int(x) for x in sys.argv[1:]] or [500, 2000, 8000]:
        p, t, init = build(n, dev)
        exp = Experiment({'processes': p, 'topology': t, 'initial_state': init, 'invoke': BatchedInvoke(dev)})
        exp.update(1.0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        exp.update(3.0)
        torch.cuda.synchronize()
        rate = 3 * n / (time.perf_counter() - t0)
        print('agents %d  batched Experiment %.0f agent-steps/s (%.1f us per agent-step)' % (n, rate, 1e6 / rate),
              flush=True)


if __name__ == '__main__':
    main()

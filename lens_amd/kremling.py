"""Batched Kremling 2007 sugar transport -- the reference's odeint path on the GPU.

``vivarium/processes/Kremling2007_transport.py`` integrates an 11-state stiff
ODE (+ 4 flux integrals) with ``scipy.integrate.odeint`` once per agent per
timestep.  :class:`KremlingColony` keeps N agents' states as SoA rows on the
device and advances all of them with one ``vk_kremling_step`` launch
(adaptive DP5(4) per lane, landing on the reference's 100-point output grid).
:class:`BatchedKremlingTransport` is the Process-API drop-in (same ``name``,
ports and update dict as ``Transport``) running a batch of one.
"""

from __future__ import annotations

import copy
import ctypes

import numpy as np
import torch

from lens_amd import native
from lens_amd.process import ProcessBase

N_A_LEGACY = 6.022140857e23

# Kremling2007_transport.py:19-70 (DEFAULT_PARAMETERS), restated
KREMLING_PARAMETERS = {
    'k1': 0.00001, 'k2': 0.0001, 'k3': 0.00016, 'K1': 3000, 'K2': 2800, 'K3': 15000, 'kd': 0.4,
    'm': 1, 'n': 2, 'x0': 0.1, 'kg6p': 2.8e6, 'Kg6p': 0.1, 'kptsup': 2.7e8, 'Kglc': 0.12,
    'Keiiap': 12, 'klac': 5.4e5, 'Km_lac': 0.13, 'Kieiia': 5.0, 'kgly': 2.80e4, 'kpyk': 9.39e5,
    'kpdh': 5.50e3, 'kpts': 1.86e5, 'km_pts': 0.7 * 1.86e5, 'Y': 1.0e-4, 'mw1': 2.602e-4,
    'mw2': 1.802e-4, 'mw3': 3.423e-4, 'Y1_sim': 6.2448e-05, 'Y2_sim': 1.0e-4, 'Y3_sim': 9.2421e-05,
    'Y4_sim': 1.0e-04, 'K': 0.4, 'kb': 600, 'ksyn': 3.2623e3, 'KI': 1 / 8000,
}
INTERNAL = ('mass', 'UHPT', 'LACZ', 'PTSG', 'G6P', 'PEP', 'PYR', 'XP')
EXTERNAL = ('GLC', 'G6P', 'LCTS')
TARGET_FLUXES = ('glc__D_e', 'GLCpts', 'PPS', 'PYK')     # Transport.defaults (:93-96)
FLUX_ROWS = ('GLCpts', 'PPS', 'PYK', 'glc__D_e')         # kernel flux[] row order
# GLC_G6P condition: internal (:121-133) + external media (data/flat/media/GLC_G6P.tsv)
GLC_G6P_INTERNAL = {'mass': 0.032, 'LACZ': 0.0, 'UHPT': 0.0003, 'PTSG': 0.007, 'G6P': 0.2057,
                    'PEP': 2.0949, 'PYR': 2.0949, 'XP': 0.0038}
GLC_G6P_MEDIA = {'ACET': 0.0, 'CO+2': 100.0, 'ETOH': 0.0, 'FORMATE': 0.0, 'GLYCEROL': 0.0, 'LAC': 0.0,
                 'LCTS': 0.0, 'OXYGEN-MOLECULE': 100.0, 'PI': 100.0, 'PYR': 0.0, 'RIB': 0.0, 'SUC': 0.0,
                 'G6P': 1.3451, 'GLC': 12.2087}


def vk_params(p) -> native.VkKremlingParams:
    out = native.VkKremlingParams()
    for name, _ in native.VkKremlingParams._fields_:
        setattr(out, name, float(p[name]))
    return out


def output_grid(timestep: float, dt: float = 0.01):
    """(grid step in hours, number of grid points) of np.arange(0, timestep/3600, dt/3600)."""
    return dt / 3600, len(np.arange(0, timestep / 3600, dt / 3600))


class KremlingColony:
    """N agents' Kremling states on one GPU (SoA, FP64)."""

    def __init__(self, n_agents: int, device=None, parameters=None, internal=None, external=None,
                 volume_fl: float = 1.0, rtol: float = 1e-8, atol: float = 1e-12, max_steps: int = 1_000_000,
                 avogadro: float = N_A_LEGACY):
        self.device = native.resolve_device(device)
        native.load()
        self.n = int(n_agents)
        self.parameters = dict(KREMLING_PARAMETERS, **(parameters or {}))
        self.rtol, self.atol, self.max_steps, self.avogadro = rtol, atol, max_steps, avogadro
        internal = dict(GLC_G6P_INTERNAL, **(internal or {}))
        external = dict(GLC_G6P_MEDIA, **(external or {}))
        col = [internal[k] for k in INTERNAL] + [external[k] for k in EXTERNAL] + [0.0] * 4
        z = lambda *shape, dtype=torch.float64: torch.zeros(shape, dtype=dtype, device=self.device)
        self.state = torch.tensor(col, dtype=torch.float64).repeat(self.n, 1).t().contiguous().to(self.device)
        self.volume = torch.full((self.n,), float(volume_fl), dtype=torch.float64, device=self.device)
        self.flux = z(4, self.n)
        self.counts = z(3, self.n, dtype=torch.int64)
        self.status = z(self.n, dtype=torch.int32)
        self.nsteps = z(self.n, dtype=torch.int32)
        self.h_state = z(self.n)

    def set_state(self, state):
        """state: [>=11, n] host/torch values for rows mass .. LCTS[e]."""
        s = torch.as_tensor(state, dtype=torch.float64)
        self.state[:s.shape[0]].copy_(s.to(self.device))

    def step(self, timestep: float = 1.0, carry_h: bool = False):
        grid_h, n_grid = output_grid(timestep)
        # the launch stream and the parameter set's device copy (cached per
        # device by the library) belong to this colony's GPU
        with torch.cuda.device(self.device):
            if not carry_h:
                self.h_state.zero_()      # odeint restarts every call
            native.check(native._lib.vk_kremling_step(
                ctypes.byref(vk_params(self.parameters)), self.n, self.n, timestep / 3600, grid_h, n_grid,
                self.rtol, self.atol, self.max_steps, native.ptr(self.state), native.ptr(self.volume),
                self.avogadro, native.ptr(self.h_state), native.ptr(self.flux), native.ptr(self.counts),
                native.ptr(self.status), native.ptr(self.nsteps), native.stream_handle()), 'vk_kremling_step')

    def check_status(self):
        st = self.status.cpu().numpy()
        if st.any():
            a = int(np.flatnonzero(st)[0])
            raise FloatingPointError('agent %d: kernel status %d' % (a, int(st[a])))


class BatchedKremlingTransport(ProcessBase):
    """Process-API drop-in for ``Transport`` (Kremling2007_transport.py:91-427)."""

    name = 'Kremling2007_transport'
    defaults = {'target_fluxes': list(TARGET_FLUXES), 'parameters': KREMLING_PARAMETERS}

    def __init__(self, initial_parameters=None):
        initial_parameters = dict(initial_parameters or {})
        self.target_fluxes = initial_parameters.get('target_fluxes', self.defaults['target_fluxes'])
        parameters = copy.deepcopy(self.defaults['parameters'])
        parameters.update(initial_parameters)
        super().__init__(parameters)

    def ports_schema(self):
        set_internal = set(INTERNAL)
        schema = {port: {} for port in ('internal', 'external', 'fields', 'fluxes', 'global', 'dimensions')}
        emit_internal = set(INTERNAL)
        for state, value in GLC_G6P_INTERNAL.items():
            schema['internal'][state] = {'_default': value, '_updater': 'set' if state in set_internal else 'accumulate',
                                         '_divider': 'set' if state in set_internal else 'accumulate',
                                         '_emit': state in emit_internal}
        for state, value in GLC_G6P_MEDIA.items():
            schema['external'][state] = {'_default': value, '_emit': state in ('G6P', 'GLC', 'LAC', 'LCTS')}
            schema['fields'][state] = {'_default': np.ones((1, 1))}
        for state in self.target_fluxes:
            schema['fluxes'][state] = {'_default': 0.0, '_updater': 'set', '_divider': 'set', '_emit': True}
        schema['global'] = {'volume': {'_default': 1}, 'location': {'_default': [0.5, 0.5]}}
        schema['dimensions'] = {'bounds': {'_default': [1, 1]}, 'n_bins': {'_default': [1, 1]},
                                'depth': {'_default': 1}}
        return schema

    def next_update(self, timestep, states):
        col = KremlingColony(1, parameters=self.parameters,
                             internal={k: float(states['internal'][k]) for k in INTERNAL},
                             external={k: float(states['external'][k]) for k in EXTERNAL},
                             volume_fl=float(getattr(states['global']['volume'], 'magnitude',
                                                     states['global']['volume'])))
        col.step(timestep)
        col.check_status()
        s = col.state[:8, 0].cpu().numpy()
        fl = dict(zip(FLUX_ROWS, col.flux[:, 0].cpu().numpy().tolist()))
        cnt = col.counts[:, 0].cpu().numpy().tolist()
        return {
            'fields': {mol: {'_value': int(c), '_updater': {
                'updater': 'update_field_with_exchange',
                'port_mapping': {'global': 'global', 'dimensions': 'dimensions'}}}
                for mol, c in zip(EXTERNAL, cnt)},
            'internal': {k: float(v) for k, v in zip(INTERNAL, s) if k in states['internal']},
            'fluxes': {k: fl[k] for k in self.target_fluxes if k in fl},
        }

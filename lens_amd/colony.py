"""Persistent SoA colony: the batched replacement of the reference's per-agent loop.

The reference advances a colony by walking its Store tree once per agent and
per process every timestep (``Experiment.update``, vivarium/core/experiment.py:
1351-1450; 59-154 us of Python per agent-step).  Here every
agent is a column of device-resident FP64 arrays and one timestep is a fixed
sequence of kernel launches on one stream:

environment ``'held'`` (BASELINE config 2)
    kinetics only; external concentrations stay at their per-agent values.
environment ``'nonspatial'`` (config 1; NonSpatialEnvironment per agent,
vivarium/processes/nonspatial_environment.py:14-82)
    kinetics -> exchange into each agent's own 1x1 field -> external := field.
a :class:`~lens_amd.lattice.Lattice` (configs 3-4; DiffusionField + agents)
    kinetics (external from the previous step: the reference's one-step lag)
    -> gather external := pre-step field at the agent's bin
    -> diffusion substeps -> exchange scatter in agent order.

Step order and quirks follow SURVEY.md Appendix A.5.
"""

from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from lens_amd import native
from lens_amd.configs import initial_conc
from lens_amd.kinetics import KineticsEngine
from lens_amd.lattice import Lattice, occupancy, N_A_LEGACY
from lens_amd.rate_law_compiler import compile_rate_laws, RateLawTable


def mmol_to_counts_from_mass(mass_fg, density_g_per_L=1100.0, avogadro=N_A_LEGACY):
    """DeriveGlobals: (N_A/mol * mass/density).to('L/mmol') (derive_globals.py:219-220)."""
    return avogadro * (mass_fg / density_g_per_L * 1e-15) * 1e-3


class Colony:
    def __init__(self, config, n_agents: int, *, capacity: Optional[int] = None, device=None,
                 integrator: str = 'dopri5', rtol: float = 1e-8, atol: float = 1e-12,
                 max_steps: int = 100000, environment='held', env_volume_L: float = 1e-14,
                 avogadro: float = N_A_LEGACY, exchange: str = 'sorted', mass_fg: float = 1339.0,
                 table: Optional[RateLawTable] = None, specialize: bool = False):
        if integrator not in ('euler', 'dopri5'):
            raise ValueError('integrator must be euler or dopri5')
        if exchange not in ('sorted', 'atomic'):
            raise ValueError('exchange must be sorted or atomic')
        self.config = config
        self.table = table or compile_rate_laws(config['reactions'], config['kinetic_parameters'])
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.engine = KineticsEngine(self.table, self.device)
        if specialize and integrator == 'dopri5':
            self.engine.specialize()     # straight-line rate laws (hiprtc), bit-identical results
        self.n = int(n_agents)
        self.ld = int(capacity or n_agents)
        if self.n > self.ld:
            raise ValueError('capacity < n_agents')
        self.integrator, self.rtol, self.atol, self.max_steps = integrator, rtol, atol, max_steps
        self.avogadro = avogadro
        self.exchange_mode = exchange
        t, ld, dev = self.table, self.ld, self.device
        z = lambda *shape, dtype=torch.float64: torch.zeros(shape, dtype=dtype, device=dev)
        self.params = torch.from_numpy(np.repeat(t.param_defaults[:, None], ld, axis=1)).to(dev).contiguous()
        self.conc = torch.from_numpy(initial_conc(t, config.get('initial_state', {}), ld)).to(dev).contiguous()
        self.m2c = torch.full((ld,), mmol_to_counts_from_mass(mass_fg, avogadro=avogadro),
                              dtype=torch.float64, device=dev)
        self.flux = z(t.n_reactions, ld)
        self.counts = z(t.n_ext, ld, dtype=torch.int64)
        self.status = z(ld, dtype=torch.int32)
        self.nsteps = z(ld, dtype=torch.int32)
        self.h_state = z(ld)
        self.time = 0.0
        self.lattice: Optional[Lattice] = None
        self.environment = environment
        if isinstance(environment, Lattice):
            self.lattice = environment
            self._setup_maps(self.lattice.molecules)
            self.location = z(2, ld)
            self.bin_lin = z(ld, dtype=torch.int32)
            self.bin_ix = z(ld, dtype=torch.int32)
        elif environment == 'nonspatial':
            mols = []
            for e in t.external_ids + [k[1] for k in t.species if k[0] == 'external']:
                if e not in mols:
                    mols.append(e)
            self._setup_maps(mols)
            self.env_molecules = mols
            self.env_fields = torch.ones((len(mols), ld), dtype=torch.float64, device=dev)
            depth_um = env_volume_L * 1e15                     # V / (1 um * 1 um)
            bin_volume = (depth_um * 1.0 * 1.0) * 1e-15 / 1    # get_bin_volume([1,1],[1,1],depth)
            self.env_binvol_avogadro = bin_volume * avogadro
            self.env_bins = torch.arange(ld, dtype=torch.int32, device=dev)
            self._env_to_external()          # derivers run once at t = 0
        elif environment != 'held':
            raise ValueError('environment must be held, nonspatial or a Lattice')

    # -- maps between SoA rows and field planes ---------------------------------
    def _setup_maps(self, molecules):
        t = self.table
        gf, gr, xc, xf = [], [], [], []
        for f, mol in enumerate(molecules):
            key = ('external', mol)
            if key in t.species:
                gf.append(f)
                gr.append(t.species.index(key))
        for e, mol in enumerate(t.external_ids):
            if mol in molecules:
                xc.append(e)
                xf.append(molecules.index(mol))
        i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=self.device)
        self.map_gather_field, self.map_gather_row = i32(gf), i32(gr)
        self.map_exch_count, self.map_exch_field = i32(xc), i32(xf)

    # -- state I/O ----------------------------------------------------------------
    def set_agents(self, params=None, conc=None, mmol_to_counts=None, location=None):
        """Upload per-agent arrays ([rows, n] numpy or torch; columns 0..n-1)."""
        def put(dst, src):
            src = torch.as_tensor(src, dtype=dst.dtype)
            if src.dim() == 1:
                dst[:self.n].copy_(src[:self.n].to(self.device))
            else:
                dst[:, :self.n].copy_(src[:, :self.n].to(self.device))
        if params is not None:
            put(self.params, params)
        if conc is not None:
            put(self.conc, conc)
        if mmol_to_counts is not None:
            put(self.m2c, mmol_to_counts)
        if location is not None:
            if self.lattice is None:
                raise ValueError('locations need a lattice environment')
            put(self.location, location)
            self.refresh_bins()

    def refresh_bins(self):
        """Recompute bin sites and the agent-ordered bin occupancy (after moves)."""
        lat = self.lattice
        lat.bin_sites(self.location, self.n, self.bin_lin, self.bin_ix)
        ix = self.bin_ix[:self.n]
        if self.n and (int(ix.min()) < lat.row_lo_global or int(ix.max()) >= lat.row_hi_global):
            raise ValueError('agents outside this rank\'s row band: route them first')
        self.occ = occupancy(self.bin_lin, self.n)

    def gather_external(self):
        """external := field at the agent's bin (get_local_environments)."""
        self.lattice.gather(self.bin_lin, self.n, self.map_gather_field, self.map_gather_row, self.conc)

    def _env_to_external(self):
        if self.map_gather_field.numel():
            native.check(native._lib.vk_gather(
                native.ptr(self.env_fields), self.ld, native.ptr(self.env_bins), self.n,
                native.ptr(self.map_gather_field), native.ptr(self.map_gather_row),
                int(self.map_gather_field.numel()), native.ptr(self.conc), self.ld,
                native.stream_handle()), 'vk_gather')

    # -- one timestep -------------------------------------------------------------
    def kinetics(self, dt: float):
        if self.integrator == 'euler':
            self.engine.euler(dt, self.params, self.conc, self.m2c, self.n, self.flux, self.counts,
                              self.status)
        else:
            self.engine.dopri5(dt, self.params, self.conc, self.m2c, self.n, self.h_state, self.rtol,
                               self.atol, self.max_steps, self.flux, self.counts, self.status,
                               self.nsteps)

    def step(self, dt: float = 1.0, halo_exchange=None, allreduce=None, timing=None):
        """One timestep.  ``timing`` (optional) = {'kin': (ev0, ev1), 'diff': (ev0, ev1)}
        of torch.cuda.Events recorded on the launch stream around those kernels."""
        timing = timing or {}
        if 'kin' in timing:
            timing['kin'][0].record()
        self.kinetics(dt)
        if 'kin' in timing:
            timing['kin'][1].record()
        if self.lattice is not None:
            lat = self.lattice
            self.gather_external()                       # pre-step field (one-step lag)
            lat.diffuse(dt, halo_exchange=halo_exchange, allreduce=allreduce,
                        events=timing.get('diff'))
            if self.map_exch_count.numel():
                if self.exchange_mode == 'sorted':
                    lat.exchange_sorted(self.occ, self.counts, self.map_exch_count, self.map_exch_field)
                else:
                    lat.exchange_atomic(self.bin_lin, self.n, self.counts, self.map_exch_count,
                                        self.map_exch_field)
        elif self.environment == 'nonspatial':
            if self.map_exch_count.numel():
                native.check(native._lib.vk_exchange_atomic(
                    native.ptr(self.env_fields), self.ld, native.ptr(self.env_bins), self.n,
                    native.ptr(self.counts), self.ld, native.ptr(self.map_exch_count),
                    native.ptr(self.map_exch_field), int(self.map_exch_count.numel()),
                    self.env_binvol_avogadro, native.stream_handle()), 'vk_exchange_atomic')
            self._env_to_external()
        self.time += dt

    def check_status(self):
        st = self.status[:self.n]
        bad = torch.nonzero(st).flatten()
        if bad.numel():
            a = int(bad[0])
            raise FloatingPointError('agent %d: kernel status %d' % (a, int(st[a])))

    # -- views ----------------------------------------------------------------------
    def species(self, port, name):
        return self.conc[self.table.species.index((port, name)), :self.n]

    def snapshot(self):
        """Host copy of the emitted state ({port: {state: ndarray[n]}})."""
        out = {}
        c = self.conc[:, :self.n].cpu().numpy()
        for s, (port, name) in enumerate(self.table.species):
            out.setdefault(port, {})[name] = c[s].copy()
        f = self.flux[:, :self.n].cpu().numpy()
        out['fluxes'] = {rid: f[r].copy() for r, rid in enumerate(self.table.reaction_ids)}
        return out

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

With a :class:`~lens_amd.cells.CellModel` the step continues like the
reference's deriver pass: the growth process (from the step-start state),
then TreeMass / DeriveGlobals (``mmol_to_counts`` for the next step's
exchange), then division: survivors keep their order, daughters are appended
in mother order, every per-agent array is gathered once with its divider.
"""

from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from lens_amd import native
from lens_amd.cells import CellModel, lineage_ids
from lens_amd.configs import initial_conc
from lens_amd.kinetics import KineticsEngine
from lens_amd.lattice import Lattice, occupancy, segment_index, N_A_LEGACY
from lens_amd.rate_law_compiler import compile_rate_laws, RateLawTable


def mmol_to_counts_from_mass(mass_fg, density_g_per_L=1100.0, avogadro=N_A_LEGACY):
    """DeriveGlobals: (N_A/mol * mass/density).to('L/mmol') (derive_globals.py:219-220)."""
    return avogadro * (mass_fg / density_g_per_L * 1e-15) * 1e-3


class Colony:
    def __init__(self, config, n_agents: int, *, capacity: Optional[int] = None, device=None,
                 integrator: str = 'dopri5', rtol: float = 1e-8, atol: float = 1e-12,
                 max_steps: int = 100000, environment='held', env_volume_L: float = 1e-14,
                 avogadro: float = N_A_LEGACY, exchange: str = 'sorted', mass_fg: float = 1339.0,
                 table: Optional[RateLawTable] = None, specialize: bool = False,
                 cells: Optional[CellModel] = None, agent_ids=None):
        if integrator not in ('euler', 'dopri5'):
            raise ValueError('integrator must be euler or dopri5')
        if exchange not in ('sorted', 'atomic'):
            raise ValueError('exchange must be sorted or atomic')
        self.config = config
        self.table = table or compile_rate_laws(config['reactions'], config['kinetic_parameters'])
        self.device = native.resolve_device(device)
        # lattice colonies: optionally run kinetics + gather on a side stream
        # beside the diffusion passes (step()); results are identical either way.
        # Off by default: on one MI355X the C4 stencil passes already fill the
        # chip, and the overlap measured 2.1003 -> 2.1001 ms per step (r01k)
        self.overlap_kinetics = False
        self._side_stream = torch.cuda.Stream(self.device) if self.device.type == 'cuda' else None
        # banded lattices: the first halo exchange of a step runs on a comm stream
        # beside the kinetics and the gather (it writes only halo rows)
        self.overlap_halo = True
        # lattice colonies stored in bin order: the gather and the exchange can ride on
        # the first and final diffusion passes (vk_diffuse_coupled; same results).  Off
        # by default: on one MI355X at C4 the coupled step ran 1.533 ms against 1.511
        # with the separate launches (profiles/r04/r04h/couple_ab.log)
        self.fuse_coupling = False
        # lattice colonies on the specialised agent-per-lane DP45 kernel: the gather of
        # the next step's local environment rides on the kinetics launch
        # (vk_step_dopri5_gather; the same values as vk_gather right after it)
        self.fuse_gather = True
        self._couple = None
        self.last_step_coupled = False
        self._comm_stream = torch.cuda.Stream(self.device) if self.device.type == 'cuda' else None
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
        self.step_index = 0
        self._layout = 0             # bumped when step buffers are reallocated (Colony.capture checks it)
        self.lattice: Optional[Lattice] = None
        self.router = None       # distributed.AgentRouter (row-banded multi-rank lattice colonies)
        self.ordinal = None      # global single-rank-order key (set by the router)
        self.location = None
        self.env_fields = None
        self.cells = cells
        if cells is not None:
            rows, m2c = cells.initial_rows(ld)
            self.cell = torch.from_numpy(rows).to(dev).contiguous()
            self.m2c.copy_(torch.from_numpy(m2c))
            self.divide = z(ld, dtype=torch.int32)
            self.roots = [str(i) for i in range(self.n)] if agent_ids is None else [str(x) for x in agent_ids]
            if len(self.roots) != self.n:
                raise ValueError('agent_ids must name every agent')
            self.lin_root = torch.arange(ld, dtype=torch.int32, device=dev)
            self.lin_depth = z(ld, dtype=torch.int32)
            self.lin_path = z(ld, dtype=torch.int64)
            self._n_out = torch.zeros(1, dtype=torch.int64, device=dev)
            self._overflow = torch.zeros(1, dtype=torch.int32, device=dev)
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

    def agent_array_names(self):
        """Every per-agent array (agent = column), as attribute names: what
        division gathers and the router migrates."""
        names = ['params', 'conc', 'm2c', 'flux', 'counts', 'status', 'nsteps', 'h_state']
        if self.location is not None:
            names.append('location')
        if self.cells is not None:
            names += ['cell', 'divide', 'lin_root', 'lin_depth', 'lin_path']
        if self.ordinal is not None:
            names.append('ordinal')
        if self.env_fields is not None:
            names.append('env_fields')      # NonSpatialEnvironment: each agent's own 1x1 field
        return names

    def refresh_bins(self):
        """Recompute bin sites and the agent-ordered bin occupancy (after moves).
        A row-banded colony with a router first moves agents that left this
        rank's band to their owner (a collective: every rank calls it)."""
        lat = self.lattice
        if self.router is not None:
            self.router.route()
        lat.bin_sites(self.location, self.n, self.bin_lin, self.bin_ix)
        ix = self.bin_ix[:self.n]
        if self.n and (int(ix.min()) < lat.row_lo_global or int(ix.max()) >= lat.row_hi_global):
            raise ValueError('agents outside this rank\'s row band: attach a distributed.AgentRouter '
                             '(division moves daughters across band edges)')
        self.occ = occupancy(self.bin_lin, self.n, getattr(self, 'agent_order', None))
        self._update_coupling()
        self._layout += 1            # captured graphs hold the old occupancy buffers

    def _update_coupling(self):
        """The segment index of the coupled passes (vk_diffuse_coupled), kept only
        while the agents are stored in bin order on a whole, unbanded plane and
        each plane gathers into / takes counts from at most one SoA row."""
        self._couple = None
        lat, n = self.lattice, self.n
        if lat is None or self.cells is not None or self.router is not None or n == 0:
            return
        if lat.pad_top or lat.pad_bot or not (lat.edge_top and lat.edge_bot):
            return
        # stored in bin order, and within a bin in the exchange's agent order
        # (occupancy: agent_order after sort_by_bin, else the column order)
        b = self.bin_lin[:n].to(torch.int64)
        key = getattr(self, 'agent_order', None)
        if n > 1:
            same = b[1:] == b[:-1]
            ok = (b[1:] > b[:-1]) | (same & (key[1:n] > key[:n - 1]) if key is not None else same)
            if not bool(ok.all()):
                return
        nf = len(lat.molecules)
        rows = []
        for fields, srcs in ((self.map_gather_field, self.map_gather_row), (self.map_exch_field, self.map_exch_count)):
            r = [-1] * nf
            for f, x in zip(fields.tolist(), srcs.tolist()):
                if r[f] != -1:
                    return
                r[f] = x
            rows.append(r)
        self._couple = (segment_index(self.bin_lin, n, lat.rows_local, lat.ny), rows[0], rows[1])

    def sort_by_bin(self):
        """Store the agents in bin order, so that the exchange scatter and the
        gather read the per-agent arrays and the lattice as streams instead of
        scattered lines.  The sort key is (bin, reference order): agents sharing
        a bin stay in the reference's relative order, and the exchange
        occupancy keeps ordering each bin by ``self.agent_order`` after later
        moves (refresh_bins), so every result is unchanged -- the exchange adds
        a bin's agents in the reference's agent order, and agents do not
        interact otherwise.  ``self.agent_order[k]`` is the index (in the
        layout before the first sort) of the agent now stored in column k.
        Sort again after agents move to keep the streams.  Colonies whose agent
        order is itself a result -- division appends daughters in mother order,
        a row band's router keeps the single-rank order -- keep their layout."""
        if self.lattice is None:
            raise ValueError('sort_by_bin: a lattice colony')
        if self.cells is not None or self.router is not None:
            raise ValueError('sort_by_bin: division and routed bands keep the reference agent order')
        n = self.n
        prev = getattr(self, 'agent_order', None)
        key = prev if prev is not None else torch.arange(n, dtype=torch.int64, device=self.device)
        by_key = torch.sort(key[:n], stable=True).indices
        perm = by_key[torch.sort(self.bin_lin[:n].to(torch.int64)[by_key], stable=True).indices]
        for name in self.agent_array_names() + ['bin_lin', 'bin_ix']:
            t = getattr(self, name)
            if t.dim() == 1:
                t[:n] = t[:n][perm]
            else:
                t[:, :n] = t[:, :n][:, perm]
        self.agent_order = key[perm]
        self.occ = occupancy(self.bin_lin, n, self.agent_order)
        self._update_coupling()
        self._layout += 1            # captured graphs hold the old occupancy buffers
        return self.agent_order

    def _gather_fused(self):
        """Whether this step's kinetics launch also does the gather."""
        return (self.fuse_gather and self.lattice is not None and self.integrator == 'dopri5' and
                self.engine.default_variant() == 2 and 0 < self.map_gather_field.numel() <= 8)

    def kinetics_and_gather(self, dt: float):
        """kinetics(dt) then gather_external(), as one launch when the kernel allows."""
        if not self._gather_fused():
            self.kinetics(dt)
            self.gather_external()
            return
        lat = self.lattice
        self.engine.dopri5_gather(dt, self.params, self.conc, self.m2c, self.n, self.h_state, self.rtol, self.atol,
                                  self.max_steps, self.flux, self.counts, self.status, self.nsteps, lat.fields,
                                  lat.field_stride, self.bin_lin, self.map_gather_field, self.map_gather_row)
        if getattr(self, 'attempts', None) is not None:
            self.attempts += self.nsteps[:self.n].sum()

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
    def count_attempts(self, on: bool = True):
        """Accumulate DP45 attempts (accepted + rejected steps) of every agent
        into ``self.attempts`` (device int64), summed right after the kinetics
        launch -- before division copies a mother's ``nsteps`` into both
        daughters (bench flop accounting)."""
        self.attempts = torch.zeros((), dtype=torch.int64, device=self.device) if on else None

    def kinetics(self, dt: float):
        if self.integrator == 'euler':
            self.engine.euler(dt, self.params, self.conc, self.m2c, self.n, self.flux, self.counts,
                              self.status)
        else:
            self.engine.dopri5(dt, self.params, self.conc, self.m2c, self.n, self.h_state, self.rtol,
                               self.atol, self.max_steps, self.flux, self.counts, self.status,
                               self.nsteps)
            if getattr(self, 'attempts', None) is not None:
                self.attempts += self.nsteps[:self.n].sum()

    def _step_buffers(self, k):
        t, ld = self.table, self.ld
        if getattr(self, 'flux_steps', None) is None or self.flux_steps.shape[0] != k:
            self.flux_steps = torch.zeros((k, t.n_reactions, ld), dtype=torch.float64, device=self.device)
            self.counts_steps = torch.zeros((k, t.n_ext, ld), dtype=torch.int64, device=self.device)
            self.nsteps_steps = torch.zeros((k, ld), dtype=torch.int32, device=self.device)
            self._layout += 1

    def step_many(self, dt: float = 1.0, steps: int = 1):
        """``steps`` timesteps of a colony whose agents do not couple between
        steps (environment 'held', no cells, DP45 with the specialised kernel)
        in ONE launch (vk_step_dopri5_multi): each step equals :meth:`step`
        bit for bit.  Every step's fluxes, exchange counts and attempts stay in
        ``flux_steps`` [steps, R, ld], ``counts_steps`` [steps, E, ld] and
        ``nsteps_steps`` [steps, ld]; ``flux`` / ``counts`` / ``nsteps`` view
        the last step's."""
        if self.environment != 'held' or self.cells is not None or self.integrator != 'dopri5':
            raise ValueError('step_many: held externals, no division, DP45 (agents must not couple between steps)')
        k = int(steps)
        self._step_buffers(k)
        self.engine.dopri5_multi(dt, k, self.params, self.conc, self.m2c, self.n, self.h_state, self.rtol,
                                 self.atol, self.max_steps, self.flux_steps, self.counts_steps, self.status,
                                 self.nsteps_steps)
        self.flux, self.counts, self.nsteps = self.flux_steps[k - 1], self.counts_steps[k - 1], self.nsteps_steps[k - 1]
        if getattr(self, 'attempts', None) is not None:
            self.attempts += self.nsteps_steps[:, :self.n].sum()
        self.time += dt * k
        self.step_index += k

    def step(self, dt: float = 1.0, halo_exchange=None, allreduce=None, timing=None, stamp=None):
        """One timestep.  ``timing`` (optional) = {'kin': (ev0, ev1), 'diff': (ev0, ev1)}
        of torch.cuda.Events recorded on the launch stream around those kernels.
        ``stamp`` (optional, a callable of 0 / 1 / 2) writes a device timestamp
        on the launch stream before the kinetics, after it, and at the end of
        the step (bench instrumentation that also works inside a captured graph)."""
        timing = {k: v for k, v in (timing or {}).items() if v is not None}
        if stamp is not None:
            stamp(0)
        if self.lattice is not None and self.overlap_kinetics:
            # kinetics + gather read only the pre-step field and agent state, so
            # they run on a side stream beside the diffusion passes; the pass
            # that overwrites the field waits for the gather, the exchange for
            # the counts (both through one event)
            lat, main = self.lattice, torch.cuda.current_stream(self.device)
            side = self._side_stream
            side.wait_stream(main)                       # previous step's writers
            with torch.cuda.stream(side):
                if 'kin' in timing:
                    timing['kin'][0].record()
                self.kinetics_and_gather(dt)             # + the pre-step field (one-step lag)
                if 'kin' in timing:
                    timing['kin'][1].record()
                done = torch.cuda.Event()
                done.record()
            lat.diffuse(dt, halo_exchange=halo_exchange, allreduce=allreduce,
                        events=timing.get('diff'), before_final=lambda: main.wait_event(done))
            self._step_exchange()
            self._finish_step(dt)
            return
        halo_done = None
        if (self.lattice is not None and halo_exchange is not None and self.overlap_halo and
                self._comm_stream is not None and (self.lattice.pad_top or self.lattice.pad_bot)):
            halo_done = self.lattice.exchange_first_halo(dt, halo_exchange, self._comm_stream)
        if 'kin' in timing:
            timing['kin'][0].record()
        coupled = (self.lattice is not None and halo_done is None and halo_exchange is None and
                   self.fuse_coupling and self._couple is not None and self.exchange_mode == 'sorted' and
                   self.lattice.coupled_plan_ok(dt))
        fused = self.lattice is not None and not coupled and self._gather_fused()
        if fused:
            self.kinetics_and_gather(dt)                     # + the pre-step field (one-step lag)
        else:
            self.kinetics(dt)
        if 'kin' in timing:
            timing['kin'][1].record()
        if stamp is not None:
            stamp(1)
        if self.lattice is not None:
            lat = self.lattice
            if not (halo_done is None and halo_exchange is None and self._coupled_step(dt, allreduce, timing)):
                if not fused:
                    self.gather_external()                   # pre-step field (one-step lag)
                # with the first halo exchange in flight, the band's interior passes run
                # first and the launch stream waits for the halo before the edge passes
                lat.diffuse(dt, halo_exchange=halo_exchange, allreduce=allreduce,
                            events=timing.get('diff'), halo_event=halo_done)
                self._step_exchange()
        elif self.environment == 'nonspatial':
            if self.map_exch_count.numel():
                native.check(native._lib.vk_exchange_atomic(
                    native.ptr(self.env_fields), self.ld, native.ptr(self.env_bins), self.n,
                    native.ptr(self.counts), self.ld, native.ptr(self.map_exch_count),
                    native.ptr(self.map_exch_field), int(self.map_exch_count.numel()),
                    self.env_binvol_avogadro, native.stream_handle()), 'vk_exchange_atomic')
            self._env_to_external()
        self._finish_step(dt)
        if stamp is not None:
            stamp(2)

    # -- multi-rate advance (Experiment.update, experiment.py:1351-1450) -------------
    def run(self, interval: float, kinetics_dt: float = 1.0, diffusion_dt: float = 1.0, halo_exchange=None,
            allreduce=None):
        """Advance a lattice colony by ``interval`` with the kinetics and the
        diffusion field on their own clocks (each agent's kinetics process's
        ``time_step``, the DiffusionField's ``time_step``), scheduled as the
        reference's Experiment.update does: a process runs when its front time
        <= time, with timestep = min(front + dt, interval) - front, and computes
        its update from the state at that moment; the global step is the
        smallest timestep that ran; updates whose front lands by then are
        applied in store order -- the environment's (fields += delta, every
        agent's external := the field at its bin when the diffusion ran)
        before the agents' (internal += delta or := the DP45 end state,
        fluxes, exchange into the field at apply time, in agent order).
        ``run(dt, dt, dt)`` equals :meth:`step` (dt) bit for bit.  A row-banded
        colony passes ``halo_exchange`` / ``allreduce`` as to :meth:`step`.
        Cells (growth / division) step with :meth:`step`."""
        if self.lattice is None:
            raise ValueError('run() schedules a lattice colony; use step() otherwise')
        if self.cells is not None:
            raise ValueError('growth and division run with step(): their derivers fix one clock')
        procs = [('diffusion', float(diffusion_dt)), ('kinetics', float(kinetics_dt))]   # store order
        front = {name: 0.0 for name, _ in procs}      # every update() call starts its fronts at 0
        pending = {}
        time = 0.0
        while time < interval:
            full_step = float('inf')
            for name, dt in procs:
                f = front[name]
                if f <= time:
                    future = min(f + dt, interval)
                    timestep = future - f
                    pending[name] = self._compute(name, timestep, halo_exchange, allreduce)
                    full_step = min(full_step, timestep)
                    front[name] = future
            future = time + full_step
            for name, _ in procs:
                if front[name] <= future and name in pending:
                    self._apply(name, pending.pop(name))
            time = future
            self.time += full_step
        self.step_index += 1
        return self

    def _compute(self, name, timestep, halo_exchange=None, allreduce=None):
        """A process's update from the current state, not yet applied."""
        lat, t = self.lattice, self.table
        if name == 'diffusion':
            delta = lat.diffuse_delta(timestep, allreduce=allreduce, halo_exchange=halo_exchange)
            ext = torch.empty((t.n_species, self.ld), dtype=torch.float64, device=self.device)
            lat.gather(self.bin_lin, self.n, self.map_gather_field, self.map_gather_row, ext)
            return delta, ext
        nd = t.n_dyn
        flux = torch.empty_like(self.flux)
        counts = torch.empty_like(self.counts)
        if self.integrator == 'euler':
            delta = torch.zeros((nd, self.ld), dtype=torch.float64, device=self.device)
            self.engine.euler(timestep, self.params, self.conc, self.m2c, self.n, flux, counts, self.status,
                              delta=delta)
            return 'delta', delta, flux, counts
        end = self.conc.clone()
        self.engine.dopri5(timestep, self.params, end, self.m2c, self.n, self.h_state, self.rtol, self.atol,
                           self.max_steps, flux, counts, self.status, self.nsteps)
        return 'set', end[:nd], flux, counts

    def _apply(self, name, update):
        lat, t = self.lattice, self.table
        n = self.n
        if name == 'diffusion':
            delta, ext = update
            own = slice(lat.row_lo, lat.row_hi)         # the accumulate updater: field + delta
            lat.fields[:, own] += delta[:, own]
            rows = self.map_gather_row.to(torch.int64)
            self.conc[rows, :n] = ext[rows, :n]         # external: set
            return
        mode, value, flux, counts = update
        nd = t.n_dyn
        if mode == 'delta':
            self.conc[:nd, :n] += value[:, :n]          # internal: accumulate
        else:
            self.conc[:nd, :n] = value[:, :n]
        self.flux.copy_(flux)
        self.counts.copy_(counts)
        self._step_exchange()

    def _coupled_step(self, dt, allreduce, timing):
        """gather + diffusion + exchange as one coupled pass sequence, when the
        colony and the plan allow it (vk_diffuse_coupled); False: nothing ran."""
        cp, lat = self._couple, self.lattice
        self.last_step_coupled = False
        if (cp is None or not self.fuse_coupling or self.exchange_mode != 'sorted' or
                not lat.coupled_plan_ok(dt)):
            return False
        seg, grow, crow = cp
        self.last_step_coupled = lat.diffuse_coupled(dt, self.bin_lin, self.n, seg, grow, self.conc, crow,
                                                     self.counts, allreduce=allreduce, events=timing.get('diff'))
        return self.last_step_coupled

    def _step_exchange(self):
        lat = self.lattice
        if self.map_exch_count.numel():
            if self.exchange_mode == 'sorted':
                lat.exchange_sorted(self.occ, self.counts, self.map_exch_count, self.map_exch_field)
            else:
                lat.exchange_atomic(self.bin_lin, self.n, self.counts, self.map_exch_count,
                                    self.map_exch_field)

    def _overlap_ok(self):
        """Whether :meth:`capture` can overlap a step's exchange with the next step's
        kinetics (and the uniform probe with the gather)."""
        lat = self.lattice
        return (lat is not None and self.cells is None and not self.overlap_kinetics and not self.fuse_coupling
                and self.device.type == 'cuda' and not (lat.pad_top or lat.pad_bot))

    def _captured_steps_overlapped(self, dt, steps, stamps):
        """The body of an overlapped capture (see :meth:`capture`).  Step k's exchange
        scatter reads the counts buffer its own kinetics wrote, and runs on a side stream
        while step k+1's kinetics writes the other buffer; the uniform probe runs on a
        second side stream beside the gather.  Every read of the planes (probe, gather,
        passes) waits for the previous exchange, so each step sees exactly the state a
        sequential step would."""
        lat = self.lattice
        if getattr(self, '_x_stream', None) is None:
            self._x_stream = torch.cuda.Stream(self.device)
            self._p_stream = torch.cuda.Stream(self.device)
        sx, sp = self._x_stream, self._p_stream
        bufs = (self.counts, self._counts_alt)
        pending = None
        for k in range(steps):
            stamp = None
            if stamps is not None:
                stamp = (lambda tag, k=k: native.check(native._lib.vk_timestamp(
                    native.ptr(stamps), 3 * k + tag, native.stream_handle()), 'vk_timestamp'))
                stamp(0)
            self.counts = bufs[(steps - 1 - k) % 2]   # the last step writes the colony's own buffer
            self.kinetics(dt)
            if stamp is not None:
                stamp(1)
            main = torch.cuda.current_stream(self.device)
            if pending is not None:
                main.wait_event(pending)             # the previous step's exchange landed
            sp.wait_stream(main)
            with torch.cuda.stream(sp):
                mm = lat.uniform_summary(None)       # the probe, beside the gather
            self.gather_external()                   # pre-step field (one-step lag)
            main.wait_stream(sp)
            lat.diffuse(dt, summary=mm)
            sx.wait_stream(main)
            with torch.cuda.stream(sx):
                self._step_exchange()                # this step's counts buffer
                pending = torch.cuda.Event()
                pending.record()
            self._finish_step(dt)
            if stamp is not None:
                stamp(2)
        torch.cuda.current_stream(self.device).wait_event(pending)

    def capture(self, dt: float = 1.0, steps: int = 1, stamps=None, steps_per_launch: int = 1, overlap=False):
        """Capture ``steps`` timesteps into one HIP graph (torch.cuda.CUDAGraph)
        and return a function that replays them.

        A small colony's step is a few short launches, and issuing them from
        Python costs more than running them (C2: 40 µs per step issued, 4.5 µs
        replayed). Replaying a captured graph leaves the host out of the loop.
        Only steps that take no host decision can be captured: no division (the
        host reads back the new agent count), no row band (its halo exchange
        is a host-driven collective), no NonSpatialEnvironment. A single-GPU
        lattice step qualifies (with ``overlap_kinetics`` too: the side stream
        forks from and joins the captured stream inside each step): the pass plan
        depends only on Δt, and the uniform-plane skip is read by the kernels
        from device memory. Capture records the launches without running them,
        so the colony state is unchanged until the first replay. The graph
        holds the buffers and the agent count of capture time: set_agents()
        values may change between replays (they are copied in place), but a
        re-binning of moved agents invalidates it (replay raises).
        ``steps_per_launch`` > 1 (a held colony without division) captures
        :meth:`step_many` launches of that many steps instead.
        ``stamps`` (optional, a device int64 tensor of 3 * steps) records each
        replayed step's segment boundaries (:meth:`step`'s ``stamp``) at
        [3k, 3k + 1, 3k + 2] -- vk_timestamp ticks, vk_wall_clock_khz per ms.
        ``overlap`` (a single-GPU lattice colony without division): within the graph,
        step k's exchange scatter runs on a side stream beside step k+1's kinetics (the
        two alternate between two counts buffers), and the uniform probe beside the
        gather.  The results are the sequential steps' bit for bit, and ``counts`` holds
        the last replayed step's counts.  Off by default: at C4 the overlapped kernels
        slow each other and each cross-stream dependency adds ~6 us, 1.518 against
        1.515 ms per step (profiles/r04/r04k)."""
        lat = self.lattice
        if (self.cells is not None or self.environment == 'nonspatial' or
                (lat is not None and (lat.pad_top or lat.pad_bot or not (lat.edge_top and lat.edge_bot)))):
            raise ValueError('Colony.capture: division, row bands and NonSpatialEnvironment take host decisions '
                             'per step and cannot be replayed from one graph (a row band: capture_banded)')
        if steps < 1:
            raise ValueError('Colony.capture: steps >= 1')
        spl = int(steps_per_launch)
        if spl > 1 and (stamps is not None or steps % spl):
            raise ValueError('Colony.capture: steps_per_launch must divide steps (and takes no stamps)')
        if spl > 1:
            self._step_buffers(spl)                 # allocated before the capture (graphs hold the pointers)
        overlap = bool(overlap) and self._overlap_ok() and spl == 1
        if overlap and (getattr(self, '_counts_alt', None) is None or self._counts_alt.shape != self.counts.shape):
            self._counts_alt = torch.zeros_like(self.counts)
        counts0 = self.counts
        graph = torch.cuda.CUDAGraph()
        t0, s0 = self.time, self.step_index
        layout, n = self._layout, self.n
        with torch.cuda.graph(graph):
            for k in range(steps // spl if spl > 1 else 0):
                self.step_many(dt, spl)
            if overlap:
                self._captured_steps_overlapped(dt, steps, stamps)
            for k in range(steps if spl == 1 and not overlap else 0):
                stamp = None
                if stamps is not None:
                    stamp = (lambda tag, k=k: native.check(native._lib.vk_timestamp(
                        native.ptr(stamps), 3 * k + tag, native.stream_handle()), 'vk_timestamp'))
                self.step(dt, stamp=stamp)
        self.time, self.step_index = t0, s0      # capture ran nothing
        if spl > 1:
            # step_many pointed flux / counts / nsteps at the last step's rows of the
            # step buffers, which is where every replay leaves them
            self.flux, self.counts, self.nsteps = (self.flux_steps[spl - 1], self.counts_steps[spl - 1],
                                                   self.nsteps_steps[spl - 1])
        else:
            self.counts = counts0

        def replay():
            # the graph holds raw device pointers and the agent count of capture time
            if self._layout != layout or self.n != n:
                raise RuntimeError('Colony.capture: the colony was re-laid out (agents moved or counted '
                                   'anew) after capture; capture again')
            graph.replay()
            self.time += dt * steps
            self.step_index += steps

        replay.graph = graph      # keep the graph (and its memory pool) alive with the replayer
        replay.stamps = stamps
        return replay

    def capture_banded(self, dt: float = 1.0, halo_exchange=None, allreduce=None):
        """Row-banded lattice colony (multi-GPU): capture each step's launch
        sequences between its collectives as HIP graphs and return a function
        that runs one step -- the collectives (halo exchange, the uniform-plane
        all-reduce) are issued eagerly, everything else is replayed.

        One step of :meth:`step` on a band is, in stream order: kinetics and the
        gather (while the first halo exchange runs on the communication
        stream), the uniform-plane probe, its all-reduce, then per halo block a
        halo exchange (the first one already done) and the block's fused
        passes, and the exchange scatter after the last block.  The segments
        between the collectives become graphs: [kinetics + gather + probe],
        then one graph per halo block (the last with the scatter).  The
        kernels and their arguments are the eager step's, so the results are
        bit-identical (tests/test_distributed_gpu.py).  As with :meth:`capture`,
        re-binned agents invalidate the graphs."""
        from lens_amd.lattice import n_substeps
        lat = self.lattice
        if lat is None or not (lat.pad_top or lat.pad_bot):
            raise ValueError('Colony.capture_banded: a row-banded lattice colony (use capture() otherwise)')
        if self.cells is not None or self.overlap_kinetics:
            raise ValueError('Colony.capture_banded: division and side-stream overlap take host decisions per step')
        if halo_exchange is None:
            raise ValueError('Colony.capture_banded: a row band needs its halo_exchange callback')
        n_sub = n_substeps(dt, lat.diffusion_dt)
        coeff_dt = lat.diffusion * min(dt, lat.diffusion_dt)
        lo_min = lat.row_lo if lat.edge_top else 0
        hi_max = lat.row_hi if lat.edge_bot else lat.rows_local
        blocks, j = [], 0
        while j < n_sub:
            cnt = min(lat.halo, n_sub - j)
            blocks.append((j, cnt))
            j += cnt
        layout, n = self._layout, self.n
        t0, s0 = self.time, self.step_index
        g_kin = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_kin):
            self.kinetics_and_gather(dt)                 # + the pre-step field (one-step lag)
            lat.uniform_summary(None)                    # the probe; its all-reduce is eager
        # the first block's interior needs no halo: it is its own graph, replayed while
        # the first halo exchange is in flight; the block's edges follow the halo
        # the overlap decision is taken once, here: g_blocks[0] holds only the edge
        # strips when the interior is split off, so step() must not re-read
        # self.overlap_halo / self._comm_stream (a later toggle would drop the interior)
        comm = self._comm_stream if self.overlap_halo else None
        g_interior = None
        if comm is not None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                j0, c0 = blocks[0]
                split = lat._run_part(j0, c0, n_sub, coeff_dt, lat.uniform, lo_min, hi_max, native.VK_PART_INTERIOR)
            g_interior = g if split else None
        g_blocks = []
        for b, (j, cnt) in enumerate(blocks):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if b == 0 and g_interior is not None:
                    lat._run_part(j, cnt, n_sub, coeff_dt, lat.uniform, lo_min, hi_max, native.VK_PART_EDGES)
                else:
                    lat._run_block(j, cnt, n_sub, coeff_dt, lat.uniform, lo_min, hi_max)
                if b == len(blocks) - 1:
                    self._step_exchange()
            g_blocks.append(g)
        self.time, self.step_index = t0, s0             # capture ran nothing

        def step():
            if self._layout != layout or self.n != n:
                raise RuntimeError('Colony.capture_banded: the colony was re-laid out after capture; capture again')
            main = torch.cuda.current_stream(self.device)
            halo_done = None
            if comm is not None:
                halo_done = lat.exchange_first_halo(dt, halo_exchange, comm)
            g_kin.replay()
            if allreduce is not None:
                allreduce(lat.uniform)
            if halo_done is not None:
                if g_interior is not None:
                    g_interior.replay()                  # beside the halo exchange
                main.wait_event(halo_done)
            else:
                halo_exchange(lat.state_buffer(0), blocks[0][1])
            for b, (j, cnt) in enumerate(blocks):
                if b:
                    halo_exchange(lat.state_buffer(j), cnt)
                g_blocks[b].replay()
            self.time += dt
            self.step_index += 1

        step.graphs = (g_kin, g_blocks)
        step.interior_graph = g_interior
        return step

    def _finish_step(self, dt):
        if self.cells is not None:
            self.grow_and_divide(dt)
        self.time += dt
        self.step_index += 1

    def set_cell_mass(self, mass):
        """Per-agent masses (fg) for agents 0..n-1 with their derived volume,
        length, surface area and mmol_to_counts (DeriveGlobals on each)."""
        cm = self.cells
        mass = np.ascontiguousarray(mass, dtype=np.float64)[:self.n]
        vol, m2c, length, area = cm.derive(mass)          # numpy: the same IEEE ops elementwise
        rows = self.cell[:, :self.n].cpu().numpy()
        rows[native.VK_CELL_MASS], rows[native.VK_CELL_VOLUME] = mass, vol
        rows[native.VK_CELL_LENGTH], rows[native.VK_CELL_SURFACE_AREA] = length, area
        self.cell[:, :self.n].copy_(torch.from_numpy(rows))
        self.m2c[:self.n].copy_(torch.from_numpy(np.ascontiguousarray(m2c)))

    # -- growth, derivers, division (a10-a13) ------------------------------------
    def grow_and_divide(self, dt: float):
        """Growth process + TreeMass/DeriveGlobals, then division.  Returns the
        number of mothers that divided."""
        cm, n = self.cells, self.n
        if n == 0 and self.router is None:
            return 0
        src = torch.empty(2 * n, dtype=torch.int32, device=self.device)
        kind = torch.empty(2 * n, dtype=torch.int32, device=self.device)
        n_out = 0
        if n:
            p = cm.vk_params(dt, self.step_index)
            u = None
            if cm.model == 'growth_protein' and cm.rng == 'stream':
                u = torch.from_numpy(cm.host_uniforms(n)).to(self.device)
            native.check(native._lib.vk_cell_step(
                ctypes.byref(p), n, self.ld, native.ptr(self.cell), native.ptr(self.m2c), native.ptr(u),
                native.ptr(self.lin_root), native.ptr(self.lin_depth), native.ptr(self.lin_path),
                native.ptr(self.divide), native.stream_handle()), 'vk_cell_step')
            scratch = torch.empty(int(native._lib.vk_divide_scratch_bytes(n)), dtype=torch.uint8,
                                  device=self.device)
            native.check(native._lib.vk_divide_plan(
                native.ptr(self.divide), n, native.ptr(src), native.ptr(kind), native.ptr(self._n_out),
                native.ptr(scratch), native.stream_handle()), 'vk_divide_plan')
            n_out = int(self._n_out.item())
        if self.router is not None:
            # collective every step: the global order of every rank's survivors
            # and daughters (AgentRouter.division_ordinals); then, if any rank
            # divided, daughters that left this band move to their owner
            new_ord, n_div = self.router.division_ordinals(self.ordinal[:n], self.divide[:n] != 0, src, kind,
                                                           n_out)
            if n_out != n:
                self._apply_division(n_out, src, kind, ordinal=new_ord)
            elif n_div:
                self.ordinal[:n] = new_ord
                self.refresh_bins()
            return n_out - n
        if n_out == n:
            return 0
        self._apply_division(n_out, src, kind)
        return n_out - n

    def _apply_division(self, n_out, src, kind, ordinal=None):
        ld_src = self.ld
        ld = max(self.ld, n_out)
        if n_out > self.ld:
            ld = max(n_out, int(self.ld * 1.25) + 64)
        dev, st = self.device, native.stream_handle()
        S, SP, Z = native.VK_DIVIDE_SET, native.VK_DIVIDE_SPLIT, native.VK_DIVIDE_ZERO

        def gather(t, divider=S, rows_slice=None):
            rows = 1 if t.dim() == 1 else t.shape[0]
            out = torch.empty((ld,) if t.dim() == 1 else (rows, ld), dtype=t.dtype, device=dev)
            native.check(native._lib.vk_divide_gather(
                n_out, native.ptr(src), native.ptr(kind), native.ptr(t), ld_src, native.ptr(out), ld, rows,
                t.element_size(), divider, st), 'vk_divide_gather')
            return out

        for name in ('params', 'conc', 'm2c', 'flux', 'counts', 'status', 'nsteps', 'h_state'):
            setattr(self, name, gather(getattr(self, name)))
        if self.env_fields is not None:
            self.env_fields = gather(self.env_fields)
            self.env_bins = torch.arange(ld, dtype=torch.int32, device=dev)
        cell = torch.empty((native.VK_CELL_ROWS, ld), dtype=torch.float64, device=dev)
        n_split = native.VK_CELL_ANGLE      # rows [0, angle) split, angle copied
        native.check(native._lib.vk_divide_gather(
            n_out, native.ptr(src), native.ptr(kind), native.ptr(self.cell), ld_src, native.ptr(cell), ld,
            n_split, 8, SP, st), 'vk_divide_gather(cell)')
        native.check(native._lib.vk_divide_gather(
            n_out, native.ptr(src), native.ptr(kind), self.cell.data_ptr() + n_split * ld_src * 8, ld_src,
            cell.data_ptr() + n_split * ld * 8, ld, native.VK_CELL_ROWS - n_split, 8, S, st),
            'vk_divide_gather(angle)')
        self.divide = gather(self.divide, Z)
        root = torch.empty(ld, dtype=torch.int32, device=dev)
        depth = torch.empty(ld, dtype=torch.int32, device=dev)
        path = torch.empty(ld, dtype=torch.int64, device=dev)
        native.check(native._lib.vk_divide_lineage(
            n_out, native.ptr(src), native.ptr(kind), native.ptr(self.lin_root), native.ptr(self.lin_depth),
            native.ptr(self.lin_path), native.ptr(root), native.ptr(depth), native.ptr(path),
            native.ptr(self._overflow), st), 'vk_divide_lineage')
        if self.location is not None:
            loc = torch.empty((2, ld), dtype=torch.float64, device=dev)
            native.check(native._lib.vk_divide_locations(
                n_out, native.ptr(src), native.ptr(kind), native.ptr(self.location), ld_src, native.ptr(loc), ld,
                native.ptr(cell), st), 'vk_divide_locations')
            self.location = loc
        self.cell, self.lin_root, self.lin_depth, self.lin_path = cell, root, depth, path
        if ordinal is not None:
            self.ordinal = torch.zeros(ld, dtype=torch.int64, device=dev)
            self.ordinal[:n_out] = ordinal
        self.n, self.ld = n_out, ld
        if self.lattice is not None:
            self.bin_lin = torch.zeros(ld, dtype=torch.int32, device=dev)
            self.bin_ix = torch.zeros(ld, dtype=torch.int32, device=dev)
            self.refresh_bins()
        if int(self._overflow.item()):
            raise OverflowError('a lineage exceeded 64 generations (phylogeny path bits)')

    def agent_ids(self):
        """Phylogeny ids of agents 0..n-1 (meta_division.py:15-18)."""
        if self.cells is None:
            return [str(a) for a in range(self.n)]
        return lineage_ids(self.roots, self.lin_root[:self.n].cpu().numpy(),
                           self.lin_depth[:self.n].cpu().numpy(), self.lin_path[:self.n].cpu().numpy())

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
        if self.cells is not None:
            c = self.cell[:, :self.n].cpu().numpy()
            out['global'] = {name: c[row].copy() for name, row in (
                ('mass', native.VK_CELL_MASS), ('volume', native.VK_CELL_VOLUME),
                ('length', native.VK_CELL_LENGTH), ('surface_area', native.VK_CELL_SURFACE_AREA),
                ('angle', native.VK_CELL_ANGLE))}
            out['global']['width'] = np.full(self.n, self.cells.width)
            out['global']['mmol_to_counts'] = self.m2c[:self.n].cpu().numpy().copy()
            out.setdefault('internal', {})['protein'] = c[native.VK_CELL_PROTEIN].copy()
        return out

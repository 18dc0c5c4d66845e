"""Device kinetics operators over SoA torch tensors (FP64, one agent per column).

Thin, shape-checked wrappers over the C ABI.  Layout (``include/vk_kinetics.h``):
``params[n_params, ld]``, ``conc[n_species, ld]``, ``mmol_to_counts[ld]``,
``flux[n_reactions, ld]``, ``counts[n_ext, ld]`` (int64); agents are columns
``0..n_agents-1``; rows follow :class:`~lens_amd.rate_law_compiler.RateLawTable`.
"""

from __future__ import annotations

import os
import ctypes

import torch

from lens_amd import native
from lens_amd.rate_law_compiler import RateLawTable

F64 = torch.float64


def _need(t, name, rows, ld, dtype, device):
    if not isinstance(t, torch.Tensor):
        raise TypeError('%s must be a torch tensor' % name)
    if t.dtype != dtype:
        raise TypeError('%s must be %s, got %s' % (name, dtype, t.dtype))
    if t.device.type != 'cuda' or (device is not None and t.device != device):
        raise ValueError('%s must live on %s' % (name, device))
    if not t.is_contiguous():
        raise ValueError('%s must be contiguous' % name)
    want = (rows, ld) if rows is not None else (ld,)
    if tuple(t.shape) != want:
        raise ValueError('%s has shape %s, kernel expects %s' % (name, tuple(t.shape), want))


class KineticsEngine:
    """A compiled network resident on one GPU."""

    def __init__(self, table: RateLawTable, device=None):
        self.table = table
        self.device = native.resolve_device(device)
        with torch.cuda.device(self.device):
            self.dev = native.DeviceTable(table)
        self.specialized = False

    def specialize(self):
        """Compile the network-specialised DP45 kernel (hiprtc) for this table.

        Afterwards :meth:`dopri5` defaults to variant 2 (straight-line rate
        laws, everything in VGPRs) instead of the generic table walk."""
        from lens_amd.codegen import dopri5_source, split_layout, wave_registers, wave_source
        if self.table.n_dyn + self.table.n_reactions > self.LANE_LIMIT:
            # too large for one lane: specialise the agent-per-wavefront kernel
            # instead, while its padded per-lane operands fit the register file
            if wave_registers(self.table) > self.WAVE_REGISTER_LIMIT:
                return self
            split = int(bool(self.WAVE_SPLIT_DEN) and split_layout(self.table) is not None)
            # 3 waves per SIMD where the split layout's estimate leaves room (C5: 162 -> 167
            # VGPRs, 16 spilled, 0.63 VALU busy); larger networks keep 2
            wpe = int(os.environ.get('VK_WAVE_WPE', 0)) or self.WAVE_WAVES_PER_SIMD or \
                (3 if split and wave_registers(self.table, True) <= 165 else 2)
            src = wave_source(self.table, wpe, self.WAVE_PAD_WRITES, self.WAVE_LDS_OPS, split,
                              int(os.environ.get('VK_WAVE_GROUP', self.WAVE_GROUP)))
        else:
            src = dopri5_source(self.table)
        with torch.cuda.device(self.device):
            native.check(native._lib.vk_table_specialize(self.dev.handle, src.encode()), 'vk_table_specialize')
        self.specialized = True
        return self

    LANE_LIMIT = 32   # integrated components an agent-per-lane kernel holds in VGPRs
    WAVE_REGISTER_LIMIT = 270   # codegen.wave_registers estimate beyond which variant 1 stays (spills)
    WAVE_PAD_WRITES = 1         # 1: branch-free LDS publishes (padding lanes write a scratch slot;
                                # C5 113.5 -> 111.9 ms, profiles/r03/r03e_c5_probe.log)
    WAVE_LDS_OPS = 0            # 1: denominator 1/Km and stoichiometry read from LDS tables (fewer VGPRs);
                                # 2: also the denominator member indices.  With split denominators
                                # (bit-identical): C5 98.6 / 113.6 ms at 3 waves/SIMD, 175.7 / 123.7 at 4,
                                # against 91.6 ms for 0 (profiles/r04/r04p_c5.log): occupancy is not what
                                # bounds the kernel
    WAVE_SPLIT_DEN = 1          # 1: the heaviest denominators split over lanes l and l + 32 (codegen.split_layout),
                                # summed in set order (bit-identical); C5 112.0 -> 87.3 ms at 3 waves/SIMD
                                # (profiles/r03/r03i_c5_probe.log)
    WAVE_GROUP = 2              # agents (waves) per workgroup of the specialised wavefront kernel: a
                                # workgroup's slots free only together, and an agent's attempt count
                                # varies 2x across a colony; C5 kinetics 37.5 ms at 4, 30.9 at 2,
                                # 30.9-31.1 at 1 (profiles/r06/c5grp; env VK_WAVE_GROUP overrides)
    WAVE_WAVES_PER_SIMD = None  # occupancy the specialised wavefront kernel is compiled for (env VK_WAVE_WPE
                                # overrides; with 2-agent workgroups 2 and 3 tie, 4 spills: profiles/r06/c5wpe);
                                # None: 3 with split
                                # denominators (190 -> 167 VGPRs, 16 spilled), else 2 (the batched gathers need
                                # 216 VGPRs; C5: 2 waves 120.5 ms, 3 waves spill, 224 ms)

    def default_variant(self) -> int:
        if self.table.n_dyn + self.table.n_reactions > self.LANE_LIMIT:
            return 3 if self.specialized else 1
        return 2 if self.specialized else 0

    # -- allocation helpers -------------------------------------------------
    def empty_like_agents(self, rows, ld, dtype=F64):
        shape = (rows, ld) if rows is not None else (ld,)
        return torch.zeros(shape, dtype=dtype, device=self.device)

    def _check_state(self, params, conc, n_agents):
        t = self.table
        ld = conc.shape[1]
        if not (0 <= n_agents <= ld):
            raise ValueError('n_agents must be in [0, ld]')
        _need(params, 'params', t.n_params, ld, F64, self.device)
        _need(conc, 'conc', t.n_species, ld, F64, self.device)
        return ld

    # -- operators ----------------------------------------------------------
    def fluxes(self, params, conc, n_agents=None, flux=None):
        n = conc.shape[1] if n_agents is None else n_agents
        ld = self._check_state(params, conc, n)
        if flux is None:
            flux = self.empty_like_agents(self.table.n_reactions, ld)
        _need(flux, 'flux', self.table.n_reactions, ld, F64, self.device)
        native.check(native._lib.vk_rate_fluxes(self.dev.handle, n, ld, native.ptr(params),
                                                native.ptr(conc), native.ptr(flux),
                                                native.stream_handle()), 'vk_rate_fluxes')
        return flux

    def euler(self, dt, params, conc, mmol_to_counts, n_agents=None, flux=None, counts=None,
              status=None, delta=None):
        """Reference Euler step; returns (flux, counts, status).

        ``delta=None`` updates ``conc`` in place; otherwise ``delta[n_dyn, ld]``
        receives the reference update values and ``conc`` is left untouched."""
        t = self.table
        n = conc.shape[1] if n_agents is None else n_agents
        ld = self._check_state(params, conc, n)
        _need(mmol_to_counts, 'mmol_to_counts', None, ld, F64, self.device)
        flux = self.empty_like_agents(t.n_reactions, ld) if flux is None else flux
        counts = self.empty_like_agents(t.n_ext, ld, torch.int64) if counts is None else counts
        status = self.empty_like_agents(None, ld, torch.int32) if status is None else status
        _need(flux, 'flux', t.n_reactions, ld, F64, self.device)
        _need(counts, 'counts', t.n_ext, ld, torch.int64, self.device)
        _need(status, 'status', None, ld, torch.int32, self.device)
        if delta is not None:
            _need(delta, 'delta', t.n_dyn, ld, F64, self.device)
        native.check(native._lib.vk_step_euler(
            self.dev.handle, n, ld, float(dt), native.ptr(params), native.ptr(conc),
            native.ptr(mmol_to_counts), native.ptr(delta), native.ptr(flux), native.ptr(counts),
            native.ptr(status), native.stream_handle()), 'vk_step_euler')
        return flux, counts, status

    def dopri5(self, dt, params, conc, mmol_to_counts, n_agents=None, h_state=None, rtol=1e-8,
               atol=1e-12, max_steps=100000, flux=None, counts=None, status=None, nsteps=None,
               variant=None, delta=None):
        """Adaptive DP5(4) over [0, dt] in place on ``conc``.

        ``variant``: 0 = agent per lane, generic table walk; 1 = agent per
        wavefront (default when n_dyn + n_reactions > 32); 2 = agent per lane,
        network-specialised; 3 = agent per wavefront, network-specialised
        (2 or 3 is the default once :meth:`specialize` ran).  Returns
        (flux = mean flux over dt, counts, status, nsteps)."""
        t = self.table
        if variant is None:
            variant = self.default_variant()
        n = conc.shape[1] if n_agents is None else n_agents
        ld = self._check_state(params, conc, n)
        _need(mmol_to_counts, 'mmol_to_counts', None, ld, F64, self.device)
        flux = self.empty_like_agents(t.n_reactions, ld) if flux is None else flux
        counts = self.empty_like_agents(t.n_ext, ld, torch.int64) if counts is None else counts
        status = self.empty_like_agents(None, ld, torch.int32) if status is None else status
        nsteps = self.empty_like_agents(None, ld, torch.int32) if nsteps is None else nsteps
        _need(flux, 'flux', t.n_reactions, ld, F64, self.device)
        _need(counts, 'counts', t.n_ext, ld, torch.int64, self.device)
        _need(status, 'status', None, ld, torch.int32, self.device)
        _need(nsteps, 'nsteps', None, ld, torch.int32, self.device)
        if h_state is not None:
            _need(h_state, 'h_state', None, ld, F64, self.device)
        if delta is not None:
            _need(delta, 'delta', t.n_dyn, ld, F64, self.device)
        opts = native.VkOdeOpts(float(rtol), float(atol), int(max_steps), int(variant))
        native.check(native._lib.vk_step_dopri5(
            self.dev.handle, n, ld, float(dt), ctypes.byref(opts), native.ptr(params),
            native.ptr(conc), native.ptr(mmol_to_counts), native.ptr(delta), native.ptr(h_state),
            native.ptr(flux),
            native.ptr(counts), native.ptr(status), native.ptr(nsteps), native.stream_handle()),
            'vk_step_dopri5')
        return flux, counts, status, nsteps

    # -- flop accounting (counted as the kernels execute) -----
    def dopri5_multi(self, dt, n_steps, params, conc, mmol_to_counts, n_agents=None, h_state=None, rtol=1e-8,
                     atol=1e-12, max_steps=100000, flux=None, counts=None, status=None, nsteps=None):
        """``n_steps`` consecutive DP5(4) agent-steps of ``dt`` in one launch
        (vk_step_dopri5_multi; agents that do not couple between steps, after
        :meth:`specialize`).  ``flux`` [n_steps, n_reactions, ld], ``counts``
        [n_steps, n_ext, ld] and ``nsteps`` [n_steps, ld] receive every step's
        outputs; ``conc`` / ``h_state`` the end state.  Each step equals one
        :meth:`dopri5` call (variant 2) bit for bit.  Returns (flux, counts,
        status, nsteps)."""
        t = self.table
        if self.default_variant() != 2:
            raise native.NativeError('dopri5_multi needs the specialised agent-per-lane kernel (specialize())')
        k = int(n_steps)
        n = conc.shape[1] if n_agents is None else n_agents
        ld = self._check_state(params, conc, n)
        _need(mmol_to_counts, 'mmol_to_counts', None, ld, F64, self.device)
        flux = torch.empty((k, t.n_reactions, ld), dtype=F64, device=self.device) if flux is None else flux
        counts = torch.empty((k, t.n_ext, ld), dtype=torch.int64, device=self.device) if counts is None else counts
        status = self.empty_like_agents(None, ld, torch.int32) if status is None else status
        nsteps = torch.empty((k, ld), dtype=torch.int32, device=self.device) if nsteps is None else nsteps
        for name, x, shape, dtype in (('flux', flux, (k, t.n_reactions, ld), F64),
                                      ('counts', counts, (k, t.n_ext, ld), torch.int64),
                                      ('nsteps', nsteps, (k, ld), torch.int32)):
            if tuple(x.shape) != shape or x.dtype != dtype or not x.is_contiguous() or x.device != self.device:
                raise ValueError('%s must be a contiguous %s %s tensor on %s' % (name, shape, dtype, self.device))
        _need(status, 'status', None, ld, torch.int32, self.device)
        if h_state is not None:
            _need(h_state, 'h_state', None, ld, F64, self.device)
        opts = native.VkOdeOpts(float(rtol), float(atol), int(max_steps), 2)
        native.check(native._lib.vk_step_dopri5_multi(
            self.dev.handle, n, ld, float(dt), k, ctypes.byref(opts), native.ptr(params), native.ptr(conc),
            native.ptr(mmol_to_counts), native.ptr(h_state), native.ptr(flux), t.n_reactions * ld,
            native.ptr(counts), t.n_ext * ld, native.ptr(status), native.ptr(nsteps), ld,
            native.stream_handle()), 'vk_step_dopri5_multi')
        return flux, counts, status, nsteps

    def dopri5_gather(self, dt, params, conc, mmol_to_counts, n_agents, h_state, rtol, atol, max_steps, flux,
                      counts, status, nsteps, fields, field_stride, bin_lin, map_field, map_row):
        """One :meth:`dopri5` step (variant 2) that also writes the next step's
        local environment: conc[map_row[i], a] := plane map_field[i] of ``fields``
        at bin_lin[a] (vk_step_dopri5_gather) -- what a vk_gather right after the
        kinetics writes."""
        if self.default_variant() != 2:
            raise native.NativeError('dopri5_gather needs the specialised agent-per-lane kernel (specialize())')
        n = int(n_agents)
        ld = self._check_state(params, conc, n)
        for name, x in (('mmol_to_counts', mmol_to_counts), ('h_state', h_state)):
            _need(x, name, None, ld, F64, self.device)
        _need(flux, 'flux', self.table.n_reactions, ld, F64, self.device)
        _need(counts, 'counts', self.table.n_ext, ld, torch.int64, self.device)
        _need(status, 'status', None, ld, torch.int32, self.device)
        _need(nsteps, 'nsteps', None, ld, torch.int32, self.device)
        n_map = int(map_field.numel())
        if n_map != int(map_row.numel()) or n_map > 8:
            raise ValueError('dopri5_gather: map_field / map_row of equal length <= 8')
        opts = native.VkOdeOpts(float(rtol), float(atol), int(max_steps), 2)
        native.check(native._lib.vk_step_dopri5_gather(
            self.dev.handle, n, ld, float(dt), ctypes.byref(opts), native.ptr(params), native.ptr(conc),
            native.ptr(mmol_to_counts), native.ptr(h_state), native.ptr(flux), native.ptr(counts),
            native.ptr(status), native.ptr(nsteps), native.ptr(fields), int(field_stride), native.ptr(bin_lin),
            native.ptr(map_field), native.ptr(map_row), n_map, native.stream_handle()), 'vk_step_dopri5_gather')
        return flux, counts, status, nsteps

    def dopri5_flops_per_attempt(self) -> int:
        """6 RHS evaluations + stage combinations + error norm per attempted step."""
        ny = self.table.n_dyn + self.table.n_reactions
        # stage inputs: 1+3+5+7+9 (a-rows with 1..5 terms: mul + fma chain + final fma),
        # solution (5 terms): 11, error (6 terms + h*): 12, norm: max/abs/fma/div/fma ~ 6
        per_component = 3 + 5 + 7 + 9 + 11 + 11 + 12 + 6
        return 6 * self.table.flops_rhs() + per_component * ny

    def dopri5_bytes_per_agent_step(self) -> int:
        """Algorithmic HBM bytes one agent-step of vk_step_dopri5 moves: reads
        conc[S] + params[P] + mmol_to_counts + h_state, writes the integrated
        rows [ND] + flux[R] + counts[n_ext] (int64) + h_state + status/nsteps (int32)."""
        t = self.table
        return 8 * (t.n_species + t.n_params + 2) + 8 * (t.n_dyn + t.n_reactions + t.n_ext + 1) + 8


"""Device-resident diffusion_field lattice (one row band per rank).

Restates ``DiffusionField`` (vivarium/processes/diffusion_field.py:209-407)
for a persistent SoA colony:

* fields live in HBM as ``[n_fields, rows_local, ny]`` FP64 planes, where
  ``rows_local = halo + owned + halo`` (axis 0 = x, as the reference's
  ndarray); a single-GPU lattice has ``halo = 0``;
* one step = the reference's ``diffusion_delta``: ``n_sub`` substeps of
  0.01 s (100 / 501 / 1001 for dt = 1 / 5 / 10 s, the reference's float
  accumulation quirk), uniform planes skipped, delta accumulated;
* multi-rank: ``halo_exchange`` callbacks refresh ``halo`` rows every
  ``halo`` substeps (k-deep halos) -- see
  :mod:`lens_amd.distributed`.
"""

from __future__ import annotations

import ctypes
from typing import Callable, Optional, Sequence

import torch

from lens_amd import native

N_A_LEGACY = 6.022140857e23   # constant the reference fixtures were produced with


def n_substeps(timestep: float, dt_max: float = 0.01) -> int:
    """Number of iterations of ``while t < timestep: t += dt`` (diffusion_field.py:388-392)."""
    t, dt, n = 0.0, min(timestep, dt_max), 0
    while t < timestep:
        t += dt
        n += 1
    return n


def stencil_depth(k: int = 0) -> int:
    """Set (1..15 odd, or 10) / query (0) the substeps fused per HBM pass; returns the previous.
    10 plans a block of a multiple of 10 substeps as 10-deep passes (vk_diffuse; in the
    exact mode the last one re-reads the step-start field, as the odd-depth plan's
    final pass does); every other call then runs at depth 9.  The default is 10."""
    native.load()
    return native._lib.vk_set_stencil_depth(int(k))


def stencil_kernel(variant: int = -1, rows: int = -1) -> int:
    """Select the fused-pass kernel and output rows per tile (0 = auto; -1 keeps);
    returns the previous variant.  Exact mode: 2 / 3 = lag-1 wave tiles with 3 / 6
    rows prefetched, 6 = 3 with streaming stores (the exact mode's default kernel).
    Tolerance mode: 20 = pair-sum passes (the default), 40 = the pair-sum 10-deep pass with its
    stages split over a workgroup's waves (the row-band choice; other depths run
    20), 6 = the 4-op FMA wave tiles.  Any other
    number (a retired variant) raises ValueError: the library would
    keep the previous variant, and a run would time something else than it names."""
    native.load()
    if int(variant) != -1 and int(variant) not in STENCIL_VARIANTS:
        raise ValueError('stencil kernel %d is not built (variants: %s)' % (variant, sorted(STENCIL_VARIANTS)))
    if int(rows) != -1 and not (int(rows) == 0 or 8 <= int(rows) <= 4096):
        raise ValueError('stencil tile rows must be 0 (auto) or 8..4096, got %d' % rows)
    return native._lib.vk_set_stencil_kernel(int(variant), int(rows))


STENCIL_VARIANTS = frozenset((2, 3, 6, 20, 40, 70))     # vk_set_stencil_kernel (vk_lattice.hip)


def stencil_mode(mode=None) -> str:
    """Set ('exact' | 'fma') / query (None) the fused passes' arithmetic; returns the
    previous mode.  'exact' (default) is bit-identical with the reference's
    scipy.ndimage.convolve update; 'fma' is the tolerance mode (vk_set_stencil_mode)."""
    native.load()
    names = ('exact', 'fma')
    code = -1 if mode is None else names.index(mode)
    return names[native._lib.vk_set_stencil_mode(code)]


class Lattice:
    def __init__(self, molecules: Sequence[str], n_bins, bounds, depth: float, diffusion: float,
                 device=None, row_band=None, halo: int = 0, avogadro: float = N_A_LEGACY,
                 initial=None):
        native.load()            # no CPU fallback: the kernels or an error
        self.molecules = list(molecules)
        self.n_bins = [int(n_bins[0]), int(n_bins[1])]
        self.bounds = [float(bounds[0]), float(bounds[1])]
        self.depth = float(depth)
        self.avogadro = float(avogadro)
        nx, ny = self.n_bins
        self.device = native.resolve_device(device)
        # DiffusionField.__init__ (diffusion_field.py:251-260)
        dx = self.bounds[0] / nx
        dy = self.bounds[1] / ny
        self.diffusion = diffusion / (dx * dy)
        self.diffusion_dt = 0.01
        # get_bin_volume (lattice_utils.py:57-58); exchange divides by bin_volume*N_A
        self.bin_volume = (self.depth * self.bounds[0] * self.bounds[1]) * 1e-15 / (nx * ny)
        self.binvol_avogadro = self.bin_volume * self.avogadro
        lo, hi = (0, nx) if row_band is None else (int(row_band[0]), int(row_band[1]))
        if not (0 <= lo < hi <= nx):
            raise ValueError('bad row band %r' % (row_band,))
        self.row_lo_global, self.row_hi_global = lo, hi
        self.halo = int(halo)
        self.edge_top = lo == 0
        self.edge_bot = hi == nx
        if not (self.edge_top and self.edge_bot) and self.halo < 1:
            # an interior band edge without halo rows would act as a reflecting
            # wall: the field would silently stop coupling across ranks
            raise ValueError('a row band %r of %d rows needs halo >= 1 (got %d)' % ((lo, hi), nx, self.halo))
        if self.halo > hi - lo and not (self.edge_top and self.edge_bot):
            raise ValueError('halo (%d) deeper than the band (%d rows)' % (self.halo, hi - lo))
        h = self.halo
        self.pad_top = 0 if self.edge_top else h
        self.pad_bot = 0 if self.edge_bot else h
        self.rows_local = self.pad_top + (hi - lo) + self.pad_bot
        self.ny = ny
        nf = len(self.molecules)
        shape = (nf, self.rows_local, ny)
        self.fields = torch.zeros(shape, dtype=torch.float64, device=self.device)
        self.work0 = torch.empty(shape, dtype=torch.float64, device=self.device)
        self.work1 = torch.empty(shape, dtype=torch.float64, device=self.device)
        self.uniform = torch.empty(2 * max(nf, 1), dtype=torch.float64, device=self.device)
        self._uniform_scratch = torch.empty(max(nf, 1) * native.VK_UNIFORM_BLOCKS, dtype=torch.int32,
                                            device=self.device)
        if initial is not None:
            for f, m in enumerate(self.molecules):
                if m in initial:
                    self.set_field(m, initial[m])
        else:
            self.fields.fill_(1.0)   # DiffusionField.ones_field default (diffusion_field.py:381-382)

    # local row index of the first owned row
    @property
    def row_lo(self) -> int:
        return self.pad_top

    @property
    def row_hi(self) -> int:
        return self.pad_top + (self.row_hi_global - self.row_lo_global)

    @property
    def field_stride(self) -> int:
        return self.rows_local * self.ny

    def set_field(self, molecule, values):
        """Set the owned rows of a plane from a global [nx, ny] array/tensor."""
        f = self.molecules.index(molecule)
        v = torch.as_tensor(values, dtype=torch.float64)
        if tuple(v.shape) != tuple(self.n_bins):
            raise ValueError('field %s must be %s' % (molecule, self.n_bins))
        band = v[self.row_lo_global:self.row_hi_global].to(self.device)
        self.fields[f, self.row_lo:self.row_hi].copy_(band)

    def owned(self, molecule=None):
        sl = self.fields[:, self.row_lo:self.row_hi]
        return sl if molecule is None else sl[self.molecules.index(molecule)]

    # -- diffusion ------------------------------------------------------------
    def uniform_summary(self, allreduce: Optional[Callable] = None):
        """Per-plane uniformity summary (vk_field_uniform): [2f] == [2f+1] iff plane f
        holds one value; ``allreduce`` (multi-rank) makes it the global test."""
        native.check(native._lib.vk_field_uniform(
            native.ptr(self.fields), len(self.molecules), self.field_stride, self.ny, self.row_lo,
            self.row_hi, native.ptr(self.uniform), native.ptr(self._uniform_scratch), native.stream_handle()),
            'vk_field_uniform')
        if allreduce is not None:
            allreduce(self.uniform)
        return self.uniform

    # substeps of the last launch that writes the field (one odd-depth pass;
    # see vk_diffuse's pass planner) -- split off so that work on another
    # stream that still READS the pre-step field can overlap all earlier passes
    FINAL_SPLIT = 7

    def diffuse(self, timestep: float, halo_exchange: Optional[Callable] = None,
                allreduce: Optional[Callable] = None, skip_uniform: bool = True, events=None,
                before_final: Optional[Callable] = None, halo_ready: bool = False, summary=None,
                halo_event=None):
        """Advance every plane by ``timestep`` (diffusion_field.py:385-407).

        ``halo_event``: the first block's halo exchange was started on another
        stream (:meth:`exchange_first_halo`) and this event marks its end: the
        block's interior passes (rows that need no halo) run first, the launch
        stream then waits for the event, and the edge passes finish the block
        (vk_diffuse_part; the same bits as the whole block).

        ``summary`` (optional): the vk_field_uniform summary of the step-start planes,
        taken by the caller (the probe is then not run again).

        ``halo_ready``: the caller already ran the first block's halo exchange
        (see :meth:`exchange_first_halo`; the launch stream waits for it).

        ``events`` = (start, end) torch.cuda.Events recorded on the launch
        stream around the substep kernels only (bench roofline timing).
        ``before_final`` is called (at enqueue time, on the host) before the
        first launch that overwrites ``fields``: the caller makes the launch
        stream wait there for readers of the pre-step field.  Every pass before
        it reads ``fields`` and writes only the work planes."""
        n_sub = n_substeps(timestep, self.diffusion_dt)
        coeff_dt = self.diffusion * min(timestep, self.diffusion_dt)
        # ``summary``: a uniform summary the caller already took of the step-start planes
        # (Colony's overlapped capture runs the probe beside the gather)
        mm = summary if summary is not None else (self.uniform_summary(allreduce) if skip_uniform else None)
        if events is not None:
            events[0].record()
        banded = bool(self.pad_top or self.pad_bot)
        if banded and halo_exchange is None:
            raise ValueError('a row band with halo rows needs a halo_exchange callback')
        k = self.halo if banded else n_sub
        lo_min = self.row_lo if self.edge_top else 0
        hi_max = self.row_hi if self.edge_bot else self.rows_local
        j = 0
        if halo_event is not None:
            halo_ready = True
        while j < n_sub:
            cnt = min(k, n_sub - j)
            if banded and not (halo_ready and j == 0):
                halo_exchange(self.state_buffer(j), cnt)
            if j == 0 and halo_event is not None:
                self._run_block_overlapped(j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max, halo_event)
                j += cnt
                continue
            split = 0
            if before_final is not None and j + cnt == n_sub:
                # unbanded: the planner's passes of [j, n_sub - 7) and [n_sub - 7, n_sub)
                # are the same passes as for [j, n_sub) (e.g. 100 = 8x9 + 3x7 | 7);
                # banded blocks are not split (their halo rows shrink over the block)
                if not banded and cnt > 2 * self.FINAL_SPLIT:
                    split = self.FINAL_SPLIT
                if split:
                    self._run_block(j, cnt - split, n_sub, coeff_dt, mm, lo_min, hi_max)
                before_final()
            if split:
                self._run_block(j + cnt - split, split, n_sub, coeff_dt, mm, lo_min, hi_max)
            else:
                self._run_block(j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max)
            j += cnt
        if events is not None:
            events[1].record()
        return n_sub

    def coupled_plan_ok(self, timestep: float) -> bool:
        """Whether :meth:`diffuse_coupled` can run this step: a whole plane (no
        row band, at most 8 planes) planned as two or more fused passes and no
        single-substep pass -- vk_diffuse's planner, restated (10-deep passes in
        the tolerance mode's depth-10 setting, else odd depths); the library makes
        the same decision and launches nothing otherwise."""
        if self.pad_top or self.pad_bot or not (self.edge_top and self.edge_bot) or len(self.molecules) > 8:
            return False
        n_sub = n_substeps(timestep, self.diffusion_dt)
        depth = native._lib.vk_set_stencil_depth(0)
        if depth == 10 and native._lib.vk_set_stencil_mode(-1) == 1 and n_sub % 10 == 0 and n_sub >= 20:
            return True
        depth = min(9 if depth == 10 else depth | 1, 15)
        passes = (n_sub + depth - 1) // depth
        if (passes & 1) != (n_sub & 1):
            passes += 1
        ks, j, left = [], 0, passes
        while j < n_sub:
            rem = n_sub - j
            k = (rem + left - 1) // left
            k += 1 - (k & 1)
            k = min(k, depth)
            while k > 1 and rem - k < left - 1:
                k -= 2
            ks.append(k)
            j += k
            left -= 1
        return len(ks) >= 2 and min(ks) >= 2

    def diffuse_coupled(self, timestep: float, bin_lin, n_agents: int, seg, gather_rows, conc, count_rows,
                        counts, allreduce: Optional[Callable] = None, events=None):
        """One whole-plane step (:meth:`diffuse`) whose first pass also gathers
        the agents' external concentrations from the pre-step planes
        (:meth:`gather`) and whose final pass also scatters the exchange counts
        into the new planes (:meth:`exchange_sorted`), with the same results
        (vk_diffuse_coupled).  The agents must be stored in bin order; ``seg``
        indexes them by 16-column segment (:func:`segment_index`).
        ``gather_rows`` / ``count_rows``: per plane, the SoA row it gathers
        into / takes its counts from (-1: none).  Check :meth:`coupled_plan_ok`
        first; returns False, having launched only the uniform probe, if the
        library declines the plan."""
        n_sub = n_substeps(timestep, self.diffusion_dt)
        coeff_dt = self.diffusion * min(timestep, self.diffusion_dt)
        mm = self.uniform_summary(allreduce)
        if events is not None:
            events[0].record()
        nf = len(self.molecules)
        rc = native._lib.vk_diffuse_coupled(
            native.ptr(self.fields), native.ptr(self.work0), native.ptr(self.work1), nf, self.field_stride,
            self.ny, self.rows_local, n_sub, coeff_dt, native.ptr(mm), native.ptr(bin_lin), native.ptr(seg),
            (self.ny + 15) // 16, int(n_agents), (ctypes.c_int32 * nf)(*gather_rows), native.ptr(conc),
            conc.shape[1], (ctypes.c_int32 * nf)(*count_rows), native.ptr(counts), counts.shape[1],
            self.binvol_avogadro, native.stream_handle())
        if rc == native.VK_ERR_LIMIT:
            return False
        native.check(rc, 'vk_diffuse_coupled')
        if events is not None:
            events[1].record()
        return True

    def exchange_first_halo(self, timestep: float, halo_exchange: Callable, stream):
        """Run the halo exchange of :meth:`diffuse`'s first block on ``stream``
        (a communication stream), so it overlaps what the launch stream does
        meanwhile -- kinetics and the gather read only owned rows, the exchange
        writes only halo rows.  Returns an event the launch stream must wait
        on before ``diffuse(..., halo_ready=True)``."""
        main = torch.cuda.current_stream(self.device)
        stream.wait_stream(main)                       # the previous step's field
        n_sub = n_substeps(timestep, self.diffusion_dt)
        with torch.cuda.stream(stream):
            halo_exchange(self.state_buffer(0), min(self.halo, n_sub))
            done = torch.cuda.Event()
            done.record()
        return done

    def diffuse_delta(self, timestep: float, delta=None, allreduce=None, halo_exchange: Optional[Callable] = None):
        """DiffusionField.next_update's field delta (diffusion_field.py:385-407):
        ``delta = new - field`` for every plane (zero for uniform planes) on the
        owned rows, with ``fields`` left as they were -- an accumulate updater
        applies it later (vk_diffuse_delta).  A row band runs the halo blocks of
        :meth:`diffuse` (``halo_exchange`` before each) and takes the delta in
        its last block."""
        banded = bool(self.pad_top or self.pad_bot)
        if banded and halo_exchange is None:
            raise ValueError('a row band with halo rows needs a halo_exchange callback')
        n_sub = n_substeps(timestep, self.diffusion_dt)
        coeff_dt = self.diffusion * min(timestep, self.diffusion_dt)
        mm = self.uniform_summary(allreduce)
        if delta is None:
            delta = torch.empty_like(self.fields)
        lo_min = self.row_lo if self.edge_top else 0
        hi_max = self.row_hi if self.edge_bot else self.rows_local
        k = self.halo if banded else n_sub
        j = 0
        while j < n_sub:
            cnt = min(k, n_sub - j)
            if banded:
                halo_exchange(self.state_buffer(j), cnt)
            if j + cnt < n_sub:
                self._run_block(j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max)
            else:
                native.check(native._lib.vk_diffuse_delta(
                    native.ptr(self.fields), native.ptr(self.work0), native.ptr(self.work1), native.ptr(delta),
                    len(self.molecules), self.field_stride, self.ny, self.row_lo, self.row_hi, lo_min, hi_max,
                    int(self.edge_top), int(self.edge_bot), j, cnt, n_sub, coeff_dt, native.ptr(mm),
                    native.stream_handle()), 'vk_diffuse_delta')
            j += cnt
        return delta

    def state_buffer(self, j: int):
        """Buffer holding the fields before substep j (vk_diffuse's rotation:
        field for j == 0, else work[(j-1) & 1])."""
        return self.fields if j == 0 else (self.work0 if ((j - 1) & 1) == 0 else self.work1)

    # passes of a band's first block whose interior runs while its halo exchange is in
    # flight (vk_diffuse_part); the edges of those passes follow the halo, then the
    # block's other passes whole.  Each interior-first pass costs a short, latency-bound
    # edge launch later, so only as many as the transfer needs to hide
    HALO_OVERLAP_PASSES = 3

    def _run_part(self, j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max, part, passes=None):
        """One part of a block (vk_diffuse_part); False if the block does not split."""
        rc = native._lib.vk_diffuse_part(
            native.ptr(self.fields), native.ptr(self.work0), native.ptr(self.work1),
            len(self.molecules), self.field_stride, self.ny, self.row_lo, self.row_hi, lo_min,
            hi_max, int(self.edge_top), int(self.edge_bot), j, cnt, n_sub, coeff_dt,
            native.ptr(mm), int(part), int(self.HALO_OVERLAP_PASSES if passes is None else passes),
            native.stream_handle())
        if rc == native.VK_ERR_LIMIT:
            return False
        native.check(rc, 'vk_diffuse_part')
        return True

    def _run_block_overlapped(self, j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max, halo_event):
        """A block whose halo exchange is still in flight (``halo_event``): its
        interior, then (after the event) its edges; the whole block after the
        event if it does not split."""
        main = torch.cuda.current_stream(self.device)
        if not self._run_part(j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max, native.VK_PART_INTERIOR):
            main.wait_event(halo_event)
            self._run_block(j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max)
            return
        main.wait_event(halo_event)
        self._run_part(j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max, native.VK_PART_EDGES)

    def _run_block(self, j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max):
        native.check(native._lib.vk_diffuse(
            native.ptr(self.fields), native.ptr(self.work0), native.ptr(self.work1),
            len(self.molecules), self.field_stride, self.ny, self.row_lo, self.row_hi, lo_min,
            hi_max, int(self.edge_top), int(self.edge_bot), j, cnt, n_sub, coeff_dt,
            native.ptr(mm), native.stream_handle()), 'vk_diffuse')

    # -- agent coupling ------------------------------------------------------
    def bin_sites(self, loc, n_agents, bin_lin=None, ix=None):
        """loc: [2, ld] float64 -> (bin_lin int32 [ld] local linear bin, ix int32 [ld])."""
        ld = loc.shape[1]
        bin_lin = torch.zeros(ld, dtype=torch.int32, device=self.device) if bin_lin is None else bin_lin
        ix = torch.zeros(ld, dtype=torch.int32, device=self.device) if ix is None else ix
        native.check(native._lib.vk_bin_sites(
            native.ptr(loc), n_agents, ld, self.n_bins[0], self.n_bins[1], self.bounds[0],
            self.bounds[1], self.row_lo_global - self.row_lo, native.ptr(bin_lin), native.ptr(ix),
            native.stream_handle()), 'vk_bin_sites')
        return bin_lin, ix

    def gather(self, bin_lin, n_agents, map_field, map_row, dst):
        """dst[map_row[i], a] = plane map_field[i] at bin_lin[a] (get_local_environments)."""
        native.check(native._lib.vk_gather(
            native.ptr(self.fields), self.field_stride, native.ptr(bin_lin), n_agents,
            native.ptr(map_field), native.ptr(map_row), int(map_field.numel()), native.ptr(dst),
            dst.shape[1], native.stream_handle()), 'vk_gather')

    def exchange_sorted(self, occ, counts, map_count, map_field):
        """Deterministic (agent-ordered) exchange; occ = (occ_bin, occ_ptr, occ_agent)."""
        occ_bin, occ_ptr, occ_agent = occ
        native.check(native._lib.vk_exchange_sorted(
            native.ptr(self.fields), self.field_stride, native.ptr(occ_bin), native.ptr(occ_ptr),
            native.ptr(occ_agent), int(occ_bin.numel()), native.ptr(counts), counts.shape[1],
            native.ptr(map_count), native.ptr(map_field), int(map_count.numel()),
            self.binvol_avogadro, native.stream_handle()), 'vk_exchange_sorted')

    def exchange_atomic(self, bin_lin, n_agents, counts, map_count, map_field):
        native.check(native._lib.vk_exchange_atomic(
            native.ptr(self.fields), self.field_stride, native.ptr(bin_lin), n_agents,
            native.ptr(counts), counts.shape[1], native.ptr(map_count), native.ptr(map_field),
            int(map_count.numel()), self.binvol_avogadro, native.stream_handle()),
            'vk_exchange_atomic')


def segment_index(bin_lin: torch.Tensor, n_agents: int, rows: int, ny: int) -> torch.Tensor:
    """For agents stored in bin order: seg[r * nseg + s] = the first agent whose
    bin is >= r * ny + 16 s (nseg = ceil(ny / 16)), the index the coupled
    passes find a row segment's agents with (vk_diffuse_coupled)."""
    nseg = (ny + 15) // 16
    dev = bin_lin.device
    targets = (torch.arange(rows, dtype=torch.int64, device=dev)[:, None] * ny +
               16 * torch.arange(nseg, dtype=torch.int64, device=dev)[None, :]).reshape(-1)
    return torch.searchsorted(bin_lin[:n_agents].to(torch.int64), targets).to(torch.int32)


def occupancy(bin_lin: torch.Tensor, n_agents: int, order_key: Optional[torch.Tensor] = None):
    """Bin -> agents CSR for :meth:`Lattice.exchange_sorted`: each bin's agents in
    agent order -- their column order, or ascending ``order_key`` (the agents'
    reference order when the columns were permuted, Colony.sort_by_bin)."""
    b = bin_lin[:n_agents].to(torch.int64)
    if order_key is None:
        order = torch.sort(b, stable=True).indices
    else:
        by_key = torch.sort(order_key[:n_agents].to(torch.int64), stable=True).indices
        order = by_key[torch.sort(b[by_key], stable=True).indices]
    sb = b[order]
    if n_agents == 0:
        z = torch.zeros(0, dtype=torch.int32, device=bin_lin.device)
        return z, torch.zeros(1, dtype=torch.int32, device=bin_lin.device), z
    uniq, cnt = torch.unique_consecutive(sb, return_counts=True)
    ptr = torch.zeros(uniq.numel() + 1, dtype=torch.int64, device=bin_lin.device)
    ptr[1:] = torch.cumsum(cnt, 0)
    return uniq.to(torch.int32), ptr.to(torch.int32), order.to(torch.int32)

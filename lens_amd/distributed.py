"""Multi-GPU row-band decomposition of the lattice (one process per GPU).

SURVEY.md §8e: the field is split into contiguous row bands (axis 0 = x),
agents live on the rank that owns their bin row, so gather and exchange stay
rank-local.  The only data-path communication is the stencil halo: every
``halo`` substeps each rank swaps ``halo`` boundary rows with its two
neighbours (point-to-point send/recv -- RCCL over xGMI with the ``nccl``
backend, or gloo on CPU), then computes ``halo`` substeps with a shrinking
region, recomputing the overlap instead of talking 100 times per step.  The
uniform-field test is the one scalar all-reduce per step.
"""

from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist


def row_bands(nx: int, world: int) -> List[Tuple[int, int]]:
    """Near-equal contiguous row bands [lo, hi) for each rank."""
    base, extra = divmod(nx, world)
    out, lo = [], 0
    for r in range(world):
        hi = lo + base + (1 if r < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


def _host_staged(dev, group) -> bool:
    """gloo moves host tensors: device buffers are staged through host memory
    (rehearsal runs of the multi-rank path on one GPU; RCCL needs no staging)."""
    return dev.type != 'cpu' and dist.get_backend(group) == 'gloo'


def make_halo_exchange(lat, rank: int, world: int, group=None):
    """Callback for :meth:`Lattice.diffuse`: fill ``lat.halo`` rows above/below
    the owned band of ``src`` (a [n_fields, rows_local, ny] tensor) from the
    neighbouring ranks' owned rows."""
    h = lat.halo
    owned = lat.row_hi - lat.row_lo
    if h < 1 and not (lat.edge_top and lat.edge_bot):
        raise ValueError('a multi-rank row band needs halo >= 1 (got %d)' % h)
    if h > owned:
        raise ValueError('halo (%d) deeper than the band (%d rows)' % (h, owned))
    nf, ny = len(lat.molecules), lat.ny
    dev = lat.fields.device
    if not _host_staged(dev, group):
        # RCCL (or gloo on host planes): each plane's boundary rows are one contiguous
        # block of the [n_fields, rows_local, ny] buffer, so they are sent from and
        # received into the buffer itself -- no staging copies around the transfer
        # (six copy launches per exchange).  Per neighbour the planes go in plane order
        # on both sides, which is how the point-to-point pairs match.
        def exchange_direct(src, cnt):
            ops = []
            for f in range(nf):
                if not lat.edge_top:      # neighbour rank-1 owns the rows above
                    ops.append(dist.P2POp(dist.isend, src[f, lat.row_lo:lat.row_lo + h], rank - 1, group))
                    ops.append(dist.P2POp(dist.irecv, src[f, lat.row_lo - h:lat.row_lo], rank - 1, group))
                if not lat.edge_bot:
                    ops.append(dist.P2POp(dist.isend, src[f, lat.row_hi - h:lat.row_hi], rank + 1, group))
                    ops.append(dist.P2POp(dist.irecv, src[f, lat.row_hi:lat.row_hi + h], rank + 1, group))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()

        return exchange_direct
    bufs = {k: torch.empty((nf, h, ny), dtype=torch.float64, device=torch.device('cpu'))
            for k in ('send_up', 'send_dn', 'recv_up', 'recv_dn')}

    def exchange(src, cnt):
        ops = []
        if not lat.edge_top:          # neighbour rank-1 owns the rows above
            bufs['send_up'].copy_(src[:, lat.row_lo:lat.row_lo + h])
            ops.append(dist.P2POp(dist.isend, bufs['send_up'], rank - 1, group))
            ops.append(dist.P2POp(dist.irecv, bufs['recv_up'], rank - 1, group))
        if not lat.edge_bot:
            bufs['send_dn'].copy_(src[:, lat.row_hi - h:lat.row_hi])
            ops.append(dist.P2POp(dist.isend, bufs['send_dn'], rank + 1, group))
            ops.append(dist.P2POp(dist.irecv, bufs['recv_dn'], rank + 1, group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if not lat.edge_top:
            src[:, lat.row_lo - h:lat.row_lo].copy_(bufs['recv_up'])
        if not lat.edge_bot:
            src[:, lat.row_hi:lat.row_hi + h].copy_(bufs['recv_dn'])

    return exchange


def make_uniform_allreduce(group=None):
    """Uniformity summary [lo0, hi0, lo1, hi1, ...] (vk_field_uniform) -> element-wise
    min of the lo entries and max of the hi entries over ranks (one all-reduce):
    lo == hi afterwards iff every rank's band holds the same single value.
    ``group``: give it its own (``dist.new_group``) when the halo exchange runs
    on another stream, so the two do not queue behind each other."""

    def allreduce(mm):
        t = mm.cpu() if _host_staged(mm.device, group) else mm
        t[0::2].neg_()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        t[0::2].neg_()
        if t is not mm:
            mm.copy_(t)

    return allreduce


# ---------------------------------------------------------------------------
# agent routing between row bands (division moves daughters across band edges)
# ---------------------------------------------------------------------------

class GlobalRoots:
    """Root agent names for a multi-rank colony: ``str(global index)``, the
    single-rank colony's default ids (Colony(agent_ids=None))."""

    def __getitem__(self, i):
        return str(int(i))

    def __len__(self):          # pragma: no cover - informational
        return 0


class AgentRouter:
    """Keeps every agent of a row-banded lattice colony on the rank that owns
    its bin row, moving daughters that division placed past a
    band edge (``daughter_locations``, vivarium/processes/multibody_physics.py:
    77-87) with one ``all_to_all`` of packed agent rows.

    Each agent also carries ``ordinal``: its position in the order a
    single-rank colony would hold it in.  The reference's order -- survivors
    in their order, then daughters in mother order, each mother's two
    daughters in id order (vivarium/core/experiment.py:664-697) -- is
    rank-count independent only through this global key: after a division
    step a survivor's new ordinal is its old one minus the number of dividing
    mothers (on ANY rank) before it, and daughter k of a mother with ordinal g
    gets (survivors everywhere) + 2 * (dividing mothers before g) + k.  One
    all-gather of the dividing mothers' ordinals per step provides that.  Each
    rank keeps its agents sorted by ordinal, so the agent-ordered exchange
    scatter adds a bin's agents in the single-rank order: a banded colony with
    division equals the single-rank colony bit for bit.

    ``agent_offset``: global index of this rank's first agent (the initial
    colony is split by band in index order); root ids become global."""

    def __init__(self, col, rank: int, world: int, group=None, agent_offset: int = None):
        self.col, self.rank, self.world, self.group = col, rank, world, group
        lat = col.lattice
        bands = row_bands(lat.n_bins[0], world)
        if (lat.row_lo_global, lat.row_hi_global) != bands[rank]:
            raise ValueError('the lattice band %r is not rank %d of row_bands' % (
                (lat.row_lo_global, lat.row_hi_global), rank))
        dev = col.device
        self.band_hi = torch.tensor([hi for _, hi in bands], dtype=torch.int64, device=dev)
        self.staged = _host_staged(dev, group)
        n = col.n
        if agent_offset is None:
            counts = self._all_gather_sizes(n)
            agent_offset = int(sum(counts[:rank]))
        col.ordinal = torch.zeros(col.ld, dtype=torch.int64, device=dev)
        col.ordinal[:n] = torch.arange(agent_offset, agent_offset + n, device=dev)
        if col.cells is not None:
            col.lin_root[:n] = col.ordinal[:n].to(torch.int32)
            col.roots = GlobalRoots()
        col.router = self

    # -- collectives (gloo stages device tensors through host memory) --------
    def _dev(self, t):
        return t.cpu() if self.staged else t

    def _all_gather_sizes(self, k: int):
        t = self._dev(torch.tensor([k], dtype=torch.int64, device=self.col.device))
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [int(x.item()) for x in out]

    def _all_gather_var(self, t):
        """Concatenation over ranks of a 1-D int64 tensor of any length."""
        sizes = self._all_gather_sizes(t.numel())
        m = max(sizes) if sizes else 0
        if m == 0:
            return torch.zeros(0, dtype=torch.int64, device=self.col.device)
        pad = torch.zeros(m, dtype=torch.int64, device=self.col.device)
        pad[:t.numel()] = t
        pad = self._dev(pad)
        out = [torch.zeros_like(pad) for _ in range(self.world)]
        dist.all_gather(out, pad, group=self.group)
        return torch.cat([o[:s] for o, s in zip(out, sizes)]).to(self.col.device)

    # -- division ------------------------------------------------------------
    def division_ordinals(self, old_ord, dividing, src, kind, n_out):
        """(new ordinals of the n_out agents of this rank's division plan, the
        number of mothers that divided on all ranks); src / kind from
        vk_divide_plan.  A collective: every rank calls it every step."""
        mothers = old_ord[dividing]
        d_all = torch.sort(self._all_gather_var(mothers)).values
        n_surv = sum(self._all_gather_sizes(int(old_ord.numel() - mothers.numel())))
        a = src[:n_out].to(torch.int64)
        kd = kind[:n_out].to(torch.int64)
        g = old_ord[a]
        before = torch.searchsorted(d_all, g)              # dividing mothers strictly before g
        return torch.where(kd < 0, g - before, n_surv + 2 * before + kd), int(d_all.numel())

    # -- migration -------------------------------------------------------------
    def route(self):
        """Send every agent whose bin row lies in another rank's band to that
        rank; keep this rank's agents sorted by ordinal.  Collective."""
        col, lat = self.col, self.col.lattice
        n = col.n
        lat.bin_sites(col.location, n, col.bin_lin, col.bin_ix)
        dest = torch.bucketize(col.bin_ix[:n].to(torch.int64), self.band_hi, right=True)
        leave = dest != self.rank
        send_counts = torch.bincount(dest[leave], minlength=self.world)
        order = torch.sort(dest[leave], stable=True).indices
        idx_leave = torch.nonzero(leave).flatten()[order]
        idx_stay = torch.nonzero(~leave).flatten()
        names = col.agent_array_names()
        send = pack_agents(col, names, idx_leave)
        send_counts_l = [int(x) for x in send_counts.tolist()]
        sc = self._dev(send_counts.to(torch.int64))
        rc = torch.zeros_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        recv_counts_l = [int(x) for x in rc.tolist()]
        # every rank joins the payload exchange, even with nothing to move
        # (skipping it locally would strand the ranks that do exchange)
        width = send.shape[1]
        recv = torch.zeros((sum(recv_counts_l), width), dtype=torch.float64,
                           device='cpu' if self.staged else col.device)
        dist.all_to_all_single(recv, self._dev(send), recv_counts_l, send_counts_l, group=self.group)
        recv = recv.to(col.device)
        if sum(send_counts_l) or sum(recv_counts_l):
            stay = {name: take_agents(col, name, idx_stay) for name in names}
            both = {name: torch.cat([stay[name], piece], dim=1)
                    for name, piece in unpack_agents(col, names, recv).items()}
            # immigrants merge with the stayers by ordinal
            perm = torch.sort(both['ordinal'].reshape(-1), stable=True).indices
            install_agents(col, names, {name: v.index_select(1, perm) for name, v in both.items()})
            col.bin_lin = torch.zeros(col.ld, dtype=torch.int32, device=col.device)
            col.bin_ix = torch.zeros(col.ld, dtype=torch.int32, device=col.device)
        return sum(recv_counts_l)


# ---------------------------------------------------------------------------
# packing per-agent SoA columns into rows of float64 (one all_to_all payload)
# ---------------------------------------------------------------------------

def take_agents(col, name, idx):
    """Columns ``idx`` of the per-agent array ``name`` as a [rows, k] tensor."""
    t = getattr(col, name)
    x = t.index_select(t.dim() - 1, idx)
    return x.reshape(1, -1) if t.dim() == 1 else x


def pack_agents(col, names, idx):
    """[k, width] float64: one row per agent; int64 columns travel as raw bits,
    int32 columns as exact float64 values."""
    cols = []
    for name in names:
        x = take_agents(col, name, idx)
        if x.dtype == torch.int64:
            x = x.contiguous().view(torch.float64)
        elif x.dtype != torch.float64:
            x = x.to(torch.float64)
        cols.append(x.t())
    return torch.cat(cols, dim=1).contiguous()


def unpack_agents(col, names, recv):
    """Inverse of :func:`pack_agents`: {name: [rows, k] tensor of the array's dtype}."""
    out, off = {}, 0
    for name in names:
        t = getattr(col, name)
        rows = 1 if t.dim() == 1 else t.shape[0]
        r = recv[:, off:off + rows].t().contiguous()
        off += rows
        if t.dtype == torch.int64:
            r = r.view(torch.int64)
        elif t.dtype != torch.float64:
            r = r.to(t.dtype)
        out[name] = r
    return out


def install_agents(col, names, pieces):
    """Replace every per-agent array by ``pieces[name]`` ([rows, n_new]),
    growing the capacity when needed."""
    n_new = pieces[names[0]].shape[1]
    ld = col.ld if n_new <= col.ld else max(n_new, int(col.ld * 1.25) + 64)
    for name in names:
        t = getattr(col, name)
        out = torch.zeros((ld,) if t.dim() == 1 else (t.shape[0], ld), dtype=t.dtype, device=col.device)
        if t.dim() == 1:
            out[:n_new] = pieces[name].reshape(-1)
        else:
            out[:, :n_new] = pieces[name]
        setattr(col, name, out)
    col.n, col.ld = n_new, ld
    if getattr(col, 'env_fields', None) is not None:
        # NonSpatialEnvironment: agent a's field is env_fields[:, a] (stride ld)
        col.env_bins = torch.arange(ld, dtype=torch.int32, device=col.device)


class AgentBalancer:
    """Agent-sharded colonies without a lattice (BASELINE configs 2 and 5):
    division is rank-local, so ranks drift apart in agent count; when the
    largest rank holds more than (1 + tolerance) x the mean, agents move
    between neighbouring ranks so that every rank holds a near-equal
    contiguous slice of the concatenated (rank-major) order -- one all_to_all
    of packed agent rows, order preserved (alltoallv after
    division imbalance).  Agents without a lattice are independent, so
    placement changes no result; ``agent_ids`` stay global (GlobalRoots)."""

    def __init__(self, col, rank: int, world: int, group=None, tolerance: float = 0.05,
                 agent_offset: int = None):
        if col.lattice is not None:
            raise ValueError('lattice colonies are placed by band: use AgentRouter')
        self.col, self.rank, self.world, self.group, self.tolerance = col, rank, world, group, tolerance
        self.staged = _host_staged(col.device, group)
        if col.cells is not None:
            if agent_offset is None:
                agent_offset = int(sum(self._sizes(col.n)[:rank]))
            col.lin_root[:col.n] = torch.arange(agent_offset, agent_offset + col.n, device=col.device,
                                                dtype=torch.int32)
            col.roots = GlobalRoots()
        self.moves = 0

    def _sizes(self, k):
        t = torch.tensor([k], dtype=torch.int64)
        t = t if self.staged or self.col.device.type == 'cpu' else t.to(self.col.device)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [int(x.item()) for x in out]

    def balance(self, force: bool = False) -> int:
        """Collective.  Returns the number of agents this rank received."""
        col = self.col
        sizes = self._sizes(col.n)
        total = sum(sizes)
        if total == 0 or (not force and max(sizes) <= (1 + self.tolerance) * total / self.world):
            return 0
        start = sum(sizes[:self.rank])
        bounds = [total * r // self.world for r in range(self.world + 1)]    # target slices
        g = torch.arange(start, start + col.n, device=col.device)
        dest = torch.bucketize(g, torch.tensor(bounds[1:], device=col.device), right=True)
        send_counts = torch.bincount(dest, minlength=self.world)
        names = col.agent_array_names()
        send = pack_agents(col, names, torch.arange(col.n, device=col.device))   # dest is monotone
        send_l = [int(x) for x in send_counts.tolist()]
        recv_l = [max(0, min(sizes_hi, bounds[self.rank + 1]) - max(sizes_lo, bounds[self.rank]))
                  for sizes_lo, sizes_hi in [(sum(sizes[:r]), sum(sizes[:r + 1])) for r in range(self.world)]]
        recv = torch.zeros((sum(recv_l), send.shape[1]), dtype=torch.float64,
                           device='cpu' if self.staged else col.device)
        dist.all_to_all_single(recv, send.cpu() if self.staged else send, recv_l, send_l, group=self.group)
        install_agents(col, names, unpack_agents(col, names, recv.to(col.device)))
        got = sum(recv_l) - send_l[self.rank]
        self.moves += got
        return got


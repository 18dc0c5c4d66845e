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
    buf_dev = torch.device('cpu') if _host_staged(dev, group) else dev
    bufs = {k: torch.empty((nf, h, ny), dtype=torch.float64, device=buf_dev)
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
    lo == hi afterwards iff every rank's band holds the same single value."""

    def allreduce(mm):
        t = mm.cpu() if _host_staged(mm.device, group) else mm
        t[0::2].neg_()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        t[0::2].neg_()
        if t is not mm:
            mm.copy_(t)

    return allreduce

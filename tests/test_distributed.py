"""Multi-rank row-band decomposition on CPU (gloo, world sizes 2 and 3).

The halo-exchange protocol, band geometry, buffer rotation and the uniform-
field all-reduce of lens_amd.distributed / Lattice.diffuse run for real over
torch.distributed; only the per-block stencil launch is replaced by a CPU
restatement of vk_diffuse's documented semantics (the kernel itself is
covered bit-for-bit by tests/test_gpu_parity.py).  The assembled bands must
equal the single-domain oracle bit for bit.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lens_amd.distributed import row_bands, make_halo_exchange, make_uniform_allreduce
from lens_amd.lattice import Lattice
from oracle import lattice as olat


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cpu_run_block(lat, j, cnt, n_sub, coeff_dt, mm, lo_min, hi_max):
    """vk_diffuse semantics (include/vk_kinetics.h) restated with torch on CPU."""
    top = lo_min if lat.edge_top else -1
    bot = hi_max - 1 if lat.edge_bot else 1 << 30
    last = j + cnt - 1
    nf, ny = len(lat.molecules), lat.ny
    for jsub in range(j, j + cnt):
        grow = last - jsub
        lo = max(lo_min, lat.row_lo - grow)
        hi = min(hi_max, lat.row_hi + grow)
        src = lat.state_buffer(jsub)
        final = jsub == n_sub - 1
        dst = lat.fields if final else (lat.work0 if (jsub & 1) == 0 else lat.work1)
        for f in range(nf):
            if mm is not None and mm[2 * f] == mm[2 * f + 1]:
                continue                      # uniform plane: the kernel writes nothing
            rows = np.arange(lo, hi)
            up = np.where(rows == top, rows, rows - 1)
            dn = np.where(rows == bot, rows, rows + 1)
            s = src[f].numpy()
            c = s[lo:hi]
            left = np.concatenate([c[:, :1], c[:, :-1]], axis=1)
            right = np.concatenate([c[:, 1:], c[:, -1:]], axis=1)
            lap = (((s[up] + left) + (-4.0 * c)) + right) + s[dn]
            v = c + coeff_dt * lap
            if final:
                base = lat.fields[f, lo:hi].numpy()
                v = base + (v - base)
            dst[f, lo:hi] = torch.from_numpy(v)


def _worker(rank, world, port, halo, f0, result_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        nx, ny = f0.shape
        band = row_bands(nx, world)[rank]
        lat = Lattice(['a', 'u'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device='cpu',
                      row_band=band, halo=halo, initial={'a': f0, 'u': np.full((nx, ny), 4.0)})
        lat._run_block = lambda *a: cpu_run_block(lat, *a)

        def uniform(allreduce=None):
            # CPU stand-in for vk_field_uniform's summary: (v, v) or (-inf, +inf)
            own = lat.fields[:, lat.row_lo:lat.row_hi]
            rows = []
            for f in range(own.shape[0]):
                v0 = own[f].flatten()[0]
                uni = bool((own[f] == v0).all())
                rows.append([v0, v0] if uni else [-float('inf'), float('inf')])
            mm = torch.tensor(rows, dtype=torch.float64).flatten().contiguous()
            if allreduce is not None:
                allreduce(mm)
            lat.uniform = mm
            return mm
        lat.uniform_summary = uniform
        lat.diffuse(1.0, halo_exchange=make_halo_exchange(lat, rank, world),
                    allreduce=make_uniform_allreduce())
        result_q.put((rank, band, lat.owned().numpy().copy()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize('world,halo', [(2, 10), (3, 7), (2, 1)])
def test_banded_diffusion_gloo_matches_oracle(world, halo):
    rng = np.random.default_rng(world * 10 + halo)
    nx, ny = 41, 23
    f0 = rng.random((nx, ny)) * 3.0
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, halo, f0, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts.sort(key=lambda t: t[0])
    got_a = np.concatenate([p[2][0] for p in parts], axis=0)
    got_u = np.concatenate([p[2][1] for p in parts], axis=0)
    ref = olat.diffuse(f0, 1.0, 5.0, (nx, ny), (float(nx), float(ny)))
    assert np.array_equal(got_a, ref)
    assert np.array_equal(got_u, np.full((nx, ny), 4.0))   # uniform plane skipped on every rank


def test_row_bands_cover_exactly():
    for nx in (7, 4096, 4097):
        for world in (1, 2, 3, 8):
            b = row_bands(nx, world)
            assert b[0][0] == 0 and b[-1][1] == nx
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


def test_interior_band_without_halo_is_rejected():
    """an interior band edge with halo 0 would act as a reflecting
    wall and silently decouple the ranks' fields."""
    with pytest.raises(ValueError):
        Lattice(['a'], (41, 23), (41.0, 23.0), 10.0, 5.0, device='cpu', row_band=(0, 20), halo=0)
    with pytest.raises(ValueError):
        Lattice(['a'], (41, 23), (41.0, 23.0), 10.0, 5.0, device='cpu', row_band=(20, 41), halo=0)
    with pytest.raises(ValueError):   # halo deeper than the band
        Lattice(['a'], (41, 23), (41.0, 23.0), 10.0, 5.0, device='cpu', row_band=(20, 25), halo=8)
    # the whole domain as one band needs no halo
    Lattice(['a'], (41, 23), (41.0, 23.0), 10.0, 5.0, device='cpu', row_band=(0, 41), halo=0)

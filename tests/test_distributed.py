"""Multi-rank row-band decomposition on CPU (gloo, world sizes 2, 3 and 8).

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


@pytest.mark.parametrize('world,halo', [(2, 10), (3, 7), (2, 1), (8, 5)])
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


# ---------------------------------------------------------------------------
# AgentRouter host logic (gloo, CPU tensors; the GPU colony version is in
# tests/test_distributed_gpu.py)
# ---------------------------------------------------------------------------

class _FakeLattice:
    def __init__(self, nx, band):
        self.n_bins = [nx, 4]
        self.row_lo_global, self.row_hi_global = band

    def bin_sites(self, loc, n, bin_lin, ix):
        ix[:n] = torch.floor(loc[0, :n]).to(torch.int32)
        bin_lin[:n] = 0


class _FakeColony:
    """The per-agent arrays AgentRouter moves, in the Colony layout."""

    def __init__(self, nx, band, xs, vals, ords, ld):
        n = len(xs)
        self.device = torch.device('cpu')
        self.lattice = _FakeLattice(nx, band)
        self.cells = None
        self.n, self.ld = n, ld
        self.location = torch.zeros((2, ld), dtype=torch.float64)
        self.location[0, :n] = torch.tensor(xs, dtype=torch.float64)
        self.params = torch.zeros((2, ld), dtype=torch.float64)
        self.params[0, :n] = torch.tensor(vals, dtype=torch.float64)
        self.params[1, :n] = -torch.tensor(vals, dtype=torch.float64)
        self.counts = torch.zeros((1, ld), dtype=torch.int64)
        self.counts[0, :n] = torch.tensor([int(v * 1e6) - (1 << 40) for v in vals], dtype=torch.int64)
        self.status = torch.zeros(ld, dtype=torch.int32)
        self.status[:n] = torch.tensor([int(v * 1000) for v in vals], dtype=torch.int32)
        self.ordinal = torch.zeros(ld, dtype=torch.int64)
        self.ordinal[:n] = torch.tensor(ords, dtype=torch.int64)
        self.bin_lin = torch.zeros(ld, dtype=torch.int32)
        self.bin_ix = torch.zeros(ld, dtype=torch.int32)

    def agent_array_names(self):
        return ['params', 'counts', 'status', 'location', 'ordinal']


def _router_worker(rank, world, port, seed, q):
    from lens_amd.distributed import AgentRouter
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        nx = 30
        bands = row_bands(nx, world)
        rng = np.random.default_rng(seed)
        n_glob = 200
        xs_all = rng.uniform(0, nx, n_glob)
        owner = rng.integers(0, world, n_glob)          # agents start on arbitrary ranks
        mine = np.flatnonzero(owner == rank)             # ordinal order = global index order
        col = _FakeColony(nx, bands[rank], xs_all[mine].tolist(), (mine / 7.0 + 0.5).tolist(), mine.tolist(),
                          ld=len(mine) + 3)
        r = AgentRouter.__new__(AgentRouter)
        r.col, r.rank, r.world, r.group, r.staged = col, rank, world, None, False
        r.band_hi = torch.tensor([hi for _, hi in bands], dtype=torch.int64)
        r.route()
        n = col.n
        got = {'ord': col.ordinal[:n].tolist(), 'x': col.location[0, :n].tolist(),
               'p0': col.params[0, :n].tolist(), 'p1': col.params[1, :n].tolist(),
               'counts': col.counts[0, :n].tolist(), 'status': col.status[:n].tolist()}
        # division ordinals: a random dividing subset of the (now routed) agents
        div = torch.tensor(rng.random(n_glob) < 0.3)[col.ordinal[:n]]
        keep = torch.nonzero(~div).flatten()
        moth = torch.nonzero(div).flatten()
        src = torch.cat([keep, moth.repeat_interleave(2)]).to(torch.int32)
        kind = torch.cat([torch.full((keep.numel(),), -1), torch.tensor([0, 1] * moth.numel())]).to(torch.int32)
        new, n_div = r.division_ordinals(col.ordinal[:n], div, src, kind, src.numel())
        got['new'] = new.tolist()
        got['src_ord'] = col.ordinal[:n][src.to(torch.int64)].tolist()
        got['kind'] = kind.tolist()
        got['n_div'] = n_div
        q.put((rank, bands[rank], got, xs_all.tolist(), (rng.random(0)).tolist()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize('world,seed', [(2, 1), (3, 2), (8, 3)])
def test_agent_router_routes_and_orders(world, seed):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_router_worker, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    xs_all = parts[0][3]
    seen = []
    for rank, band, got, _, _ in parts:
        # every agent now lives in its band, sorted by ordinal, payload intact
        assert all(band[0] <= int(np.floor(x)) < band[1] for x in got['x'])
        assert got['ord'] == sorted(got['ord'])
        for o, x, p0, p1, c, s in zip(got['ord'], got['x'], got['p0'], got['p1'], got['counts'], got['status']):
            assert x == xs_all[o] and p0 == o / 7.0 + 0.5 and p1 == -p0
            assert c == int(p0 * 1e6) - (1 << 40) and s == int(p0 * 1000)
        seen += got['ord']
    assert sorted(seen) == list(range(200))
    # division ordinals == positions in the single-rank order (survivors, then daughters in mother order)
    divided = sorted(o for _, _, got, _, _ in parts for o, k in zip(got['src_ord'], got['kind']) if k == 0)
    survivors = sorted(set(range(200)) - set(divided))
    want = {('s', o): i for i, o in enumerate(survivors)}
    for i, o in enumerate(divided):
        want[('d', o, 0)] = len(survivors) + 2 * i
        want[('d', o, 1)] = len(survivors) + 2 * i + 1
    allnew = []
    for _, _, got, _, _ in parts:
        assert got['n_div'] == len(divided)
        for o, k, g in zip(got['src_ord'], got['kind'], got['new']):
            assert g == want[('s', o) if k < 0 else ('d', o, k)]
            allnew.append(g)
    assert sorted(allnew) == list(range(len(survivors) + 2 * len(divided)))


def _balance_worker(rank, world, port, sizes, q):
    from lens_amd.distributed import AgentBalancer
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        start = sum(sizes[:rank])
        g = list(range(start, start + sizes[rank]))
        col = _FakeColony(30, (0, 30), [0.5] * len(g), [x / 3.0 for x in g], g, ld=len(g) + 1)
        col.lattice = None
        b = AgentBalancer(col, rank, world, tolerance=0.05)
        got = b.balance()
        n = col.n
        q.put((rank, col.ordinal[:n].tolist(), col.params[0, :n].tolist(), col.counts[0, :n].tolist(), got))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize('sizes', [(10, 50), (40, 3, 17), (0, 12, 30, 1)])
def test_agent_balancer_evens_out_in_order(sizes):
    world = len(sizes)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balance_worker, args=(r, world, port, list(sizes), q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = sum(sizes)
    glob = [o for _, ords, _, _, _ in parts for o in ords]
    assert glob == list(range(total))                     # rank-major order preserved
    for r, ords, p0, counts, _ in parts:
        assert len(ords) == (r + 1) * total // world - r * total // world
        assert p0 == [o / 3.0 for o in ords]
        assert counts == [int(o / 3.0 * 1e6) - (1 << 40) for o in ords]


class _FakeNonspatialColony(_FakeColony):
    """A NonSpatialEnvironment colony's per-agent arrays: each agent owns a
    column of ``env_fields`` (its 1x1 field per molecule) addressed through
    ``env_bins`` (the balancer must move both)."""

    def __init__(self, g, ld):
        super().__init__(30, (0, 30), [0.5] * len(g), [x / 3.0 for x in g], g, ld=ld)
        self.lattice = None
        self.location = None
        self.env_fields = torch.zeros((2, ld), dtype=torch.float64)
        self.env_fields[0, :len(g)] = torch.tensor([1000.0 + x for x in g], dtype=torch.float64)
        self.env_fields[1, :len(g)] = torch.tensor([-0.5 * x for x in g], dtype=torch.float64)
        self.env_bins = torch.arange(ld, dtype=torch.int32)

    def agent_array_names(self):
        from lens_amd.colony import Colony
        names = Colony.agent_array_names(self)     # the real list, env_fields included
        return [n for n in names if hasattr(self, n)]

    # attributes Colony.agent_array_names reads
    cells = None
    ordinal = None


def _balance_nonspatial_worker(rank, world, port, sizes, q):
    from lens_amd.distributed import AgentBalancer
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        start = sum(sizes[:rank])
        g = list(range(start, start + sizes[rank]))
        col = _FakeNonspatialColony(g, ld=len(g) + 1)
        assert 'env_fields' in col.agent_array_names()
        AgentBalancer(col, rank, world, tolerance=0.05).balance()
        n = col.n
        q.put((rank, col.ordinal[:n].tolist(), col.env_fields[:, :n].tolist(), col.env_bins.tolist(), col.ld))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_agent_balancer_moves_nonspatial_fields():
    sizes = (5, 40, 2)
    world = len(sizes)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balance_nonspatial_worker, args=(r, world, port, list(sizes), q))
             for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    glob = [o for _, ords, _, _, _ in parts for o in ords]
    assert glob == list(range(sum(sizes)))
    for _, ords, env, bins, ld in parts:
        assert env[0] == [1000.0 + o for o in ords]         # each agent keeps its own environment
        assert env[1] == [-0.5 * o for o in ords]
        assert bins == list(range(ld))                       # env_bins follows the new stride

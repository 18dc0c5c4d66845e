"""The real multi-rank lattice colony on one MI355X (needs a GPU).

2 and 3 ranks (gloo; device buffers staged through host memory, as the
driver's RCCL run does over xGMI) each own a row band of the lattice and the
agents in it, and run the full ``Colony.step`` on cuda:0 through the HIP
kernels: kinetics, one-step-lag gather, banded diffusion with k-deep halo
exchange, agent-ordered exchange scatter, growth, derivers and division, and
``AgentRouter`` migration of daughters placed past a band edge
(``daughter_locations``, vivarium/processes/multibody_physics.py:77-87).
After every step the assembled colony must equal the single-rank colony bit
for bit: the same agents (phylogeny ids), in the same global order, with the
same state, and the same fields.
"""

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

NX, NY, N, STEPS = 40, 32, 300, 30


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _colony_inputs():
    """Global colony, in band-major order (the initial split keeps index order)."""
    from lens_amd import configs
    from lens_amd.rate_law_compiler import compile_rate_laws
    cfg = configs.glc_ac_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    rng = np.random.default_rng(77)
    x = rng.uniform(0.0, NX, N)
    x[:60] = rng.uniform(NX / 2 - 1.0, NX / 2 + 1.0, 60)          # crowd the band edges
    x[60:100] = rng.uniform(NX / 3 - 1.0, NX / 3 + 1.0, 40)
    x[100:140] = rng.uniform(2 * NX / 3 - 1.0, 2 * NX / 3 + 1.0, 40)
    loc = np.stack([x, rng.uniform(0.0, NY, N)])
    order = np.argsort(np.floor(loc[0]), kind='stable')           # by bin row
    loc = np.ascontiguousarray(loc[:, order])
    params, conc = configs.heterogeneous_colony(t, cfg, N, seed=5)
    mass = rng.uniform(1339.0, 2.4 * 1100.0, N)
    angle = rng.uniform(0, 2 * np.pi, N)
    return cfg, t, params, conc, loc, mass, angle


def _make(dev, cfg, t, band, halo, params, conc, loc, mass, angle):
    from lens_amd import configs, native
    from lens_amd.cells import CellModel
    from lens_amd.colony import Colony
    from lens_amd.lattice import Lattice
    lat = Lattice(['glc__D_e', 'ac_e'], (NX, NY), (float(NX), float(NY)), 10.0, 5.0, device=dev,
                  row_band=band, halo=halo,
                  initial={'glc__D_e': configs.gaussian_bump_field((NX, NY)), 'ac_e': np.zeros((NX, NY))})
    cm = CellModel(model='growth', growth_rate=0.003, division_volume=2.4)
    n = conc.shape[1]
    col = Colony(cfg, n, device=dev, integrator='euler', environment=lat, table=t, cells=cm)
    col.set_agents(params=params, conc=conc, location=loc)
    col.set_cell_mass(mass)
    rows = col.cell.cpu().numpy()
    rows[native.VK_CELL_ANGLE, :n] = angle
    col.cell.copy_(torch.from_numpy(rows))
    col.gather_external()
    return col, lat


def _state(col, lat):
    """{(root, depth, path): bytes of every per-agent array}, [(ordinal, key)],
    the owned fields.  Root indices are global in both runs (the single-rank
    colony's agents are the global colony in index order)."""
    n = col.n
    names = [a for a in col.agent_array_names() if a != 'ordinal']
    arrays = {a: getattr(col, a)[..., :n].cpu().numpy() for a in names}
    keys = list(zip(arrays['lin_root'].tolist(), arrays['lin_depth'].tolist(), arrays['lin_path'].tolist()))
    per = {}
    for j, key in enumerate(keys):
        per[key] = {a: np.ascontiguousarray(v[..., j]).tobytes() for a, v in arrays.items()}
    ords = col.ordinal[:n].cpu().numpy().tolist() if col.ordinal is not None else list(range(n))
    return per, list(zip(ords, keys)), lat.owned().cpu().numpy().copy()


def _worker(rank, world, port, halo, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from lens_amd.distributed import row_bands, make_halo_exchange, make_uniform_allreduce, AgentRouter
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        cfg, t, params, conc, loc, mass, angle = _colony_inputs()
        band = row_bands(NX, world)[rank]
        rows = np.floor(loc[0]).astype(int)
        mine = np.flatnonzero((rows >= band[0]) & (rows < band[1]))
        offset = int(mine[0]) if len(mine) else int(np.sum(rows < band[0]))
        col, lat = _make(dev, cfg, t, band, halo, params[:, mine], conc[:, mine], loc[:, mine], mass[mine],
                         angle[mine])
        AgentRouter(col, rank, world, agent_offset=offset)
        ex = make_halo_exchange(lat, rank, world)
        ar = make_uniform_allreduce()
        hist = []
        for _ in range(STEPS):
            col.step(1.0, halo_exchange=ex, allreduce=ar)
            torch.cuda.synchronize()
            hist.append(_state(col, lat))
        col.check_status()
        q.put((rank, band, hist))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize('world,halo', [(2, 8), (3, 5)])
def test_banded_colony_with_migration_equals_single_rank(world, halo):
    import torch.multiprocessing as mp
    from lens_amd.distributed import row_bands
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    cfg, t, params, conc, loc, mass, angle = _colony_inputs()
    col, lat = _make(dev, cfg, t, None, 0, params, conc, loc, mass, angle)
    ref = []
    for _ in range(STEPS):
        col.step(1.0)
        torch.cuda.synchronize()
        ref.append(_state(col, lat))
    assert col.n > N + 20                    # the run divided
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, halo, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted([q.get(timeout=150) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    bands = row_bands(NX, world)
    moved = 0
    for step in range(STEPS):
        per_ref, ord_ref, f_ref = ref[step]
        merged, ords, fields = {}, [], []
        for rank, band, hist in parts:
            per, ordr, f = hist[step]
            assert not set(per) & set(merged)
            merged.update(per)
            ords += ordr
            fields.append(f)
        assert sorted(merged) == sorted(per_ref), step
        # the global order: ordinals are the single-rank positions
        ords.sort()
        assert [o for o, _ in ords] == list(range(len(per_ref))), step
        assert [aid for _, aid in ords] == [aid for _, aid in ord_ref], step
        for aid, arrays in per_ref.items():
            assert merged[aid] == arrays, (step, aid)
        assert np.array_equal(np.concatenate(fields, axis=1), f_ref), step
        # every agent sits in its rank's band (bin rows wrap: get_bin_site, lattice_utils.py:34-40)
        for rank, band, hist in parts:
            for aid in hist[step][0]:
                x = np.frombuffer(hist[step][0][aid]['location'], dtype=np.float64)[0]
                assert band[0] <= int(np.floor(x * NX / NX)) % NX < band[1]
    # some daughters crossed a band edge: agents on a rank their root did not start on
    for rank, band, hist in parts:
        for root, depth, path in hist[-1][0]:
            moved += not (band[0] <= np.floor(loc[0, root]) < band[1])
    assert moved > 0


# ---------------------------------------------------------------------------
# C5-style agent sharding without a lattice: rank-local division + rebalancing
# ---------------------------------------------------------------------------

N5, STEPS5 = 600, 20


def _c5_inputs():
    from lens_amd import configs
    from lens_amd.rate_law_compiler import compile_rate_laws
    cfg = configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10)
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    params, conc = configs.heterogeneous_colony(t, cfg, N5, seed=9, sigma=0.2)
    rng = np.random.default_rng(10)
    mass = rng.uniform(1339.0, 2.4 * 1100.0, N5)
    mass[:N5 // 3] = rng.uniform(2.3 * 1100.0, 2.4 * 1100.0, N5 // 3)     # rank 0 divides first
    return cfg, t, params, conc, mass


def _c5_colony(dev, cfg, t, params, conc, mass):
    from lens_amd.cells import CellModel
    from lens_amd.colony import Colony
    cm = CellModel(model='growth', growth_rate=0.003, division_volume=2.4)
    n = conc.shape[1]
    col = Colony(cfg, n, device=dev, integrator='dopri5', environment='held', table=t, cells=cm,
                 capacity=n + 64)
    col.set_agents(params=params, conc=conc)
    col.set_cell_mass(mass)
    return col


def _c5_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from lens_amd.distributed import AgentBalancer
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        cfg, t, params, conc, mass = _c5_inputs()
        lo, hi = N5 * rank // world, N5 * (rank + 1) // world
        col = _c5_colony(dev, cfg, t, params[:, lo:hi], conc[:, lo:hi], mass[lo:hi])
        bal = AgentBalancer(col, rank, world, tolerance=0.02, agent_offset=lo)
        sizes = []
        for _ in range(STEPS5):
            col.step(1.0)
            sizes.append(col.n)
            bal.balance()
        col.check_status()
        torch.cuda.synchronize()
        q.put((rank, _state_held(col), sizes, bal.moves))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _state_held(col):
    n = col.n
    arrays = {a: getattr(col, a)[..., :n].cpu().numpy() for a in col.agent_array_names()}
    keys = list(zip(arrays['lin_root'].tolist(), arrays['lin_depth'].tolist(), arrays['lin_path'].tolist()))
    return [(k, {a: np.ascontiguousarray(v[..., j]).tobytes() for a, v in arrays.items()})
            for j, k in enumerate(keys)]


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_c5_with_rebalancing_equals_single_rank(world):
    """Agent-per-wavefront DP45 on the C5 network + growth/division, agents
    sharded over ranks and rebalanced after divisions: every agent's state
    equals the single-rank colony's bit for bit (without a lattice agents are
    independent, so their placement -- and the order of the concatenated
    ranks -- changes no result)."""
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    cfg, t, params, conc, mass = _c5_inputs()
    col = _c5_colony(dev, cfg, t, params, conc, mass)
    for _ in range(STEPS5):
        col.step(1.0)
    col.check_status()
    ref = _state_held(col)
    assert col.n > N5 + 50
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted([q.get(timeout=150) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = dict(item for _, st, _, _ in parts for item in st)
    assert len(merged) == sum(len(st) for _, st, _, _ in parts)
    assert sorted(merged) == sorted(k for k, _ in ref)
    for k, b in ref:
        assert merged[k] == b, k
    assert sum(m for _, _, _, m in parts) > 0                  # rebalancing moved agents
    final = [len(st) for _, st, _, _ in parts]
    assert max(final) <= 1.02 * sum(final) / world + 1          # within the balancer's tolerance


# ---------------------------------------------------------------------------
# the multi-rate loop (Colony.run: kinetics and diffusion on their own clocks)
# on row bands
# ---------------------------------------------------------------------------

RUNS = [(3.0, 1.0, 2.5), (5.0, 1.0, 2.5), (2.0, 0.5, 1.5), (4.0, 2.0, 1.0)]   # (interval, kinetics_dt, diffusion_dt)


def _run_colony(dev, band, halo, integrator):
    from lens_amd import configs
    from lens_amd.colony import Colony
    from lens_amd.lattice import Lattice
    cfg, t, params, conc, loc, _, _ = _colony_inputs()
    if band is not None:
        rows = np.floor(loc[0]).astype(int)
        mine = np.flatnonzero((rows >= band[0]) & (rows < band[1]))
        params, conc, loc = params[:, mine], conc[:, mine], loc[:, mine]
    lat = Lattice(['glc__D_e', 'ac_e'], (NX, NY), (float(NX), float(NY)), 10.0, 5.0, device=dev,
                  row_band=band, halo=halo,
                  initial={'glc__D_e': configs.gaussian_bump_field((NX, NY)), 'ac_e': np.zeros((NX, NY))})
    col = Colony(cfg, conc.shape[1], device=dev, integrator=integrator, environment=lat, table=t)
    col.set_agents(params=params, conc=conc, location=loc)
    col.gather_external()
    return col, lat


def _run_worker(rank, world, port, halo, integrator, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from lens_amd.distributed import row_bands, make_halo_exchange, make_uniform_allreduce
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        band = row_bands(NX, world)[rank]
        col, lat = _run_colony(dev, band, halo, integrator)
        ex, ar = make_halo_exchange(lat, rank, world), make_uniform_allreduce()
        hist = []
        for interval, kdt, ddt in RUNS:
            col.run(interval, kinetics_dt=kdt, diffusion_dt=ddt, halo_exchange=ex, allreduce=ar)
            torch.cuda.synchronize()
            hist.append((col.conc[:, :col.n].cpu().numpy().copy(), lat.owned().cpu().numpy().copy()))
        q.put((rank, hist))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize('world,halo,integrator', [(2, 20, 'euler'), (3, 7, 'dopri5')])
def test_banded_multirate_run_equals_single_rank(world, halo, integrator):
    """Colony.run on 2/3 row bands (banded vk_diffuse_delta with halo blocks,
    kinetics and diffusion fronts as Experiment.update schedules them) equals
    the single-domain run bit for bit, agent states and fields."""
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    dev = torch.device('cuda', 0)
    col, lat = _run_colony(dev, None, 0, integrator)
    ref = []
    for interval, kdt, ddt in RUNS:
        col.run(interval, kinetics_dt=kdt, diffusion_dt=ddt)
        torch.cuda.synchronize()
        ref.append((col.conc[:, :col.n].cpu().numpy().copy(), lat.owned().cpu().numpy().copy()))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_worker, args=(r, world, port, halo, integrator, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted([q.get(timeout=150) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i in range(len(RUNS)):
        conc = np.concatenate([hist[i][0] for _, hist in parts], axis=1)   # band-major = global order
        fields = np.concatenate([hist[i][1] for _, hist in parts], axis=1)
        assert np.array_equal(conc, ref[i][0]), i
        assert np.array_equal(fields, ref[i][1]), i


# ---------------------------------------------------------------------------
# HIP-graph replay on multi-rank steps: row bands (sub-graphs between the
# collectives) and agent shards without a per-step collective (C2)
# ---------------------------------------------------------------------------

GSTEPS = 6


def _graph_worker(rank, world, port, halo, q, toggle=False):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from lens_amd.distributed import row_bands, make_halo_exchange, make_uniform_allreduce
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        band = row_bands(NX, world)[rank]
        eager, lat_e = _run_colony(dev, band, halo, 'dopri5')
        graphed, lat_g = _run_colony(dev, band, halo, 'dopri5')
        ex_e, ex_g = make_halo_exchange(lat_e, rank, world), make_halo_exchange(lat_g, rank, world)
        ar = make_uniform_allreduce()
        eager.step(1.0, halo_exchange=ex_e, allreduce=ar)        # first use of every kernel
        graphed.step(1.0, halo_exchange=ex_g, allreduce=ar)
        step = graphed.capture_banded(1.0, ex_g, ar)
        if toggle:
            # the overlap decision is frozen at capture: turning it off afterwards
            # must not drop the first block's interior
            graphed.overlap_halo = False
        same = []
        for _ in range(GSTEPS):
            eager.step(1.0, halo_exchange=ex_e, allreduce=ar)
            step()
            torch.cuda.synchronize()
            n = eager.n
            same.append(bool(torch.equal(eager.conc[:, :n], graphed.conc[:, :n]) and
                             torch.equal(eager.counts[:, :n], graphed.counts[:, :n]) and
                             torch.equal(lat_e.owned(), lat_g.owned())))
        q.put((rank, same, graphed.step_index, len(step.graphs[1])))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize('world,halo,toggle', [(2, 100, False), (3, 7, False), (2, 100, True)])
def test_banded_step_graph_replay_equals_eager(world, halo, toggle):
    """Colony.capture_banded: each rank's step replayed as [kinetics + gather +
    uniform probe] and one graph per halo block, with the halo exchanges and
    the uniform all-reduce issued eagerly between them, equals the eager
    banded step bit for bit on every rank, every step (a band-deep halo: 5
    blocks of 20 substeps; halo 7: 15 blocks)."""
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    halo = min(halo, NX // world)
    procs = [ctx.Process(target=_graph_worker, args=(r, world, port, halo, q, toggle)) for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted([q.get(timeout=150) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same, steps, blocks in parts:
        assert all(same), (rank, same)
        assert steps == GSTEPS + 1
        assert blocks == -(-100 // halo)


def _c2_graph_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from lens_amd import configs
        from lens_amd.colony import Colony
        from lens_amd.rate_law_compiler import compile_rate_laws
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        cfg = configs.glc_lct_config()
        t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
        n_all = 3000
        params, conc = configs.heterogeneous_colony(t, cfg, n_all)
        lo, hi = n_all * rank // world, n_all * (rank + 1) // world
        cols = []
        for _ in range(2):
            c = Colony(cfg, hi - lo, device=dev, integrator='dopri5', table=t, specialize=True)
            c.set_agents(params=params[:, lo:hi], conc=conc[:, lo:hi])
            c.step(1.0)
            cols.append(c)
        replay = cols[1].capture(1.0, 5)        # an agent shard: no per-step collective
        for _ in range(2):
            for _ in range(5):
                cols[0].step(1.0)
            replay()
        torch.cuda.synchronize()
        q.put((rank, bool(torch.equal(cols[0].conc, cols[1].conc) and torch.equal(cols[0].h_state, cols[1].h_state))))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_sharded_c2_graph_replay_equals_eager():
    """C2 on 2 ranks (agents sharded by index, no per-step collective): each
    rank's colony replays its steps from a HIP graph, bit-identical to eager."""
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c2_graph_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = [q.get(timeout=150) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in parts)

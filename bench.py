"""Headline benchmark: agent-steps/s of the batched colony (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c3|c2|c5|kremling]

One "step" = one Delta t = 1 s of the whole colony: every agent's kinetics
(adaptive DP5(4), FP64, rtol 1e-8 / atol 1e-12), the local-environment
gather, 100 diffusion substeps of every lattice field, and the agent-ordered
exchange scatter.  Default workload = BASELINE config 4 (1M agents on a
4096 x 4096 lattice, glucose + acetate), strong-scaled over N ranks by row
bands (one process per GPU, RCCL halo exchange).  Inputs are resident in
HBM before the timed region.  Rank 0 prints one JSON line.

Untimed before the K timed steps: W warmup steps, then settle steps until
the warmup has lasted --settle-ms.  The chip runs the first ~10 ms after an
idle spell slower, and W short steps do not cover that.  On one GPU without
division, the settle steps are replays of a HIP graph of the step that runs
after the capture.  Their count is reported as untimed_settle_steps.
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))


def _gpus_flag(argv):
    """The value of --gpus in `argv` (1 if absent), without the full parser."""
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument('--gpus', type=int, default=1)
    return p.parse_known_args(argv)[0].gpus


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def rank_launch_command(argv, n, port):
    """The child command that runs `bench.py <argv>` as n ranks, one per GPU."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
            '--master-addr', '127.0.0.1', '--master-port', str(port),
            os.path.join(REPO, 'bench.py')] + list(argv)


def launch_ranks(argv, environ=None, popen=subprocess.Popen):
    """Make `--gpus N` mean N ranks.  Runs before anything touches the GPU.

    - WORLD_SIZE unset and N > 1: start torch.distributed.run with N ranks as a
      CHILD process (never an exec: on this pool a process that initialised
      the GPU must not be replaced), wait for it, and return its exit code.
    - WORLD_SIZE set and different from N: exit non-zero (a launcher with a
      different rank count than the run claims).
    - Otherwise return None: this process is a rank (or the only one).

    Replaces the reference's parallel dispatch of agent processes
    (/root/reference/vivarium/core/experiment.py:1171-1178) at the job level:
    one process per GPU."""
    environ = os.environ if environ is None else environ
    n = _gpus_flag(argv)
    if n < 1:
        raise SystemExit('bench.py: --gpus must be >= 1 (got %d)' % n)
    world = environ.get('WORLD_SIZE')
    if world is not None:
        if int(world) != n:
            raise SystemExit('bench.py: --gpus %d but WORLD_SIZE=%s: the launcher started a different number '
                             'of ranks than the run reports' % (n, world))
        return None
    if n == 1:
        return None
    child = popen(rank_launch_command(argv, n, _free_port()))

    def forward(signum, _frame):
        child.send_signal(signum)
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        return child.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)


if __name__ == '__main__':
    # before lens_amd (which loads the HIP library) and before any torch.cuda call
    _rc = launch_ranks(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, REPO)

from lens_amd import configs  # noqa: E402
from lens_amd.colony import Colony  # noqa: E402
from lens_amd.lattice import Lattice, n_substeps  # noqa: E402
from lens_amd.rate_law_compiler import compile_rate_laws  # noqa: E402

METRIC = 'agent-steps/sec (whole node) at 1M agents; FP64 % peak; stencil HBM GB/s'
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: 8 TB/s spec
FP64_PEAK_TFLOPS = 78.6         # 256 CU x 4 SIMD x 16 lanes x 2 x 2.4 GHz (vector FP64, spec)

WORKLOADS = {
    # name: (agents, lattice n, bounds um, description)
    'c4': (1_000_000, 4096, 4096.0, 'BASELINE config 4: 1M agents + 4096x4096 diffusion_field lattice'),
    'c3': (100_000, 1024, 1024.0, 'BASELINE config 3: 100k agents + 1024x1024 diffusion_field lattice'),
    'c2': (10_000, 0, 0.0, 'BASELINE config 2: 10k heterogeneous agents, no lattice'),
    'c5': (1_000_000, 0, 0.0, 'BASELINE config 5: 50-species / 40-reaction network per agent (~85 integrated '
                              'components, agent-per-wavefront DP45) + Growth/DeriveGlobals/DivisionVolume '
                              'division events'),
    'kremling': (1_000_000, 0, 0.0, 'BASELINE config 5 known-answer: the reference\'s stiff Kremling 2007 sugar '
                                    'transport ODE (odeint path, 11 states + 4 flux integrals, 100-point output '
                                    'grid per 1 s step), heterogeneous agents'),
}

# Kremling2007_transport.py:220-351 (oracle/kremling.rhs), counted as executed on the
# G6P branch: uptake1 4, uptake2 13, hill 9, synthesis 11, rgly/rpdh 2, rpts 6,
# f/rpyk 4, mu 3, derivatives 19 (a divide = 1 flop, XP**6 = 3 multiplies)
KREMLING_RHS_FLOPS = 71
N_SIMDS = 256 * 4          # MI355X: 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
KREMLING_NY = 15
SPLIT_STEPS = 6            # eager steps timed for the kinetics / diffusion split (the first is dropped)


def stencil_kernel_name(variant, depth, mode='exact', pass_bytes=None):
    """rocprof name of the non-final fused pass of `depth` substeps (vk_diffuse):
    the full template argument list, as rocprofv3 prints it.  ``pass_bytes``
    (source + destination rows of one pass): a 10-deep pass of at most 192 MiB
    stores through the caches (vk_stencil_ps10.hip), CP = 2.  The tolerance mode
    runs pair-sum passes at depths 3-11 (odd) and 10, whatever the variant but 40;
    other depths, and the exact mode, run the wave tiles (vk_lattice.hip launch_pass)."""
    if mode == 'fma' and depth <= 11 and (depth % 2 == 1 or depth == 10):
        if variant == 40 and depth == 10:
            return 'vk_sp::k_diffuse_sp<10, 4, 2, 5, true, 0>'
        # k_diffuse_ps<K, PD, C, SC, CP, KHO> (vk_stencil_ps.h); SC = the rescaled form (coef not
        # ~1/4); KHO = 16 halo columns for variant 70's line-aligned 10-deep tiles
        kho = 16 if (variant == 70 and depth == 10) else 0
        if depth == 10 and pass_bytes is not None and pass_bytes <= 192 * 1024 * 1024:
            return 'vk_ps::k_diffuse_ps<10, 4, 2, true, 2, %d>' % kho
        return 'vk_ps::k_diffuse_ps<%d, 4, 2, true, 0, %d>' % (depth, kho)
    if depth == 10:    # the exact mode's 10-deep whole-step plan
        return 'vk_nt::k_diffuse_wl<10, 3, false>'
    if variant in (6, 20, 40) and depth in (7, 9, 11):
        return 'vk_nt::k_diffuse_wl<%d, 6, false>' % depth
    return 'k_diffuse_wl<%d, %d, false>' % (depth, 3 if variant == 2 else 6)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=None,
                   help='timed steps (default 10; C2, whose replayed step is ~5 us, 200 so that the timed '
                        'region is not the barrier and synchronisation around it)')
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--workload', default='c4', choices=sorted(WORKLOADS))
    p.add_argument('--integrator', default='dopri5', choices=['dopri5', 'euler'])
    p.add_argument('--halo', type=int, default=None,
                   help='halo depth = substeps per halo exchange (multi-GPU; default min(100, band rows): '
                        'one exchange per step; scripts/halo_sweep.py, profiles/r02_halo_sweep/)')
    p.add_argument('--exchange', default='sorted', choices=['sorted', 'atomic'])
    p.add_argument('--no-sort-agents', dest='sort_agents', action='store_false',
                   help='keep the agents in their generated order instead of bin order (Colony.sort_by_bin)')
    p.add_argument('--generic-kernel', action='store_true',
                   help='use the table-walking DP45 kernel instead of the specialised one')
    p.add_argument('--stencil-kernel', type=int, default=None, choices=[2, 3, 6, 20, 40, 70],
                   help='tolerance mode: 20 = pair-sum passes (default on one GPU), 40 = the 10-deep pair-sum '
                        'pass with its stages split '
                        'over a workgroup\'s waves (default on row bands), 6 = the variant-6 FMA form; exact '
                        'mode: 2 / 3 = wave tiles prefetching 3 / 6 rows, 6 (and 20, 40) = 3 with streaming '
                        'stores')
    p.add_argument('--stencil-depth', type=int, default=None,
                   help='substeps fused per HBM pass (odd, or 10: tolerance-mode whole steps as 10-deep passes); '
                        'default 10 for C4 in the fma mode, else 9')
    p.add_argument('--stencil-mode', default='fma', choices=['fma', 'exact'],
                   help='fma (default): tolerance mode, FMA-contracted passes within 1e-13 of the exact mode '
                        '(tests/test_stencil_modes.py); exact: bit-identical with scipy.ndimage.convolve')
    p.add_argument('--stencil-rows', type=int, default=None,
                   help='output rows per wave tile (default: 34 for C4 on one GPU, else 0 = auto by band height '
                        'and wave count)')
    p.add_argument('--dist-backend', default='nccl', choices=['nccl', 'gloo'],
                   help='nccl (= RCCL) for real runs; gloo stages through host memory (rehearsal only)')
    p.add_argument('--overlap-kinetics', action='store_true',
                   help='run kinetics + gather on a side stream beside the diffusion passes')
    p.add_argument('--graph', choices=['auto', 'on', 'off'], default='auto',
                   help='replay the timed steps from a captured HIP graph (auto: every single-GPU step that takes '
                        'no host decision, i.e. no division: C2, C3, C4)')
    p.add_argument('--couple', action='store_true',
                   help='carry the gather and the exchange in the first / final diffusion pass (vk_diffuse_coupled; '
                        'same results; off by default: 1.533 vs 1.511 ms per C4 step, profiles/r04/r04h)')
    p.add_argument('--steps-per-launch', type=int, default=None,
                   help='held colonies (C2): timesteps per kernel launch (vk_step_dopri5_multi, each step bit for '
                        'bit the one-step kernel\'s); default = the steps per replayed graph')
    p.add_argument('--settle-ms', type=float, default=30.0,
                   help='after the W warmup steps, run more untimed steps until the warmup has kept the GPU '
                        'busy this long (power-management transient, profiles/r02g_eager_trace_gaps.log); '
                        'reported as untimed_settle_steps')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--secondary-steps', type=int, default=10,
                   help='C4 on one GPU: timed steps of the bounded C5 and Kremling legs (0 = skip them)')
    p.add_argument('--cpu-seconds', type=float, default=12.0)
    args = p.parse_args(argv)
    if args.steps is None:
        args.steps = 200 if args.workload == 'c2' else 10
    return args


def stencil_settings(args, world):
    """(mode, depth, kernel, rows) of the fused passes for this run -- what the
    bench times, and what tests/test_configs.py checks at full size."""
    depth = args.stencil_depth
    if depth is None:
        # 100 substeps as 10 passes of 10 instead of 8 x 9 + 4 x 7: -2.3 % per 100 substeps,
        # -3 % per step (profiles/r03/r03v/); the 10-deep pass keeps the 9-deep pass's column
        # halo (KH = 10)
        # (row bands too: a middle rank's step at N = 2 / 4 / 8 runs 0.968 / 0.610 / 0.432 ms
        # against 0.995 / 0.628 / 0.450 at depth 9, profiles/r03/r03x_rank_emulate.log)
        # (exact mode too since round 4: 1.830 / 1.850 / 1.827 against 1.873 / 1.867 / 1.908 ms
        # per C4 step at depth 9, profiles/r04/r04af/)
        # (C3 in the tolerance mode too, with the stage-split pass below)
        depth = 10 if (args.workload == 'c4' or (args.workload == 'c3' and args.stencil_mode == 'fma')) else 9
    kernel = args.stencil_kernel
    if kernel is None:
        # row bands (N > 1) and C3 in the tolerance mode: the stage-split 10-deep pass, whose
        # chunks fill whole rounds of resident workgroups (vk_sp::round_rows; a middle rank's
        # step at N = 8 / 4 / 2: 0.333 / 0.498 / 0.803 against 0.372 / 0.544 / 0.884 ms with
        # variant 20, profiles/r05/r05fg/, r05r/; C3 0.222 against 0.320 ms per step with the
        # 9-deep variant-20 plan, r05q/); the whole C4 plane keeps variant 20 (a tie, r05r/)
        # (N = 2 keeps variant 20 since the edge-first tile order: 0.746 against 0.762 ms, r05w/;
        # N = 4 too since the XCD-aware block order of the pair-sum pass: 0.436 / 0.434 / 0.433
        # against 0.447 / 0.439 / 0.434 ms, r05bm/, r05bn/; N = 8 keeps variant 40: 0.295 / 0.297
        # against 0.305 / 0.305)
        kernel = 40 if ((world > 4 or args.workload == 'c3') and args.stencil_mode == 'fma' and depth == 10) else 20
        # the whole C4 plane: variant 70, the 10-deep pass with line-aligned tiles (96 written
        # columns; 1.262-1.273 against 1.280-1.303 ms per C4 step, passes 1.160 against 1.188 ms
        # per step, profiles/r06/r06l/); row bands keep theirs (N = 2 / 4 / 8: 0.693 / 0.438 /
        # 0.315 against 0.687 / 0.432 / 0.297 ms with variant 20 / 20 / 40, r06m/)
        if kernel == 20 and world == 1 and args.workload == 'c4' and args.stencil_mode == 'fma' and depth == 10:
            kernel = 70
    rows = args.stencil_rows
    if rows is None:
        # 64-row tiles on the whole 4096^2 plane (64 chunks of each plane exactly): since the
        # edge-first tile order and the side-tile body, 1.290-1.307 ms per C4 step against
        # 1.311 at 32 rows, 1.321-1.345 at 34 (the choice while the last wave round held the
        # edge tiles, profiles/r03/r03h_stencil_rows_sweep.log), 1.320-1.327 at 68 and
        # 1.35-1.61 at 60 / 72-128 (profiles/r05/r05an-r05ap); else the auto rule (chunk_rows)
        rows = 64 if (world == 1 and args.workload == 'c4') else 0
    return args.stencil_mode, depth, kernel, rows


def settle_steps_needed(warmup_s: float, warmup_steps: int, settle_ms: float, cap: int = 2000) -> int:
    """Untimed steps to add after `warmup_steps` steps that took `warmup_s` seconds
    so that the warmup lasts at least `settle_ms` (at the warmup's own pace)."""
    if settle_ms <= 0 or warmup_steps <= 0:
        return 0
    per = max(warmup_s / warmup_steps, 1e-6)
    return int(min(cap, np.ceil(max(0.0, settle_ms * 1e-3 - warmup_s) / per)))


def build_rank(args, rank, world, dev):
    """This rank's share of the workload: (colony, lattice or None, host inputs).
    ``args.agents`` (optional) overrides the agent count (tests)."""
    n_total, nx, bound, _ = WORKLOADS[args.workload]
    n_total = getattr(args, 'agents', None) or n_total
    cells = None
    if args.workload == 'c5':
        from lens_amd.cells import CellModel
        cfg = configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10)
        cells = CellModel(model='growth', growth_rate=0.0006, division_volume=2.4)
    else:
        cfg = configs.glc_ac_config() if nx else configs.glc_lct_config()
    table = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    rng = np.random.default_rng(configs.SEED + rank)
    lat = None
    if nx:
        from lens_amd.distributed import row_bands
        band = row_bands(nx, world)[rank]
        n_local = n_total // world + (1 if rank < n_total % world else 0)
        glc = configs.gaussian_bump_field((nx, nx))
        lat = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (bound, bound), 10.0, 5.0, device=dev,
                      row_band=band if world > 1 else None,
                      halo=(args.halo if args.halo is not None else min(100, band[1] - band[0])) if world > 1 else 0,
                      initial={'glc__D_e': glc, 'ac_e': np.zeros((nx, nx))})
        x = rng.uniform(band[0] * bound / nx, band[1] * bound / nx, n_local)
        y = rng.uniform(0.0, bound, n_local)
        loc = np.stack([x, y])
    else:
        n_local = n_total // world + (1 if rank < n_total % world else 0)
    params, conc = configs.heterogeneous_colony(table, cfg, n_local, seed=configs.SEED + rank,
                                                sigma=0.2 if cells is not None else 0.25)
    col = Colony(cfg, n_local, device=dev, integrator=args.integrator, environment=lat or 'held',
                 table=table, exchange=args.exchange, specialize=not args.generic_kernel, cells=cells,
                 capacity=int(n_local * 1.05) + 64 if cells is not None else None)
    col.overlap_kinetics = bool(getattr(args, 'overlap_kinetics', False))
    col.set_agents(params=params, conc=conc, location=loc if nx else None)
    if nx and getattr(args, 'sort_agents', False):
        # agents stored in bin order: the exchange and the gather stream (Colony.sort_by_bin);
        # the host copies follow, for the CPU baseline
        order = col.sort_by_bin().cpu().numpy()
        params, conc, loc = params[:, order], conc[:, order], loc[:, order]
    if cells is not None:
        # a colony spread over one generation: divisions every step from the start
        col.set_cell_mass(rng.uniform(1339.0, 2.4 * 1100.0, n_local))
    if nx:
        col.gather_external()
    return col, lat, (params, conc, loc if nx else None)


def pass_plan(n_sub, depth):
    """Substeps of each fused pass of one whole step, as vk_diffuse plans it
    (vk_lattice.hip odd_plan / the 10-deep block plan)."""
    if depth == 10 and n_sub % 10 == 0:
        return [10] * (n_sub // 10)
    d = min(9 if depth == 10 else depth | 1, 15)
    passes = (n_sub + d - 1) // d
    if (passes & 1) != (n_sub & 1):
        passes += 1
    ks, j, left = [], 0, passes
    while j < n_sub:
        rem = n_sub - j
        k = (rem + left - 1) // left
        k += 1 - (k & 1)
        k = min(k, d)
        while k > 1 and rem - k < left - 1:
            k -= 2
        ks.append(k)
        j += k
        left -= 1
    return ks


def time_stencil_pass(lat, depth, reps=5):
    """Average duration of one fused pass of `depth` substeps as the step runs it:
    whole 100-substep steps of the planes through vk_diffuse (its block plan, the
    passes rotating through the three buffers, the cone of a row band), HIP events
    on the launch stream, divided by the passes per step.  The planes are restored
    afterwards.  (A single pass repeated on the same buffers ran ~5 % faster than
    the same kernel inside the step, rocprof: profiles/r05/r05ah/.)"""
    from lens_amd import native
    lo_min = lat.row_lo if lat.edge_top else 0
    hi_max = lat.row_hi if lat.edge_bot else lat.rows_local
    coeff = lat.diffusion * 0.01
    n_passes = len(pass_plan(100, depth))
    saved = lat.fields.clone()

    def one():
        native.check(native._lib.vk_diffuse(
            native.ptr(lat.fields), native.ptr(lat.work0), native.ptr(lat.work1), len(lat.molecules),
            lat.field_stride, lat.ny, lat.row_lo, lat.row_hi, lo_min, hi_max, int(lat.edge_top),
            int(lat.edge_bot), 0, 100, 100, coeff, 0, native.stream_handle()), 'vk_diffuse')
    one()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        one()
    e1.record()
    torch.cuda.synchronize()
    lat.fields.copy_(saved)
    return e0.elapsed_time(e1) / (reps * n_passes)


def time_copy_floor(lat, reps=20):
    """Average duration of the box's fastest streaming copy of the planes a pass
    streams (one 8-B read + one 8-B write per cell, the algorithmic bytes of one
    fused pass): vk_copy_stream, one 16-B element per thread with a non-temporal
    store -- 84.4 us / 6.36 TB/s for the 4096^2 x 2 pair in
    scripts/micro/copy_floor.hip, where torch's copy_ (the round-1..5 floor) took
    ~99 us / 5.4 TB/s.  HIP events on the launch stream.  The copies ping-pong
    between the two work buffers (scratch between steps), so every copy reads
    what the previous one streamed out past the 256 MiB Infinity Cache: one
    source read twenty times over (fields -> work0) stays in that cache -- the
    plane pair is 256 MiB -- and read at 7.4 TB/s (profiles/r06/r06c/), which is
    no HBM floor."""
    from lens_amd import native
    bufs = (lat.work0.reshape(-1), lat.work1.reshape(-1))
    n = bufs[0].numel() & ~1

    def one(r):
        src, dst = bufs[r & 1], bufs[1 - (r & 1)]
        native.check(native._lib.vk_copy_stream(native.ptr(src), native.ptr(dst), n, native.stream_handle()),
                     'vk_copy_stream')
    for r in range(4):
        one(r)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for r in range(reps):
        one(r)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, 16.0 * n


def cpu_baseline(args, col, host_state):
    """The oracle's C restatement (OpenMP) on this host, on a bounded sample of
    the same workload: whole steps, repeated until ~cpu_seconds have passed."""
    from oracle import cpu
    threads = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(os.sched_getaffinity(0))
    os.environ.setdefault('OMP_NUM_THREADS', str(threads))
    cpu.build()
    params, conc, loc = host_state
    t = col.table
    desc = cpu.Desc(t)
    n = conc.shape[1]
    if col.lattice is None and n > 4096:
        # no lattice: agents are independent -> a bounded sample of them, scaled per agent
        n = 4096
        params = np.ascontiguousarray(params[:, :n])
        conc = np.ascontiguousarray(conc[:, :n])
    conc = conc.copy()
    m2c = col.m2c[:n].cpu().numpy().copy()
    h = np.zeros(n)
    lat = col.lattice
    fields = None
    if lat is not None:
        nx = lat.n_bins[0]
        fields = [np.ascontiguousarray(configs.gaussian_bump_field((nx, nx))), np.zeros((nx, nx))]
        coef = lat.diffusion * 0.01
        n_sub = n_substeps(1.0)
        bin_lin = col.bin_lin[:n].cpu().numpy().astype(np.int32)
    steps, t0 = 0, time.perf_counter()
    while True:
        _, counts, _, _ = cpu.step_dopri5(desc, 1.0, params, conc, m2c, h_state=h,
                                          rtol=col.rtol, atol=col.atol)
        if fields is not None:
            for f in fields:
                cpu.diffuse(f, coef, n_sub)
            for e, mol in enumerate(t.external_ids):
                fi = lat.molecules.index(mol)
                cpu.exchange(fields[fi].reshape(-1), bin_lin, counts[e], lat.binvol_avogadro)
        steps += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or steps >= 20 or (fields is None and el >= args.cpu_seconds / 3):
            break
    return {'value': steps * n / el, 'unit': 'agent-steps/s', 'cores': threads, 'kind': 'port',
            'sample': '%d full step(s) of %d agents of the same workload (DP45 kinetics%s), %.1f s, '
                      'oracle/cpu_kinetics.c with OpenMP%s' % (
                          steps, n, ' + 100-substep stencil x %d fields + exchange' % len(fields)
                          if fields is not None else '', el,
                          '; growth/division not included (negligible work)' if col.cells is not None else '')}


def kremling_colony(n, dev, seed):
    """Heterogeneous Kremling colony: GLC_G6P condition, internal x U(0.7, 1.3),
    external x U(0.5, 1.5), volume U(0.5, 3) fL (tests/test_kremling.py's spread)."""
    from lens_amd import kremling as lk
    rng = np.random.default_rng(seed)
    s0 = np.array([lk.GLC_G6P_INTERNAL[k] for k in lk.INTERNAL] + [lk.GLC_G6P_MEDIA[k] for k in lk.EXTERNAL])
    states = np.repeat(s0[:, None], n, axis=1)
    states[:8] *= rng.uniform(0.7, 1.3, (8, n))
    states[8:11] *= rng.uniform(0.5, 1.5, (3, n))
    col = lk.KremlingColony(n, device=dev)
    col.set_state(states)
    col.volume.copy_(torch.from_numpy(rng.uniform(0.5, 3.0, n)))
    return col, states, col.volume.cpu().numpy()


def cpu_baseline_odeint_worker(job):
    """One agent-step through scipy's odeint (LSODA) on the restated right-hand side."""
    kind, payload = job
    if kind == 'kremling':
        from oracle import kremling as ok
        state, vol = payload
        ok.step(np.asarray(state), volume_fL=vol)
    else:
        from oracle.kinetics import OracleODE, params_dict
        cfg, param_names, pvec, conc, m2c = payload
        ode = OracleODE(cfg['reactions'], params_dict(param_names, cfg, pvec))
        ode.step(conc, 1.0, m2c, rtol=1e-8, atol=1e-12)
    return 1


def cpu_baseline_odeint(jobs, seconds, cores):
    """SURVEY §8d CPU leg (ii): the reference's own algorithm -- scipy.integrate.odeint
    (ODEPACK LSODA), one call per agent-step as Kremling2007_transport.py:384 makes
    it -- on the restated right-hand side, over every host core (multiprocessing),
    on a sample of the workload's agents, timed and scaled to agent-steps/s."""
    from multiprocessing import get_context
    with get_context('spawn').Pool(cores) as pool:       # fresh interpreters: nothing of the GPU process
        pool.map(cpu_baseline_odeint_worker, jobs[:cores], chunksize=1)     # start-up off the clock
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            done += sum(pool.map(cpu_baseline_odeint_worker, jobs, chunksize=max(1, len(jobs) // (4 * cores))))
        el = time.perf_counter() - t0
    return {'value': done / el, 'unit': 'agent-steps/s', 'cores': cores, 'kind': 'port',
            'sample': '%d agent-steps (%d sampled agents, repeated) through scipy odeint (LSODA) on the '
                      'restated RHS, multiprocessing over %d cores, %.1f s' % (done, len(jobs), cores, el)}


def run_kremling(args, rank, world, dev, dist):
    n_total = getattr(args, 'agents', None) or WORKLOADS['kremling'][0]
    n_local = n_total // world + (1 if rank < n_total % world else 0)
    col, states, vols = kremling_colony(n_local, dev, configs.SEED + rank)
    for _ in range(args.warmup):
        col.step(1.0)
    torch.cuda.synchronize()
    col.check_status()
    attempts = torch.zeros((), dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        col.step(1.0)
        attempts += col.nsteps.sum()
    e1.record()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    col.check_status()
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    agents = torch.tensor([float(n_local * args.steps)], dtype=torch.float64, device=dev)
    if dist is not None:
        if args.dist_backend == 'gloo':
            el, agents = el.cpu(), agents.cpu()
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(agents, op=dist.ReduceOp.SUM)
    if rank != 0:
        return None
    kms = e0.elapsed_time(e1) / args.steps
    att = float(attempts.item()) / (n_local * args.steps)
    flops_attempt = 6 * KREMLING_RHS_FLOPS + 64 * KREMLING_NY
    tflops = att * flops_attempt * n_local / (kms * 1e-3) / 1e12
    bytes_agent = 8 * (11 + 1 + 1) + 8 * (8 + 4 + 3 + 1) + 8
    out = {
        'metric': METRIC, 'value': float(agents.item()) / float(el.item()), 'unit': 'agent-steps/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': float(el.item()) / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'strong',
        'vs_baseline': None, 'dtype': 'f64',
        'data': 'synthetic (seeded heterogeneous Kremling colony around the reference GLC_G6P condition)',
        'config': {'workload': WORKLOADS['kremling'][3], 'agents': n_total, 'dt_s': 1.0, 'output_grid': 100,
                   'integrator': 'dopri5 landing on the odeint output grid', 'rtol': col.rtol, 'atol': col.atol,
                   'parallelism': 'agents x%d' % world},
        'roofline': {'bound': 'fp64-valu', 'kernel': 'k_kremling_step', 'achieved': tflops,
                     'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': tflops / FP64_PEAK_TFLOPS,
                     'traffic': None, 'avg_launch_ms': kms, 'dp45_attempts_per_agent_step': att,
                     'flops_per_attempt': flops_attempt,
                     'hbm_gbps': n_local * bytes_agent / (kms * 1e-3) / 1e9},
    }
    if world == 1 and not args.no_cpu_baseline:
        cores = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(os.sched_getaffinity(0))
        jobs = [('kremling', (states[:, a].tolist() + [0.0] * 4, float(vols[a]))) for a in range(0, n_local, n_local // 256)]
        out['cpu_baseline'] = cpu_baseline_odeint(jobs, args.cpu_seconds, cores)
    return out


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # one rank per GPU; a rehearsal with more ranks than GPUs (--dist-backend gloo) shares them
    dev = torch.device('cuda', local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)       # RCCL over xGMI
        else:
            dist.init_process_group(args.dist_backend)
    if args.workload == 'kremling':
        out = run_kremling(args, rank, world, dev, dist)
    else:
        out = run(args, rank, world, dev, dist)
    if out is not None and world == 1 and args.workload == 'c4' and args.secondary_steps > 0:
        # the north star's FP64 bar is carried by C5 and Kremling: bounded legs of both,
        # after the headline and outside its timed region, in the same JSON line
        out['secondary'] = secondary_legs(args, dev)
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def run(args, rank, world, dev, dist):
    """One lattice / agent-shard workload (everything but Kremling): warmup, the
    timed steps, the split and the roofline; rank 0 returns the JSON object."""
    from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode
    args.stencil_mode, args.stencil_depth, args.stencil_kernel, args.stencil_rows = stencil_settings(args, world)
    stencil_depth(args.stencil_depth)
    stencil_mode(args.stencil_mode)
    stencil_kernel(args.stencil_kernel, args.stencil_rows)
    col, lat, host_state = build_rank(args, rank, world, dev)
    col.fuse_coupling = bool(args.couple)
    halo_ex = allred = balancer = None
    if world > 1 and lat is not None:
        from lens_amd.distributed import make_halo_exchange, make_uniform_allreduce
        halo_ex = make_halo_exchange(lat, rank, world)
        # the uniform summary's all-reduce gets a communicator of its own: on the default
        # group it would queue behind the first halo exchange (one NCCL stream per group)
        # and the band's interior passes, which need the summary, could not overlap it
        allred = make_uniform_allreduce(group=dist.new_group(list(range(world))))
    elif world > 1 and col.cells is not None:
        # agent-sharded C5: divisions are rank-local; even the shards out when
        # they drift more than 5 % apart (one all_to_all)
        from lens_amd.distributed import AgentBalancer
        balancer = AgentBalancer(col, rank, world, tolerance=0.05)

    def one_step(timing):
        col.step(1.0, halo_exchange=halo_ex, allreduce=allred, timing=timing)
        if balancer is not None:
            balancer.balance()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    ev = lambda: torch.cuda.Event(enable_timing=True)
    mk = lambda: ({'kin': (ev(), ev()), 'diff': (ev(), ev())} if lat is not None else {'kin': (ev(), ev())})
    # Per-step bookkeeping inside the timed region is kept to what cannot be had
    # afterwards.  Lattice steps record no HIP events (the kinetics / diffusion
    # split comes from eager steps after the timed region).  A non-dividing
    # colony integrates the same agents every step, so its DP45 attempts are read
    # from the last step's per-agent counts (a per-step torch reduction or device
    # copy of the counts is a launch of its own in every step).  Eager vs graph
    # C4: profiles/r02f_eager_vs_graph.log, profiles/r02g_eager_trace_gaps.log.
    timing = [mk() if lat is None else None for _ in range(args.steps)]
    # with division the per-agent counts are reshuffled after the kinetics: the
    # colony sums them itself, right after the launch (an 85-ms C5 step does not
    # notice the reduction)
    divides = col.cells is not None
    col.count_attempts(divides)
    # The status check's first call loads torch's nonzero kernels (~40 ms with the
    # GPU idle).  Done only after the warmup, that idle sat right before the timed
    # region: the chip then ran the first ~10 ms of renewed load up to 40 % slower
    # (every kernel, profiles/r02g_eager_trace_gaps.log).  So it runs first.
    col.check_status()
    barrier()
    # HIP-graph replay of the timed steps: every step whose launch sequence takes no
    # host decision (one GPU, no division).  A C2 step is one 4-us launch that costs
    # 40 us to issue from Python.  Multi-GPU steps stay eager (host-driven halo
    # collectives).
    # Multi-GPU: an agent shard without a lattice (C2) has no per-step collective and
    # replays like one GPU; a row band replays the launch sequences between its
    # collectives (Colony.capture_banded), which stay eager.
    banded = lat is not None and world > 1
    use_graph = (args.graph == 'on' or (args.graph == 'auto' and col.cells is None)) and balancer is None
    # warmup runs exactly the timed loop body (first-use costs land here)
    t_warm = time.perf_counter()
    for k in range(args.warmup):
        one_step(mk() if lat is None else None)
    barrier()
    # Settle: the chip runs the first ~10 ms of load after an idle spell up to
    # 40 % slower (profiles/r02g_eager_trace_gaps.log), and W short steps (a
    # 0.3-ms banded step at 8 GPUs) do not cover that.  More untimed steps run
    # until the warmup has lasted --settle-ms; every rank runs the same count.
    # With graph replay the settle replays come after the capture (below).
    settle_steps = 0
    if args.settle_ms > 0 and args.warmup > 0 and (not use_graph or banded):
        need = torch.tensor([float(settle_steps_needed(time.perf_counter() - t_warm, args.warmup, args.settle_ms))],
                            dtype=torch.float64, device=dev)
        if dist is not None:
            if args.dist_backend == 'gloo':
                need = need.cpu()
            dist.all_reduce(need, op=dist.ReduceOp.MAX)
        settle_steps = int(need.item())
        for k in range(settle_steps):
            one_step(mk() if lat is None else None)
        barrier()
    col.check_status()
    graph_info = None
    if use_graph and banded:
        banded_step = col.capture_banded(1.0, halo_ex, allred)
        banded_step()                        # first replay of the segment graphs: warmup, not timed
        barrier()
        col.check_status()
        settle_steps += 1
        graph_info = {'mode': 'row-band segments: [kinetics + gather + uniform probe] and one graph per halo '
                              'block replayed, halo exchange and uniform all-reduce eager',
                      'graphs_per_step': 1 + len(banded_step.graphs[1])}
    elif use_graph:
        # a held colony's agents do not couple between steps: a graph of up to 100 steps
        # is one launch of that many steps (vk_step_dopri5_multi) instead of one per step
        multi_ok = (lat is None and col.cells is None and col.integrator == 'dopri5' and
                    col.engine.default_variant() == 2)
        per_graph = next(g for g in ((100, 50, 20, 10, 5, 2, 1) if multi_ok else (10, 5, 2, 1))
                         if args.steps % g == 0)
        spl = args.steps_per_launch if args.steps_per_launch is not None else (per_graph if multi_ok else 1)
        if spl > 1 and (not multi_ok or per_graph % spl):
            raise SystemExit('--steps-per-launch: a held DP45 colony, dividing the %d steps per graph' % per_graph)
        replay = col.capture(1.0, per_graph, steps_per_launch=spl)
        replay()             # uploads the graph; its steps are warmup, not timed
        barrier()
        col.check_status()
        if args.settle_ms > 0:
            # the capture left the GPU idle: settle again, with replays, right
            # before the timed region (a 10-step C3 replay lasts only 3.7 ms)
            t_rep = time.perf_counter()
            replay()
            barrier()
            need = torch.tensor([float(settle_steps_needed(time.perf_counter() - t_rep, 1, args.settle_ms))],
                                dtype=torch.float64, device=dev)
            if dist is not None:
                if args.dist_backend == 'gloo':
                    need = need.cpu()
                dist.all_reduce(need, op=dist.ReduceOp.MAX)
            for k in range(int(need.item())):
                replay()
            barrier()
            settle_steps += (1 + int(need.item())) * per_graph
        graph_info = {'steps_per_graph': per_graph, 'replays': args.steps // per_graph,
                      'untimed_warmup_replay_steps': per_graph, 'steps_per_launch': spl}
    agent_steps = 0          # agents integrated, summed over the timed steps (divisions grow n)
    n_start = col.n
    if divides:
        col.attempts.zero_()
    barrier()
    if use_graph and banded:
        t0 = time.perf_counter()
        for k in range(args.steps):
            agent_steps += col.n
            banded_step()
    elif use_graph:
        e_all = (ev(), ev())
        t0 = time.perf_counter()
        e_all[0].record()
        for k in range(args.steps // per_graph):
            agent_steps += col.n * per_graph
            replay()
        e_all[1].record()
    else:
        att_hist = torch.zeros(args.steps, dtype=torch.int64, device=dev) if divides else None
        n_hist = []
        t0 = time.perf_counter()
        for k in range(args.steps):
            n_k = col.n                   # agents integrated this step (division comes after the kinetics)
            agent_steps += n_k
            one_step(timing[k])
            n_hist.append(n_k)
            if divides:
                att_hist[k] = col.attempts        # running total (the colony's own sum)
    barrier()
    elapsed = time.perf_counter() - t0
    col.check_status()
    stencil_pass_ms = time_stencil_pass(lat, args.stencil_depth) if lat is not None else None
    exact_pass_ms = None
    if lat is not None and args.stencil_mode != 'exact':
        stencil_mode('exact')             # the bit-exact pass on the same planes, for comparison
        exact_pass_ms = time_stencil_pass(lat, args.stencil_depth)
        stencil_mode(args.stencil_mode)
    copy_floor = time_copy_floor(lat) if lat is not None and world == 1 else None
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    n_agents = torch.tensor([float(agent_steps)], dtype=torch.float64, device=dev)
    per_step = None
    attempts_from = 'per-agent attempt counts of the last timed step x steps'
    if divides:
        cum = att_hist.cpu().numpy().astype(float)
        attempts = float(col.attempts.item())
        per_step = [round(a / n, 4) for a, n in zip(np.diff(np.concatenate([[0.0], cum])), n_hist)]
        attempts_from = 'colony sum after every kinetics launch'
    else:                             # same agents every step (no division): last step x steps
        attempts = float(col.nsteps[:col.n].sum().item()) * args.steps
    if lat is None and use_graph:     # the replayed step is the kinetics launch
        kin_ms = e_all[0].elapsed_time(e_all[1]) / args.steps
        diff_ms = None
    elif lat is None:
        kin_ms = sum(t['kin'][0].elapsed_time(t['kin'][1]) for t in timing) / args.steps
        diff_ms = None
    elif use_graph and not banded:
        # The kinetics / diffusion split from graph-replayed steps: a replay of the
        # timed steps' graph with device timestamps (vk_timestamp, one-lane kernels)
        # before the kinetics, after it, and at the end of every step.  Each stamp
        # adds a launch boundary (~1-2 us) inside the step; the stamped step is
        # reported beside ms_per_step.  (torch refuses events inside a graph on
        # ROCm; eager steps after the timed region ran ~7 % longer than replayed
        # ones, r03 VERDICT.)
        from lens_amd import native
        stamps = torch.zeros(3 * per_graph, dtype=torch.int64, device=dev)
        replay_s = col.capture(1.0, per_graph, stamps=stamps)
        replay_s()                        # upload
        barrier()
        kin_l, diff_l, step_l, gap_l = [], [], [], []
        khz = float(native._lib.vk_wall_clock_khz())
        for _ in range(3):
            replay_s()
            barrier()
            s_ = stamps.cpu().numpy().reshape(per_graph, 3).astype(np.float64) / khz      # ms
            kin_l += list(s_[:, 1] - s_[:, 0])
            diff_l += list(s_[:, 2] - s_[:, 1])
            step_l += list(np.diff(s_[:, 0]))
            gap_l += list(s_[1:, 0] - s_[:-1, 2])          # two adjacent stamps, nothing between
        # each segment spans one stamp-to-stamp launch boundary more than its kernels:
        # the interval between two adjacent stamps (end of step k -> start of step k+1)
        gap = float(np.median(gap_l)) if gap_l else 0.0
        kin_ms, diff_ms = float(np.median(kin_l)) - gap, float(np.median(diff_l)) - gap
        graph_info['kernel_split_from'] = (
            'median over %d graph-replayed steps with device timestamps before the kinetics, after it and at the '
            'end of each step (vk_timestamp, %g kHz clock), less the stamp-to-stamp interval of two adjacent '
            'stamps (%.4f ms); the stamped step (three stamps) %.4f ms' % (3 * per_graph, khz, gap,
                                                                            float(np.median(step_l))))
        graph_info['stamped_step_ms'] = float(np.median(step_l)) if step_l else None
        graph_info['stamp_gap_ms'] = gap
    else:
        # Eager multi-GPU / dividing steps: HIP events around the kinetics launch and
        # the diffusion passes of eager steps after the timed region.  A lattice step
        # is ~10x longer on the GPU than its issue from Python, so from the second
        # step on the host runs ahead and the events bracket kernel time only (the
        # first step still waits for its issue: dropped).
        marks = [mk() for _ in range(SPLIT_STEPS)]
        barrier()
        for t_k in marks:
            one_step(t_k)
        barrier()
        kin_ms = float(np.median([t['kin'][0].elapsed_time(t['kin'][1]) for t in marks[1:]]))
        diff_ms = float(np.median([t['diff'][0].elapsed_time(t['diff'][1]) for t in marks[1:]]))
        if graph_info is not None:
            graph_info['kernel_split_from'] = ('median of %d eager steps after the timed region (HIP events; the '
                                               'host issues ahead of the GPU after the first)' % (SPLIT_STEPS - 1))
    if dist is not None:
        if args.dist_backend == 'gloo':
            el, n_agents = el.cpu(), n_agents.cpu()
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(n_agents, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    total_agent_steps = float(n_agents.item())
    value = total_agent_steps / elapsed

    if rank == 0:
        n_total, nx, bound, desc = WORKLOADS[args.workload]
        integ_flops = attempts * col.engine.dopri5_flops_per_attempt() / args.steps  # per step, rank 0
        variant = col.engine.default_variant()
        kname_i = {0: 'k_dopri5_thread', 1: 'k_dopri5_wave', 2: 'vk_dopri5_spec', 3: 'vk_dopri5_wspec'}[variant]
        # the kinetics launch also gathers the next step's local environment (Colony.fuse_gather)
        gathered = lat is not None and col._gather_fused() and not getattr(col, 'fuse_coupling', False)
        if gathered:
            kname_i = 'vk_dopri5_spec_gather'
        integ = {'kernel': kname_i, 'avg_ms_per_step': kin_ms,
                 'dp45_attempts_per_agent_step': attempts / agent_steps,
                 # integrator steps (accepted + rejected) and RHS evaluations
                 # per second over the timed region (rank 0; DP45 with FSAL: 6 new RHS per attempt)
                 'dp45_attempts_per_s': attempts / elapsed if elapsed else None,
                 'rhs_evals_per_s': 6.0 * attempts / elapsed if elapsed else None,
                 'dp45_attempts_per_agent_step_by_step': per_step, 'attempts_from': attempts_from,
                 'flops_per_attempt': col.engine.dopri5_flops_per_attempt(),
                 'achieved_tflops': integ_flops / (kin_ms * 1e-3) / 1e12 if kin_ms else None,
                 'peak_tflops': FP64_PEAK_TFLOPS}
        if integ['achieved_tflops'] is not None:
            integ['frac'] = integ['achieved_tflops'] / FP64_PEAK_TFLOPS
            # the agent state is streamed once per step: at a few flops per byte
            # (small networks) the launch is HBM-bound, not FP64-bound
            bpa = col.engine.dopri5_bytes_per_agent_step()
            if gathered:   # + per gathered field: its value at the agent's bin read, the external row written
                bpa += 16 * int(col.map_gather_field.numel())
            gbps = (agent_steps / args.steps) * bpa / (kin_ms * 1e-3) / 1e9
            t_flop = integ_flops / (FP64_PEAK_TFLOPS * 1e12)
            t_byte = (agent_steps / args.steps) * bpa / (HBM_PEAK_GBPS * 1e9)
            integ.update({'bytes_per_agent_step': bpa, 'achieved_gbps': gbps,
                          'roofline_bound': 'fp64' if t_flop >= t_byte else 'hbm',
                          'roofline_frac': max(t_flop, t_byte) / (kin_ms * 1e-3)})
        roofline = None
        if lat is not None:
            # dominant kernel: one fused pass of `depth` substeps (k_diffuse_wt<depth>)
            depth = args.stencil_depth
            cells = (lat.row_hi - lat.row_lo) * lat.ny * len(lat.molecules)
            launch_ms = stencil_pass_ms
            bytes_per_launch = 16.0 * cells          # algorithmic: read + write each cell once
            achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
            traffic = valu = traffic_from = None
            kname = stencil_kernel_name(args.stencil_kernel, depth, args.stencil_mode, bytes_per_launch)
            import glob
            for pmc in sorted(glob.glob(os.path.join(REPO, 'profiles', 'pmc_stencil*.json'))) if world == 1 else []:
                with open(pmc) as f:
                    rec = json.load(f)
                # the committed PMC pass must describe this exact launch geometry and mode, and
                # name the kernel this run launches (rocprof's full template name): a record
                # of an older kernel build is refused
                if (rec.get('depth'), rec.get('rows'), rec.get('cells'), rec.get('variant'),
                        rec.get('mode', 'exact'), rec.get('kernel')) == (depth, args.stencil_rows, cells,
                                                                         args.stencil_kernel, args.stencil_mode,
                                                                         kname):
                    traffic_from = os.path.relpath(pmc, REPO) + (' (commit %s)' % rec['commit']
                                                                 if rec.get('commit') else '')
                    traffic = rec.get('hbm_bytes_per_launch')
                    if rec.get('valu_insts_per_launch') and rec.get('clock_ghz'):
                        # the pass against the VALU-issue bound: one wave64 VALU instruction
                        # per 4 cycles per SIMD (1024 SIMDs) at the counter-measured clock,
                        # for the counted instructions, over this run's launch time
                        issue_s = rec['valu_insts_per_launch'] * 4.0 / (N_SIMDS * rec['clock_ghz'] * 1e9)
                        valu = {'insts_per_launch': rec['valu_insts_per_launch'], 'clock_ghz': rec['clock_ghz'],
                                'issue_bound_ms': issue_s * 1e3, 'frac': issue_s / (launch_ms * 1e-3),
                                'busy_counter': rec.get('valu_busy_per_simd')}
            roofline = {'bound': 'hbm', 'kernel': kname, 'achieved': achieved,
                        'peak': HBM_PEAK_GBPS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBPS,
                        'traffic': traffic, 'traffic_from': traffic_from, 'bytes_per_launch': bytes_per_launch,
                        'avg_launch_ms': launch_ms, 'substeps_per_launch': depth,
                        'effective_stencil_gbps': bytes_per_launch * depth / (launch_ms * 1e-3) / 1e9,
                        'fp64_tflops': 6.0 * cells * depth / (launch_ms * 1e-3) / 1e12,
                        'fp64_frac': 6.0 * cells * depth / (launch_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                        'valu_issue': valu, 'step_diffusion_ms': diff_ms, 'stencil_mode': args.stencil_mode,
                        'exact_mode_avg_launch_ms': exact_pass_ms,
                        'exact_mode_frac': (bytes_per_launch / (exact_pass_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
                                            if exact_pass_ms else None)}
            if copy_floor is not None:
                # the pass against the HBM rate this box delivers to its fastest streaming copy
                # of the same planes (vk_copy_stream; 8 TB/s is the spec, the copy ~6.3)
                cms, cbytes = copy_floor
                floor_ms = cms * bytes_per_launch / cbytes
                roofline['copy_floor'] = {'copy_ms': cms, 'copy_gbps': cbytes / (cms * 1e-3) / 1e9,
                                          'floor_ms_per_launch': floor_ms, 'frac': floor_ms / launch_ms}
        else:
            roofline = {'bound': 'fp64-valu', 'kernel': kname_i,
                        'achieved': integ.get('achieved_tflops'), 'peak': FP64_PEAK_TFLOPS,
                        'unit': 'TFLOP/s', 'frac': integ.get('frac'), 'traffic': None}
        out = {
            'metric': METRIC, 'value': value, 'unit': 'agent-steps/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': elapsed / args.steps * 1e3,
            'untimed_settle_steps': settle_steps,
            'higher_is_better': True, 'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic (seeded heterogeneous colony, SURVEY.md §8d distributions)',
            'config': {'workload': desc, 'agents': n_total, 'lattice': [nx, nx] if nx else None,
                       'agents_end': col.n if world == 1 else None, 'agents_start': n_start if world == 1 else None,
                       'fields': lat.molecules if lat is not None else None, 'dt_s': 1.0,
                       'substeps_per_step': n_substeps(1.0) if nx else 0,
                       'integrator': args.integrator, 'rtol': col.rtol, 'atol': col.atol,
                       'exchange': args.exchange, 'parallelism': 'row-bands x%d' % world,
                       'agents_in_bin_order': bool(nx and args.sort_agents),
                       'coupled_passes': bool(args.couple and getattr(col, '_couple', None) is not None),
                       'stencil_mode': args.stencil_mode if nx else None,
                       'halo': (col.lattice.halo if col.lattice is not None else 0) if world > 1 else 0},
            'roofline': roofline,
            'integrator': integ,
            'hip_graph': graph_info,
        }
        if world == 1 and not args.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline(args, col, host_state)
            # leg (ii): the reference's own odeint on the restated RHS, sampled agents
            params, conc, _ = host_state
            t = col.table
            cores = out['cpu_baseline']['cores']
            stride = max(1, conc.shape[1] // 256)
            jobs = [('convenience', (col.config, t.param_names, params[:, a].tolist(),
                                     {k: float(conc[s_, a]) for s_, k in enumerate(t.species)},
                                     float(col.m2c[a])))
                    for a in range(0, conc.shape[1], stride)][:256]
            out['cpu_baseline_odeint'] = cpu_baseline_odeint(jobs, min(8.0, args.cpu_seconds), cores)
        return out
    return None


def secondary_legs(args, dev):
    """Bounded C5 and Kremling legs on this GPU (1M agents each, --secondary-steps
    timed steps after 3 warmup steps, no CPU baselines): the integrator's FP64
    roofline, which the C4 headline (1.0 DP45 attempt per agent-step, 4 % of its
    step) does not exercise.  Reported under 'secondary' of the headline's line."""
    legs, t_all = {}, time.perf_counter()
    for wl in ('c5', 'kremling'):
        t0 = time.perf_counter()
        sub = argparse.Namespace(**vars(args))
        sub.workload, sub.steps, sub.warmup, sub.no_cpu_baseline = wl, args.secondary_steps, 3, True
        sub.stencil_mode, sub.stencil_depth, sub.stencil_kernel, sub.stencil_rows = 'fma', None, None, None
        sub.agents, sub.couple, sub.graph = None, False, 'auto'
        try:
            o = run_kremling(sub, 0, 1, dev, None) if wl == 'kremling' else run(sub, 0, 1, dev, None)
        except Exception as e:          # a failed leg must not cost the headline its line
            legs[wl] = {'error': '%s: %s' % (type(e).__name__, e), 'wall_s': time.perf_counter() - t0}
            torch.cuda.empty_cache()
            continue
        r = o['roofline']
        integ = o.get('integrator') or {}
        legs[wl] = {
            'workload': o['config']['workload'], 'agents': o['config']['agents'], 'value': o['value'],
            'unit': o['unit'], 'ms_per_step': o['ms_per_step'], 'steps': sub.steps, 'warmup': sub.warmup,
            'kernel': r['kernel'],
            'kinetics_ms_per_step': r.get('avg_launch_ms', integ.get('avg_ms_per_step')),
            'dp45_attempts_per_agent_step': r.get('dp45_attempts_per_agent_step',
                                                  integ.get('dp45_attempts_per_agent_step')),
            'dp45_attempts_per_agent_step_by_step': integ.get('dp45_attempts_per_agent_step_by_step'),
            'flops_per_attempt': r.get('flops_per_attempt', integ.get('flops_per_attempt')),
            'achieved_tflops': r['achieved'], 'peak_tflops': r['peak'], 'frac': r['frac'],
            'wall_s': time.perf_counter() - t0}
        torch.cuda.empty_cache()
    legs['wall_s'] = time.perf_counter() - t_all
    return legs


if __name__ == '__main__':
    main()

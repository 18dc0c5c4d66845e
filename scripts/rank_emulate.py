"""Per-rank cost of strong-scaled C4 diffusion on ONE GPU: a middle rank's row band
(4096/N rows + halo rows both sides), 100 substeps per step in blocks of `halo`
substeps, each block preceded by a local stand-in for the halo exchange (the
same 4 row-copies per field the real exchange does; no RCCL).  The whole plane is
timed live in the same process with the settings the one-GPU bench uses (34-row
tiles, variant 20, depth 10, tolerance mode), and each band is reported against
1/N of it.  Prints ms per step.

    python scripts/rank_emulate.py N halo rows [variant depth [mode]]     (mode: exact | fma)
    python scripts/rank_emulate.py N --sweep halo:rows:variant:depth,...  (tolerance mode)

XFER_US (env, default 0): the stand-in exchange also holds its stream for that
long (torch.cuda._sleep, calibrated), standing in for the RCCL transfer over xGMI
(~6.5 MB per neighbour and step at h = 100: ~100 us at ~65 GB/s).  Each band
case is then timed twice: the exchange before the block on the launch stream
(serial), and on a side stream beside the block's interior passes, the edge
passes after it (overlap, Lattice.diffuse(halo_event=...)).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from lens_amd import configs  # noqa: E402
from lens_amd.distributed import row_bands  # noqa: E402
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel, stencil_mode  # noqa: E402

dev = torch.device('cuda', 0)
nx = 4096


def time_steps(fn, warm=20, reps=10):
    for _ in range(warm):   # past the power-management transient after setup (profiles/r02g_eager_trace_gaps.log)
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def whole_plane_ms(variant=20, depth=10, rows=34):
    glc0 = configs.gaussian_bump_field((nx, nx))
    whole = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (4096.0, 4096.0), 10.0, 5.0, device=dev,
                    initial={'glc__D_e': glc0, 'ac_e': glc0 * 0.5})
    stencil_kernel(variant, rows)
    stencil_depth(depth)
    ms = time_steps(lambda: whole.diffuse(1.0))
    del whole
    return ms


XFER_US = float(os.environ.get('XFER_US', '0'))
if os.environ.get('OVERLAP_PASSES'):       # passes whose interior runs beside the stand-in transfer
    Lattice.HALO_OVERLAP_PASSES = int(os.environ['OVERLAP_PASSES'])
_CYCLES_PER_US = None


def _sleep_us(us):
    """Hold the current stream for ~us microseconds (calibrated spin kernel)."""
    global _CYCLES_PER_US
    if us <= 0:
        return
    if _CYCLES_PER_US is None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1000000)
        e0.record()
        torch.cuda._sleep(10000000)
        e1.record()
        torch.cuda.synchronize()
        _CYCLES_PER_US = 10000000 / (e0.elapsed_time(e1) * 1e3)
    torch.cuda._sleep(int(us * _CYCLES_PER_US))


def band_ms(world, halo, rows, variant, depth, overlap=False):
    band = row_bands(nx, world)[1 if world > 2 else 0]
    glc = configs.gaussian_bump_field((nx, nx))
    lat = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (4096.0, 4096.0), 10.0, 5.0, device=dev, row_band=band,
                  halo=halo, initial={'glc__D_e': glc, 'ac_e': glc * 0.5})
    stencil_kernel(variant, rows)
    stencil_depth(depth)
    h = lat.halo
    bufs = [torch.empty((2, h, nx), dtype=torch.float64, device=dev) for _ in range(4)]

    def fake_exchange(src, cnt):
        _sleep_us(XFER_US)
        if not lat.edge_top:
            bufs[0].copy_(src[:, lat.row_lo:lat.row_lo + h]); bufs[1].copy_(bufs[0])
            src[:, lat.row_lo - h:lat.row_lo].copy_(bufs[1])
        if not lat.edge_bot:
            bufs[2].copy_(src[:, lat.row_hi - h:lat.row_hi]); bufs[3].copy_(bufs[2])
            src[:, lat.row_hi:lat.row_hi + h].copy_(bufs[3])

    side = torch.cuda.Stream(device=dev)

    def one_step():
        if overlap:
            done = lat.exchange_first_halo(1.0, fake_exchange, side)
            lat.diffuse(1.0, halo_exchange=fake_exchange, allreduce=lambda mm: None, halo_event=done)
        else:
            lat.diffuse(1.0, halo_exchange=fake_exchange, allreduce=lambda mm: None)

    ms = time_steps(one_step)
    # the same step with its launch sequence replayed from one HIP graph (the stand-in
    # exchange included), as the bench replays a band's halo blocks: the GPU's time
    # without the host's issue of ~20 launches per step
    one_step()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        one_step()
    torch.cuda.current_stream(dev).wait_stream(s)
    g.replay()
    graph_ms = time_steps(g.replay)
    del lat
    return band, ms, graph_ms


def main():
    world = int(sys.argv[1])
    if len(sys.argv) > 2 and sys.argv[2] == '--sweep':
        stencil_mode('fma')
        whole = whole_plane_ms()
        print(json.dumps({'world': world, 'whole_plane_ms': round(whole, 4), 'ideal_ms': round(whole / world, 4)}),
              flush=True)
        for v in os.environ.get('WHOLE_VARIANTS', '').split(','):   # A/B of the whole plane's kernel: variant[:rows]
            if v:
                v, r = (int(x) for x in (v + ':34').split(':')[:2])
                print(json.dumps({'world': 1, 'variant': v, 'rows': r, 'whole_plane_ms': round(whole_plane_ms(v, rows=r), 4)}),
                      flush=True)
        for spec in sys.argv[3].split(','):
            halo, rows, variant, depth = (int(x) for x in spec.split(':'))
            for overlap in ((False, True) if XFER_US > 0 else (False,)):
                band, ms, graph_ms = band_ms(world, halo, rows, variant, depth, overlap)
                print(json.dumps({'world': world, 'band': list(band), 'halo': halo, 'rows': rows, 'variant': variant,
                                  'depth': depth, 'xfer_us': XFER_US, 'overlap': overlap,
                                  'overlap_passes': Lattice.HALO_OVERLAP_PASSES,
                                  'ms_per_step': round(ms, 4), 'efficiency': round(whole / world / ms, 3),
                                  'graph_ms_per_step': round(graph_ms, 4),
                                  'graph_efficiency': round(whole / world / graph_ms, 3)}), flush=True)
        return
    halo, rows = int(sys.argv[2]), int(sys.argv[3])
    variant = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    depth = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    mode = sys.argv[6] if len(sys.argv) > 6 else 'fma'
    stencil_mode(mode)
    whole = whole_plane_ms()
    band, ms, graph_ms = band_ms(world, halo, rows, variant, depth)
    print('N=%d band=%s halo=%d rows=%d variant=%d depth=%d mode=%s: %.3f ms/step (graph %.3f); whole plane %.3f ms '
          '(live), ideal %.3f = 1/N of it, diffusion efficiency %.2f (graph %.2f)'
          % (world, band, halo, rows, variant, depth, mode, ms, graph_ms, whole, whole / world, whole / world / ms,
             whole / world / graph_ms))


if __name__ == '__main__':
    main()

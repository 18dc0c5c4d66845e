"""Per-rank cost of strong-scaled C4 diffusion on ONE GPU: a middle rank's row band
(4096/N rows + halo rows both sides), 100 substeps per step in blocks of `halo`
substeps, each block preceded by a local stand-in for the halo exchange (the
same 4 row-copies per field the real exchange does; no RCCL).  Prints ms per step.

    python scripts/rank_emulate.py N halo rows [variant depth [mode]]     (mode: exact | fma)
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from lens_amd import configs
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel
from lens_amd.distributed import row_bands
world, halo, rows = (int(x) for x in sys.argv[1:4])
variant = int(sys.argv[4]) if len(sys.argv) > 4 else 3
depth = int(sys.argv[5]) if len(sys.argv) > 5 else 9
mode = sys.argv[6] if len(sys.argv) > 6 else 'exact'
from lens_amd.lattice import stencil_mode
stencil_mode(mode)
dev = torch.device('cuda', 0)
nx = 4096
band = row_bands(nx, world)[1 if world > 2 else 0]
glc = configs.gaussian_bump_field((nx, nx))
lat = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (4096.0, 4096.0), 10.0, 5.0, device=dev, row_band=band,
              halo=halo, initial={'glc__D_e': glc, 'ac_e': glc * 0.5})
stencil_kernel(variant, rows)
stencil_depth(depth)
h = lat.halo
bufs = [torch.empty((2, h, nx), dtype=torch.float64, device=dev) for _ in range(4)]

def fake_exchange(src, cnt):
    if not lat.edge_top:
        bufs[0].copy_(src[:, lat.row_lo:lat.row_lo + h]); bufs[1].copy_(bufs[0])
        src[:, lat.row_lo - h:lat.row_lo].copy_(bufs[1])
    if not lat.edge_bot:
        bufs[2].copy_(src[:, lat.row_hi - h:lat.row_hi]); bufs[3].copy_(bufs[2])
        src[:, lat.row_hi:lat.row_hi + h].copy_(bufs[3])

for _ in range(20):   # past the power-management transient after setup (profiles/r02g_eager_trace_gaps.log)
    lat.diffuse(1.0, halo_exchange=fake_exchange, allreduce=lambda mm: None)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    lat.diffuse(1.0, halo_exchange=fake_exchange, allreduce=lambda mm: None)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / 10 * 1e3
print('N=%d band=%s halo=%d rows=%d variant=%d depth=%d mode=%s: %.3f ms/step (ideal %.3f = 1/N of the whole)' % (
    world, band, halo, rows, variant, depth, mode, ms, 1.95 / world))

"""Halo depth / tile rows / pass depth sweep for strong-scaled C4 diffusion on ONE GPU.

Emulates one middle rank's row band (4096/N rows + halo rows on both sides)
like scripts/rank_emulate.py -- 100 substeps per step in blocks of `halo`
substeps, each block preceded by a local stand-in for the halo exchange (the
same row copies the real exchange does, no RCCL) -- for every combination in
the grid, in one process, interleaved over rounds.  Prints one JSON line per
configuration with the median ms per step.

    python scripts/halo_sweep.py N [halo,...] [rows,...] [depth,...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lens_amd import configs  # noqa: E402
from lens_amd.distributed import row_bands  # noqa: E402
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel  # noqa: E402

world = int(sys.argv[1])
halos = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else '9,18,27,36,50,100').split(',')]
rows_l = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else '0,16,32,64').split(',')]
depths = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else '5,7,9').split(',')]
dev = torch.device('cuda', 0)
nx = 4096
band = row_bands(nx, world)[1 if world > 2 else 0]
glc = configs.gaussian_bump_field((nx, nx))
lats = {}
for halo in halos:
    lat = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (4096.0, 4096.0), 10.0, 5.0, device=dev, row_band=band,
                  halo=halo, initial={'glc__D_e': glc, 'ac_e': glc * 0.5})
    h = lat.halo
    bufs = [torch.empty((2, h, nx), dtype=torch.float64, device=dev) for _ in range(4)]

    def fake_exchange(src, cnt, lat=lat, h=h, bufs=bufs):
        if not lat.edge_top:
            bufs[0].copy_(src[:, lat.row_lo:lat.row_lo + h]); bufs[1].copy_(bufs[0])
            src[:, lat.row_lo - h:lat.row_lo].copy_(bufs[1])
        if not lat.edge_bot:
            bufs[2].copy_(src[:, lat.row_hi - h:lat.row_hi]); bufs[3].copy_(bufs[2])
            src[:, lat.row_hi:lat.row_hi + h].copy_(bufs[3])
    lats[halo] = (lat, fake_exchange)

cases = [(h, r, d) for h in halos for r in rows_l for d in depths]
res = {c: [] for c in cases}
stencil_kernel(6, 0)
for rnd in range(3):
    for c in cases:
        halo, rows, depth = c
        lat, ex = lats[halo]
        stencil_kernel(-1, rows)
        stencil_depth(depth)
        lat.diffuse(1.0, halo_exchange=ex, allreduce=lambda mm: None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(3):
            lat.diffuse(1.0, halo_exchange=ex, allreduce=lambda mm: None)
        e1.record()
        torch.cuda.synchronize()
        res[c].append(e0.elapsed_time(e1) / 3)
for c in cases:
    print(json.dumps({'world': world, 'band_rows': band[1] - band[0], 'halo': c[0], 'rows': c[1], 'depth': c[2],
                      'ms_per_step': round(float(np.median(res[c])), 4)}), flush=True)

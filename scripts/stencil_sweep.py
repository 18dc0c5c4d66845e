"""A/B sweep of the stencil kernel variant / depth / rows-per-tile (interleaved rounds, one process).

    python scripts/stencil_sweep.py [n] [variant:depth:rows[:mode],...]     (mode 0 = exact, 1 = fma)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lens_amd import configs  # noqa: E402
from lens_amd import native  # noqa: E402
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
spec = sys.argv[2] if len(sys.argv) > 2 else '0:11:128,1:7:128,1:9:128,1:11:128,1:13:128,1:15:128,1:9:64,1:11:256'
cases = [tuple(int(x) for x in (c + ':0').split(':')[:4]) for c in spec.split(',')]
dev = torch.device('cuda', 0)
glc = configs.gaussian_bump_field((n, n))
lat = Lattice(['glc__D_e', 'ac_e'], (n, n), (float(n), float(n)), 10.0, 5.0, device=dev,
              initial={'glc__D_e': glc, 'ac_e': glc * 0.5})
res = {c: [] for c in cases}
for rnd in range(4):
    for c in cases:
        v, d, rows, mode = c
        native._lib.vk_set_stencil_mode(mode)
        stencil_kernel(v, rows)
        stencil_depth(d)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        lat.diffuse(1.0)
        torch.cuda.synchronize()
        lat.diffuse(1.0, events=(e0, e1))
        torch.cuda.synchronize()
        res[c].append(e0.elapsed_time(e1))
cells = 2 * n * n
for c in cases:
    ms = float(np.median(res[c]))
    print(json.dumps({'variant': c[0], 'depth': c[1], 'rows': c[2], 'mode': c[3], 'ms_per_100_substeps': round(ms, 4),
                      'effective_GBps': round(16 * cells * 100 / (ms * 1e-3) / 1e9)}))

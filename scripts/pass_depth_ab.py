"""One fused tolerance-mode pass of D substeps on the C4 planes (4096^2 x 2,
34-row tiles, variant 20): per-pass and per-substep time for D = 10 / 12,
interleaved rounds (bench.time_stencil_pass: HIP events around 20 launches).
Ran against an experimental build with a 12-deep block plan (reverted after
this A/B: profiles/r04/r04aj/); on the current build depth 12 is not offered.

    python scripts/pass_depth_ab.py [rounds]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lens_amd import configs  # noqa: E402
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel, stencil_mode  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device('cuda', 0)
    glc = configs.gaussian_bump_field((4096, 4096))
    lat = Lattice(['glc__D_e', 'ac_e'], (4096, 4096), (4096.0, 4096.0), 10.0, 5.0, device=dev,
                  initial={'glc__D_e': glc, 'ac_e': glc * 0.5})
    stencil_mode('fma')
    stencil_kernel(20, 34)
    res = {10: [], 12: []}
    for _ in range(rounds):
        for d in (10, 12):
            stencil_depth(d)
            res[d].append(bench.time_stencil_pass(lat, d))
    for d, v in res.items():
        m = float(np.median(v))
        print(json.dumps({'depth': d, 'ms_per_pass': round(m, 4), 'us_per_substep': round(m * 1e3 / d, 2),
                          'all': [round(x, 4) for x in v]}), flush=True)


if __name__ == '__main__':
    main()

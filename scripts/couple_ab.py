"""A/B of how a graph-replayed C4 step is laid out on the bench's colony
(bench.build_rank, bin order, DP45, the bench's stencil settings): sequential
launches, the overlapped capture (step k's exchange beside step k+1's kinetics,
the uniform probe beside the gather; Colony.capture(overlap=True)), and the coupled
passes (gather / exchange inside the first / final pass).  Interleaved rounds in
one process; prints ms per step.

    python scripts/couple_ab.py [rounds]
"""
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device('cuda', 0)
    args = bench.parse(['--workload', 'c4'])
    mode, depth, kernel, rows = bench.stencil_settings(args, 1)
    stencil_mode(mode)
    stencil_depth(depth)
    build = types.SimpleNamespace(workload='c4', integrator='dopri5', halo=0, exchange='sorted',
                                  generic_kernel=False, agents=None, overlap_kinetics=False, sort_agents=True)
    col, lat, _ = bench.build_rank(build, 0, 1, dev)
    configs = [('sequential', False, False), ('overlapped', False, True), ('coupled', True, False)]
    stencil_kernel(kernel, rows)
    graphs = {}
    for name, fused, overlap in configs:
        col.fuse_coupling = fused
        graphs[name] = col.capture(1.0, 10, overlap=overlap)
        graphs[name]()                     # upload + warm
    torch.cuda.synchronize()
    res = {name: [] for name, _, _ in configs}
    for _ in range(rounds):
        for name, _, _ in configs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graphs[name]()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 10)
    for name, _, _ in configs:
        print(json.dumps({'config': name, 'ms_per_step_median': round(float(np.median(res[name])), 4),
                          'ms_per_step_all': [round(x, 4) for x in res[name]]}), flush=True)


if __name__ == '__main__':
    main()

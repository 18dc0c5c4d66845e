"""Does recording HIP events around the kinetics and the diffusion of every
step (the bench's eager timing) cost time?  C4 on one GPU: 20 eager steps with
and without the per-step events, and 20 steps replayed from a graph.

    python scripts/event_cost.py
"""
import os
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from lens_amd.lattice import stencil_kernel  # noqa: E402

dev = torch.device('cuda', 0)
stencil_kernel(6, 64)
args = types.SimpleNamespace(workload='c4', halo=0, integrator='dopri5', exchange='sorted', generic_kernel=False,
                             agents=None, overlap_kinetics=False)
col, lat, _ = bench.build_rank(args, 0, 1, dev)
ev = lambda: torch.cuda.Event(enable_timing=True)


def run(k, timed):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        col.step(1.0, timing={'kin': (ev(), ev()), 'diff': (ev(), ev())} if timed else None)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


run(3, False)
replay = col.capture(1.0, 10)
replay()
for rnd in range(2):
    a = run(20, True)
    b = run(20, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    replay()
    replay()
    torch.cuda.synchronize()
    c = (time.perf_counter() - t0) / 20 * 1e3
    print('ms per step: eager with per-step events %.3f, eager without %.3f, graph %.3f' % (a, b, c), flush=True)

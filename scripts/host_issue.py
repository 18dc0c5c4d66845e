"""Host issue time of one colony step: a lattice colony so small that its GPU
work is negligible, stepped eagerly; ms per step = what Python + the C ABI
cost per step (the floor of an eager multi-GPU step, whose ranks cannot use
graph replay).  Also the same colony replayed from a graph.

    python scripts/host_issue.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lens_amd import configs  # noqa: E402
from lens_amd.colony import Colony  # noqa: E402
from lens_amd.lattice import Lattice  # noqa: E402
from lens_amd.rate_law_compiler import compile_rate_laws  # noqa: E402

dev = torch.device('cuda', 0)
cfg = configs.glc_ac_config()
t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
nx, n = 64, 256
lat = Lattice(['glc__D_e', 'ac_e'], (nx, nx), (float(nx), float(nx)), 10.0, 5.0, device=dev,
              initial={'glc__D_e': configs.gaussian_bump_field((nx, nx)), 'ac_e': np.zeros((nx, nx))})
params, conc = configs.heterogeneous_colony(t, cfg, n)
col = Colony(cfg, n, device=dev, integrator='dopri5', environment=lat, table=t, specialize=True)
col.set_agents(params=params, conc=conc, location=np.random.default_rng(1).uniform(0, nx, (2, n)))
for _ in range(5):
    col.step(1.0)
torch.cuda.synchronize()
steps = 200
t0 = time.perf_counter()
for _ in range(steps):
    col.step(1.0)
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
replay = col.capture(1.0, 10)
replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps // 10):
    replay()
torch.cuda.synchronize()
t_graph = time.perf_counter() - t0
print('eager: %.1f us per step issued, %.1f us per step to completion; graph: %.1f us per step'
      % (t_issue / steps * 1e6, t_all / steps * 1e6, t_graph / steps * 1e6))

"""Time the C4 colony's DP45 kinetics launch and its lane efficiency (profiling driver).

    python scripts/dp45_probe.py [steps]

lane efficiency = attempts summed over agents / (64 x the slowest lane of each
wavefront, summed over wavefronts): the fraction of issued lane-attempts that
do useful work under wave divergence.  VK_DOPRI5_TEMPLATE selects another
specialised-kernel template (A/B runs)."""
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device('cuda', 0)
args = types.SimpleNamespace(workload=os.environ.get('WORKLOAD', 'c4'), halo=0, integrator='dopri5',
                             exchange='sorted', generic_kernel=False, agents=None, overlap_kinetics=False)
col, lat, _ = bench.build_rank(args, 0, 1, dev)
ev = lambda: torch.cuda.Event(enable_timing=True)
kin, eff, att = [], [], []
for k in range(steps + 2):
    t = {'kin': (ev(), ev()), 'diff': (ev(), ev())}
    col.step(1.0, timing=t)
    torch.cuda.synchronize()
    if k >= 2:
        kin.append(t['kin'][0].elapsed_time(t['kin'][1]))
        ns = col.nsteps[:col.n].to(torch.float64)
        m = (col.n // 64) * 64
        w = ns[:m].view(-1, 64)
        eff.append(float(w.sum() / (64.0 * w.max(dim=1).values.sum())))
        att.append(float(ns.mean()))
fl = col.engine.dopri5_flops_per_attempt()
ms = sorted(kin)[len(kin) // 2]
print(json.dumps({'template': os.environ.get('VK_DOPRI5_TEMPLATE', 'default'), 'agents': col.n,
                  'kin_ms_median': ms, 'attempts_per_agent': sum(att) / len(att),
                  'lane_efficiency': sum(eff) / len(eff), 'flops_per_attempt': fl,
                  'tflops': col.n * (sum(att) / len(att)) * fl / (ms * 1e-3) / 1e12}))

"""Lane efficiency of the Kremling kernel (one agent per lane, the wave runs until
its slowest lane lands): DP45 attempts per agent-step, the mean over 64-agent
waves of (mean attempts / max attempts), and the same with the agents ordered by
their previous step's attempts.  Times a step in both layouts.

    python scripts/kremling_probe.py [n_agents]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def wave_eff(ns):
    w = ns[:len(ns) // 64 * 64].reshape(-1, 64).astype(np.float64)
    return float(w.mean() / w.max(axis=1).mean())


def timed(col, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(reps):
        e0.record()
        col.step(1.0)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return float(np.median(out))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    dev = torch.device('cuda', 0)
    col, states, vols = bench.kremling_colony(n, dev, 7)
    col.step(1.0)
    torch.cuda.synchronize()
    ns = col.nsteps[:n].cpu().numpy()
    ms = timed(col)
    ns2 = col.nsteps[:n].cpu().numpy()
    order = np.argsort(ns2, kind='stable')
    col2, _, _ = bench.kremling_colony(n, dev, 7)
    st = col2.state[:, :n].cpu().numpy()
    col2.set_state(st[:, order])
    col2.volume[:n].copy_(col2.volume[:n][torch.from_numpy(order).to(dev)])
    col2.step(1.0)
    ms_sorted = timed(col2)
    ns3 = col2.nsteps[:n].cpu().numpy()
    print(json.dumps({'agents': n, 'attempts_mean': float(ns2.mean()), 'attempts_p10_p50_p90':
                      [float(x) for x in np.percentile(ns2, [10, 50, 90])],
                      'wave_efficiency': round(wave_eff(ns2), 3), 'ms_per_step': round(ms, 3),
                      'sorted_wave_efficiency': round(wave_eff(ns3), 3), 'sorted_ms_per_step': round(ms_sorted, 3)}))


if __name__ == '__main__':
    main()

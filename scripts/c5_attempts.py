"""Distribution of DP45 attempts per agent in the C5 colony (bench.build_rank's
'c5' workload, one GPU): percentiles after each of a few steps, and the share of
the kinetics launch's work in its slowest agents (how long a tail the launch's
last wave round can have)."""
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    args = types.SimpleNamespace(workload='c5', integrator='dopri5', halo=0, exchange='sorted', generic_kernel=False,
                                 agents=None, overlap_kinetics=False, sort_agents=False)
    col, _, _ = bench.build_rank(args, 0, 1, dev)
    for step in range(3):
        col.step(1.0)
        torch.cuda.synchronize()
        ns = col.nsteps[:col.n].cpu().numpy().astype(np.int64)
        q = np.percentile(ns, [0, 50, 90, 99, 99.9, 100])
        print('step %d: agents %d mean %.1f  p0/p50/p90/p99/p99.9/max %s' % (step, col.n, ns.mean(), q.tolist()),
              flush=True)
        last = ns[-3072:]                                  # the launch's last wave round, in dispatch order
        print('   last 3072 agents: mean %.1f max %d  (all: mean %.1f)' % (last.mean(), last.max(), ns.mean()),
              flush=True)


if __name__ == '__main__':
    main()

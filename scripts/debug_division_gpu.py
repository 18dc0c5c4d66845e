"""Where do the batched loop and the oracle loop part ways on the dividing
colony of tests/test_engine_gpu.py?  Logs every GrowthProtein.next_update call
(timestep, protein, divide flag) and every MetaDivision division in both runs and
prints the first difference."""
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))

import test_engine_gpu as t                       # noqa: E402
from lens_amd import division                    # noqa: E402
from lens_amd.engine import Experiment           # noqa: E402
from lens_amd.invoke import BatchedInvoke        # noqa: E402
from oracle.experiment import OracleExperiment   # noqa: E402

LOG = []
_gp, _md = division.GrowthProtein.next_update, division.MetaDivision.next_update


def gp(self, timestep, states):
    u = _gp(self, timestep, states)
    LOG.append(('grow', float(timestep), float(states['internal']['protein']), u['global']['divide']))
    return u


def md(self, timestep, states):
    u = _md(self, timestep, states)
    if u:
        LOG.append(('divide', self.agent_id))
    return u


division.GrowthProtein.next_update, division.MetaDivision.next_update = gp, md


def run(batched, intervals):
    LOG.clear()
    dev = torch.device('cuda', 0)
    np.random.seed(21)
    random.seed(21)
    p, tp, init = t._dividing_colony(batched, dev)
    exp = (Experiment({'processes': p, 'topology': tp, 'initial_state': init, 'invoke': BatchedInvoke(dev)})
           if batched else OracleExperiment(p, tp, init))
    marks = []
    for iv in intervals:
        exp.update(iv)
        marks.append(len(LOG))
        LOG.append(('interval', iv, list(exp.state['agents'])))
    return list(LOG), marks


intervals = (1.0, 3.0, 0.5, 4.5, 2.0, 5.0)
g, gm = run(True, intervals)
r, rm = run(False, intervals)
print('calls', len(g), len(r))
for i, (a, b) in enumerate(zip(g, r)):
    if a != b:
        print('first difference at', i)
        for k in range(max(0, i - 6), min(len(g), len(r), i + 6)):
            print(k, 'GPU', g[k][:3] if g[k][0] == 'interval' else g[k])
            print(k, 'REF', r[k][:3] if r[k][0] == 'interval' else r[k])
        break
else:
    print('no difference in the common prefix')

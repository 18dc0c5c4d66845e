"""Two Kremling steps (1 s each) on N agents (default 100k) -- profiling driver for PMC passes."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device('cuda', 0)
col, _, _ = bench.kremling_colony(int(os.environ.get('N', '100000')), dev, 7)
for _ in range(2):
    col.step(1.0)
torch.cuda.synchronize()
print('done')

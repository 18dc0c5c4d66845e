"""C4 colony steps for PMC passes on the kinetics launch (profiling driver): the
bench's own colony (bench.build_rank, 1M agents in bin order, 4096^2 x 2), three
steps with the gather fused into the DP45 launch (vk_dopri5_spec_gather), then
three with the separate launches (vk_dopri5_spec + k_gather), so one pass of
counters shows the fused launch's traffic beside its two parts."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402

args = bench.parse(['--no-cpu-baseline'])
args.stencil_mode, args.stencil_depth, args.stencil_kernel, args.stencil_rows = bench.stencil_settings(args, 1)
from lens_amd.lattice import stencil_depth, stencil_kernel, stencil_mode  # noqa: E402
stencil_depth(args.stencil_depth)
stencil_mode(args.stencil_mode)
stencil_kernel(args.stencil_kernel, args.stencil_rows)
dev = torch.device('cuda', 0)
col, lat, _ = bench.build_rank(args, 0, 1, dev)
for fused in (True, False):
    col.fuse_gather = fused
    for _ in range(3):
        col.step(1.0)
torch.cuda.synchronize()
print('done')

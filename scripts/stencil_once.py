"""Run the 4096^2 x 2-field diffusion (100 substeps) a few times at one depth (profiling driver).
Defaults: the C4 bench pass (bench.stencil_settings at N = 1: depth 10, fma, variant 70, 64 rows)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from lens_amd import configs
from lens_amd.lattice import Lattice, stencil_depth
n = int(os.environ.get('N', '4096')); depth = int(os.environ.get('DEPTH', '10')); reps = int(os.environ.get('REPS', '3'))
dev = torch.device('cuda', 0)
glc = configs.gaussian_bump_field((n, n))
lat = Lattice(['glc__D_e', 'ac_e'], (n, n), (float(n), float(n)), 10.0, 5.0, device=dev,
              initial={'glc__D_e': glc, 'ac_e': glc * 0.5})
stencil_depth(depth)
from lens_amd.lattice import stencil_kernel
stencil_kernel(int(os.environ.get('VARIANT', '70')), int(os.environ.get('ROWS', '64')))
from lens_amd.lattice import stencil_mode
stencil_mode(os.environ.get('MODE', 'fma'))
for _ in range(reps):
    lat.diffuse(1.0)
torch.cuda.synchronize()
print('done depth', depth)

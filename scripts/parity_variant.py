import numpy as np, torch, sys
sys.path.insert(0, '.')
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel, stencil_mode
from oracle import cpu
dev = torch.device('cuda', 0)
def run(f0, v, rows=64):
    nx, ny = f0.shape
    pm, pd, pk = stencil_mode('fma'), stencil_depth(10), stencil_kernel(v, rows)
    lat = Lattice(['a'], (nx, ny), (float(nx), float(ny)), 10.0, 5.0, device=dev, initial={'a': f0})
    lat.diffuse(1.0); torch.cuda.synchronize()
    stencil_mode(pm); stencil_depth(pd); stencil_kernel(pk, 0)
    return lat.owned('a').cpu().numpy()
rng = np.random.default_rng(5)
for shape in [(640, 1000), (333, 517), (4096, 4096), (300, 96), (200, 97)]:
    f0 = rng.random(shape) + 0.5
    a, b = run(f0, int(sys.argv[1]) if len(sys.argv) > 1 else 70), run(f0, 20)
    ok = np.array_equal(a, b)
    ref = np.ascontiguousarray(f0.copy()); cpu.diffuse(ref, 0.05, 100) if shape[0] < 1000 else None
    rel = float(np.abs(a - ref).max() / np.abs(ref).max()) if shape[0] < 1000 else 0.0
    print(shape, 'bitwise==v20', ok, 'rel vs oracle', rel)
    assert ok and rel < 1e-13
print("parity ok")

#!/bin/bash
# (Record of a reverted experiment: the VK_ZONES hook is no longer built; DESIGN §10, profiles/r06/zones.)
# Zoned chunk heights (VK_ZONES="rows2,pct": the last pct % of rows in rows2-row tiles,
# dispatched last) against one zone: bitwise check, wave stamps, bench arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-zones}; mkdir -p $O
export TMPDIR=/tmp
VK_ZONES=32,25 timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.')
import numpy as np, torch
from lens_amd import native
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel, stencil_mode
dev = torch.device('cuda', 0)
native.load()
rng = np.random.default_rng(3)
for shape in [(4096, 4096), (1000, 1300), (700, 1000)]:
    f0 = rng.random(shape) + 0.5
    out = []
    for z in ((0, 0), (32, 25), (16, 30)):
        native._lib.vk_set_stencil_zones(*z)
        stencil_mode('fma'); stencil_depth(10); stencil_kernel(70, 64)
        lat = Lattice(['a', 'b'], shape, (float(shape[0]), float(shape[1])), 10.0, 5.0, device=dev, initial={'a': f0, 'b': f0 * 0.5})
        lat.diffuse(1.0); torch.cuda.synchronize()
        out.append((lat.owned('a').cpu().numpy(), lat.owned('b').cpu().numpy()))
    for o in out[1:]:
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1]), shape
    print(shape, 'zoned bitwise ok')
" > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -3 $O/parity.log
for z in ${ZSTAMPS:-32,25 32,15 16,10}; do
  VK_ZONES=$z OUT=$O/st_$z.npy timeout -k 10 120 python scripts/ps_wave_stamps.py > $O/st_$z.log 2>&1 || { tail -5 $O/st_$z.log; exit 2; }
  echo "zones $z: $(grep span_us $O/st_$z.log | cut -c1-200)"
done
IFS=' ' read -ra ZS <<< "${ZARMS:-32,25 32,15 16,10}"
ARMS="z0:"
for z in "${ZS[@]}"; do ARMS="$ARMS|z$z:"; done
for r in 1 2; do
  for z in 0,0 "${ZS[@]}"; do
    VK_ZONES=$z timeout -k 10 200 python bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 > $O/b_${z}_$r.json 2> $O/b_${z}_$r.err || { echo "arm $z failed"; tail -5 $O/b_${z}_$r.err; exit 3; }
    python -c "import json; d=json.loads(open('$O/b_${z}_$r.json').read().strip().splitlines()[-1]); print('zones $z round $r: %.4f ms/step  pass %.1f us frac %.3f' % (d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac']))"
  done
done

"""Diagnostic (needs a build with VK_PS_STAMPS): per-wave start/end times of the C4
pass (4096^2 x 2, depth 10, variant 70, 64-row tiles), slot occupancy over time.

The instrumentation was a temporary patch, reverted after the measurement: the
kernel read s_memrealtime at its start and end, and lane 0 stored {start, end,
HW_ID, XCC_ID} with vector stores into a device buffer set by vk_ps_set_stamps
(profiles/r06/stamps)."""
import os, sys, ctypes, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from lens_amd import configs, native
from lens_amd.lattice import Lattice, stencil_depth, stencil_kernel, stencil_mode
dev = torch.device('cuda', 0)
n = 4096
rows = int(os.environ.get('ROWS', '64'))
glc = configs.gaussian_bump_field((n, n))
lat = Lattice(['glc__D_e', 'ac_e'], (n, n), (float(n), float(n)), 10.0, 5.0, device=dev,
              initial={'glc__D_e': glc, 'ac_e': glc * 0.5})
native.load()
stencil_depth(10); stencil_kernel(int(os.environ.get('VARIANT', '70')), rows); stencil_mode('fma')
if os.environ.get('VK_ZONES'):
    native._lib.vk_set_stencil_zones(*(int(x) for x in os.environ['VK_ZONES'].split(',')))
for _ in range(5):
    lat.diffuse(1.0)
torch.cuda.synchronize()
tiles_x = (n + 95) // 96
waves = tiles_x * ((n + 8 - 1) // 8) * 2   # upper bound
st = torch.zeros((waves, 4), dtype=torch.int64, device=dev)
lib = native._lib
lib.vk_ps_set_stamps.argtypes = [ctypes.c_void_p]
assert lib.vk_ps_set_stamps(st.data_ptr()) == 0
lat.diffuse(1.0)
torch.cuda.synchronize()
lib.vk_ps_set_stamps(None)
a = st.cpu().numpy()
a = a[a[:, 1] != 0]
waves = len(a)
t0 = a[:, 0] - a[:, 0].min()
t1 = a[:, 1] - a[:, 0].min()
dur = (t1 - t0) * 0.01   # 100 MHz -> us
span = t1.max() * 0.01
print(json.dumps({'waves': waves, 'span_us': float(span), 'dur_mean': float(dur.mean()), 'dur_p10': float(np.percentile(dur, 10)),
                  'dur_p50': float(np.median(dur)), 'dur_p90': float(np.percentile(dur, 90)), 'dur_max': float(dur.max()),
                  'occupancy': float(dur.sum() / (3072 * span))}))
# occupancy timeline (resident waves per 2-us bucket)
edges = np.arange(0, span + 2, 2.0)
res = [int(((t0 * 0.01 <= e) & (t1 * 0.01 > e)).sum()) for e in edges]
print('resident per 2 us:', res)
starts = np.sort(t0 * 0.01)
print('start quantiles (us): 3072nd wave', float(starts[min(3071, waves - 1)]), 'last', float(starts[-1]))
# by tile kind: wave index order is edge tiles first
xcc = (a[:, 3] & 0xF)
for x in range(8):
    m = xcc == x
    if m.any():
        print('xcc', x, 'waves', int(m.sum()), 'dur mean %.1f' % dur[m].mean(), 'end max %.1f' % (t1[m].max() * 0.01))
print('first 600 waves (edge tiles) dur mean %.1f, rest %.1f' % (dur[:600].mean(), dur[600:].mean()))
np.save(os.environ.get('OUT', 'gpurun_out/ps_stamps.npy'), a)
